#!/bin/bash
# Round 6: attention Q-wait rewrite (PDM_WAIT_Q) A/B vs HEAD on the same box + the tests it touches.
set -o pipefail
O=gpurun_out/r06b; mkdir -p $O
T="timeout -k 10"
$T 600 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_gpu_kernels.py tests/test_gpu_streamk.py tests/test_gpu_train.py -k "attention or label or sk or stream" > $O/pytest.txt 2>&1 || exit 1
for r in 1 2; do
  for lib in ab/libpdm_head.so panopticdiffusionmodels_amd/libpdm.so; do
    tag=$(basename $lib .so)
    PDM_LIB_PATH=$lib $T 120 python tools/attn_bench.py 100 258 16 64 11 >> $O/attn_v3_$tag.txt 2>&1 || exit 1
    PDM_LIB_PATH=$lib $T 120 python tools/attn_bench.py 50 258 16 64 11 >> $O/attn_v3_$tag.txt 2>&1 || exit 1
    PDM_LIB_PATH=$lib $T 120 python tools/attn_bench.py 100 258 16 72 0 >> $O/attn_h72_$tag.txt 2>&1 || exit 1
  done
done
