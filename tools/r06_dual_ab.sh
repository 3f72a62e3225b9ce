#!/bin/bash
# Round 6: single-operand refill path (DUAL = 0) -- GEMM / forward / t2i / fp8 tests, then the default bench A/B
# against the round-5 library and per-shape timings
set -o pipefail
O=gpurun_out/r06o; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 250 --timeout-method thread tests/test_gpu_kernels.py tests/test_gpu_streamk.py tests/test_gpu_fp8.py tests/test_gpu_t2i.py tests/test_gpu_configs.py > $O/pytest.txt 2>&1 || exit 1
timeout -k 10 300 python -u -m pytest -x -q --timeout 250 --timeout-method thread tests/test_gpu_benchbatch.py > $O/pytest_bb.txt 2>&1 || exit 1
for r in 1 2; do
  for lib in ab/libpdm_head.so panopticdiffusionmodels_amd/libpdm.so; do
    PDM_LIB_PATH=$lib timeout -k 10 300 python3 bench.py --steps 4 --warmup 1 --cpu-baseline off > $O/ab_$(basename $lib .so)_$r.txt 2>&1 || exit 1
  done
done
for lib in ab/libpdm_head.so panopticdiffusionmodels_amd/libpdm.so; do
  echo "== $lib rows 50" >> $O/shapes.txt
  PDM_LIB_PATH=$lib timeout -k 10 120 python tools/g8s_diag.py 50 2>&1 | grep -v amdgpu.ids >> $O/shapes.txt || exit 1
done
