#!/bin/bash
# attention change check: attention / forward / full-size parity GPU tests, then attn_bench at the L/2 (Dh 64) and
# H/2 (Dh 72) shapes for ab/libpdm_head.so vs the tree, and the default bench for both.  Usage: TAG
set -e
OUT=gpurun_out/${1:-attab}
mkdir -p $OUT
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_kernels.py -k attention tests/test_gpu_uvit.py tests/test_fullsize_golden.py > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
for L in ab/libpdm_head.so panopticdiffusionmodels_amd/libpdm.so; do
  for S in "50 258 16 64 4" "190 258 16 64 4" "50 258 16 72 0"; do
    PDM_LIB_PATH=$L timeout -k 10 120 python3 tools/attn_bench.py $S 2>&1 | grep -v amdgpu.ids | sed "s|^|$L |"
  done
done
for i in 1 2; do
  PDM_LIB_PATH=ab/libpdm_head.so timeout -k 10 300 python3 bench.py --cpu-baseline off > $OUT/bench_head_$i.log 2>&1
  timeout -k 10 300 python3 bench.py --cpu-baseline off > $OUT/bench_new_$i.log 2>&1
done
for f in $OUT/bench_*.log; do echo "$f $(grep -o '"value": [0-9.]*' $f | head -1)"; done
