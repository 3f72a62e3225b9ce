#!/bin/bash
# attention A/B: attention parity tests, then attn_bench at the L/2, t2i and H shapes for ab/libpdm_head.so vs the
# tree (interleaved per shape).  Usage: TAG [bench]
set -e
OUT=gpurun_out/${1:-attab}
mkdir -p $OUT
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_kernels.py -k attention > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
for S in "50 258 16 64 0" "100 258 16 64 0" "32 334 8 64 0" "32 590 8 64 0" "50 258 16 72 0"; do
  for L in ${LIBS:-ab/libpdm_head.so panopticdiffusionmodels_amd/libpdm.so ab/libpdm_head.so panopticdiffusionmodels_amd/libpdm.so}; do
    PDM_LIB_PATH=$L timeout -k 10 120 python3 tools/attn_bench.py $S 2>&1 | grep -v amdgpu.ids | sed "s|^|$L |" | sed 's/maxrelerr=[^|]*| sdpa *[0-9.]* us *[0-9.]* TF\/s | //'
  done
done | tee $OUT/attn.log
if [ "$2" = bench ]; then
  for i in 1 2; do
    PDM_LIB_PATH=ab/libpdm_head.so timeout -k 10 300 python3 bench.py --cpu-baseline off > $OUT/bench_head_$i.log 2>&1
    timeout -k 10 300 python3 bench.py --cpu-baseline off > $OUT/bench_new_$i.log 2>&1
  done
  for f in $OUT/bench_*.log; do echo "$f $(grep -o '"value": [0-9.]*' $f | head -1)"; done
fi
