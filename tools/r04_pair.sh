#!/bin/bash
# Grouped t2i block GEMMs: kernel + t2i parity tests, then the t2i bench A/B (grouped vs algo-7 fallback is not
# comparable, so: this tree's line vs the validated r04v line) and the t2i forward.
OUT=${GRAFT_REPO_ROOT:-.}/gpurun_out/${1:-r04p}
mkdir -p $OUT
stop_on_fault() { case $1 in 0|1) return 0;; *) echo "step exited $1: stopping"; exit $1;; esac; }
timeout -k 10 900 python3 -u -m pytest -x -q -rf --timeout 300 --timeout-method thread tests/test_gpu_kernels.py tests/test_gpu_configs.py tests/test_fullsize_golden.py \
  -m gpu -k "gemm or mscoco or t2i" > $OUT/pytest.log 2>&1
s=$?; tail -4 $OUT/pytest.log; [ $s -ne 0 ] && exit $s
for r in 1 2; do
  timeout -k 10 300 python3 bench.py --config mscoco_uvit_small --steps 3 --warmup 1 --cpu-baseline off > $OUT/bench_t2i_$r.log 2>&1
  s=$?; tail -1 $OUT/bench_t2i_$r.log | cut -c1-200; stop_on_fault $s
done
for r in 1 2 3; do
  for lib in ab/libpdm_head.so panopticdiffusionmodels_amd/libpdm.so; do
    n=$(basename $lib .so)
    PDM_LIB_PATH=$lib timeout -k 10 200 python3 tools/time_forward.py mscoco_uvit_small 32 20 >> $OUT/t2i_fwd_$n.log 2>&1
    s=$?; stop_on_fault $s
    PDM_LIB_PATH=$lib timeout -k 10 200 python3 tools/time_forward.py imagenet256_uvit_large 100 10 >> $OUT/l2_fwd_$n.log 2>&1
    s=$?; stop_on_fault $s
  done
done
grep -h ms/forward $OUT/t2i_fwd_*.log $OUT/l2_fwd_*.log
echo done
