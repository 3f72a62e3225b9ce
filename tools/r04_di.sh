#!/bin/bash
# Persistent GEMM phase-B DMA placement A/B (algo 11 = read window, 12 = after the barrier, 13 = split around the
# quadrants): GEMM kernel tests at the new algos, then interleaved forwards at the bench rows.
OUT=${GRAFT_REPO_ROOT:-.}/gpurun_out/${1:-r04n}
mkdir -p $OUT
stop_on_fault() { case $1 in 0|1) return 0;; *) echo "step exited $1: stopping"; exit $1;; esac; }
timeout -k 10 600 python3 -u -m pytest -x -q -rf --timeout 120 --timeout-method thread tests/test_gpu_kernels.py \
  -m gpu -k "gemm" > $OUT/pytest.log 2>&1
s=$?; tail -4 $OUT/pytest.log; [ $s -ne 0 ] && exit $s
export SOL_MODES="a11:11:0,a12:12:0,a13:13:0"
for r in 100 50; do
  timeout -k 10 300 python3 tools/sol_forward.py imagenet256_uvit_large $r 7 > $OUT/sol_l2_r$r.log 2>&1
  s=$?; cat $OUT/sol_l2_r$r.log; stop_on_fault $s
done
timeout -k 10 300 python3 tools/sol_forward.py mscoco_uvit_small 48 5 > $OUT/sol_t2i.log 2>&1
s=$?; cat $OUT/sol_t2i.log; stop_on_fault $s
echo done
