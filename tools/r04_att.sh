#!/bin/bash
# Attention ragged split: kernel tests, then A/B (4 = split, 11 = no split) on the bench shapes.
OUT=${GRAFT_REPO_ROOT:-.}/gpurun_out/${1:-r04i}
mkdir -p $OUT
stop_on_fault() { case $1 in 0|1) return 0;; *) echo "step exited $1: stopping"; exit $1;; esac; }
timeout -k 10 600 python3 -u -m pytest -x -q -rf --timeout 300 --timeout-method thread tests/test_gpu_kernels.py \
  -m gpu -k "attention" > $OUT/pytest.log 2>&1
s=$?; tail -4 $OUT/pytest.log; stop_on_fault $s
[ $s -ne 0 ] && exit 1
for r in 100 190; do
  timeout -k 10 200 python3 tools/attn_bench.py $r 258 16 64 4,11 > $OUT/attn_r$r.log 2>&1
  s=$?; cat $OUT/attn_r$r.log; stop_on_fault $s
done
timeout -k 10 200 python3 tools/attn_bench.py 8 257 8 64 4,11 > $OUT/attn_cifar.log 2>&1
s=$?; cat $OUT/attn_cifar.log; stop_on_fault $s
echo done
