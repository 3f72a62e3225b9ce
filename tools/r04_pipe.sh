#!/bin/bash
# Pipelined attention (algo 11): kernel tests, then A/B vs v2 (algo 4) on the bench shapes.
OUT=${GRAFT_REPO_ROOT:-.}/gpurun_out/${1:-r04l}
mkdir -p $OUT
stop_on_fault() { case $1 in 0|1) return 0;; *) echo "step exited $1: stopping"; exit $1;; esac; }
timeout -k 10 600 python3 -u -m pytest -x -q -rf --timeout 120 --timeout-method thread tests/test_gpu_kernels.py \
  -m gpu -k "attention" > $OUT/pytest.log 2>&1
s=$?; tail -4 $OUT/pytest.log; [ $s -ne 0 ] && exit $s
for r in 50 100 190; do
  timeout -k 10 200 python3 tools/attn_bench.py $r 258 16 64 4,11 > $OUT/attn_r$r.log 2>&1 && timeout -k 10 200 python3 tools/attn_bench.py $r 256 16 64 4,11 >> $OUT/attn_r$r.log 2>&1
  s=$?; cat $OUT/attn_r$r.log; stop_on_fault $s
done
timeout -k 10 200 python3 tools/attn_bench.py 128 590 8 64 4,11 > $OUT/attn_t2i590.log 2>&1
s=$?; cat $OUT/attn_t2i590.log; stop_on_fault $s
timeout -k 10 200 python3 tools/attn_bench.py 128 334 8 64 4,11 > $OUT/attn_t2i334.log 2>&1
s=$?; cat $OUT/attn_t2i334.log; stop_on_fault $s
echo done
