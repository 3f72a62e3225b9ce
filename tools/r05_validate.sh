#!/bin/bash
# Round-5 validation of the tree on one MI355X: GPU suite, smoke, the default bench line and every other config's
# line, each with its CPU baseline, then the rocprof evidence (kernel trace + FETCH / WRITE) of
# the default bench.  Usage: TAG [skip_tests]
TAG=${1:-r05v}
OUT=${GRAFT_REPO_ROOT:-.}/gpurun_out/$TAG
mkdir -p $OUT
stop_on_fault() { case $1 in 0|1) return 0;; *) echo "step exited $1: stopping"; exit $1;; esac; }
if [ -z "$2" ]; then
  timeout -k 10 1100 python3 -u -m pytest -q -rf --timeout 300 --timeout-method thread tests -m gpu > $OUT/pytest.log 2>&1
  s=$?; tail -4 $OUT/pytest.log; stop_on_fault $s
  timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1
  s=$?; tail -3 $OUT/smoke.log; stop_on_fault $s
fi
timeout -k 10 400 python3 bench.py --steps 5 --warmup 2 > $OUT/bench.log 2>&1
s=$?; tail -1 $OUT/bench.log | cut -c1-300; stop_on_fault $s
for c in imagenet256_uvit_huge imagenet512_uvit_huge mscoco_uvit_small cifar10_uvit_small; do
  timeout -k 10 600 python3 bench.py --config $c --steps 3 --warmup 1 > $OUT/bench_$c.log 2>&1
  s=$?; tail -1 $OUT/bench_$c.log | cut -c1-260; stop_on_fault $s
done
echo done
