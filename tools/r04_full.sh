#!/bin/bash
# Full GPU validation of HEAD + the default bench (and a lanes-1 A/B); every GPU step time-limited, faults stop it.
OUT=${GRAFT_REPO_ROOT:-.}/gpurun_out/${1:-r04d}
mkdir -p $OUT
stop_on_fault() { case $1 in 0|1) return 0;; *) echo "step exited $1: stopping"; exit $1;; esac; }
timeout -k 10 1000 python3 -u -m pytest -q -rf --timeout 300 --timeout-method thread tests -m gpu > $OUT/pytest.log 2>&1
s=$?; tail -6 $OUT/pytest.log; stop_on_fault $s
timeout -k 10 300 python3 bench.py --steps 5 --warmup 2 --cpu-baseline off > $OUT/bench.log 2>&1
s=$?; tail -1 $OUT/bench.log | cut -c1-400; stop_on_fault $s
timeout -k 10 300 python3 bench.py --steps 3 --warmup 1 --lanes 1 --cpu-baseline off > $OUT/bench_l1.log 2>&1
s=$?; tail -1 $OUT/bench_l1.log | cut -c1-300; stop_on_fault $s
echo done
