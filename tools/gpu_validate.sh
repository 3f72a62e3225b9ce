#!/bin/bash
# One GPU validation pass from the repo root on the GPU box: -m gpu suite, smoke(), a short bench.
# Each GPU step has its own time limit; a fault / abort / timeout ends the script (test failures do not).
OUT=${GRAFT_REPO_ROOT:-.}/gpurun_out/${1:-val}
mkdir -p $OUT
stop_on_fault() {  # $1 = exit status; 0/1 (pytest failures) continue, anything else stops
  case $1 in 0|1) return 0;; *) echo "step exited $1: stopping"; exit $1;; esac
}
timeout -k 10 ${PYTEST_LIMIT:-900} python3 -m pytest tests -m gpu -q -rf --durations=15 ${PYTEST_ARGS} > $OUT/pytest.log 2>&1
s=$?; tail -30 $OUT/pytest.log; stop_on_fault $s
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1
s=$?; cat $OUT/smoke.log | tail -5; stop_on_fault $s
if [ -z "$NO_BENCH" ]; then
timeout -k 10 400 python3 bench.py ${BENCH_ARGS} > $OUT/bench.log 2>&1
s=$?; tail -3 $OUT/bench.log; stop_on_fault $s
fi
echo done
