#!/bin/bash
OUT=${GRAFT_REPO_ROOT:-.}/gpurun_out/${1:-r04x}
mkdir -p $OUT
timeout -k 10 900 python3 -u -m pytest -q -rf --timeout 300 --timeout-method thread tests -m gpu > $OUT/pytest.log 2>&1
s=$?; tail -4 $OUT/pytest.log; exit $s
