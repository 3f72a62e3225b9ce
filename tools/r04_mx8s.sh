#!/bin/bash
# MXFP8-output persistent GEMM (H/4 bf16 fc1): new bit-exact test + the fp8 suite, then the H/4 forward A/B.
OUT=${GRAFT_REPO_ROOT:-.}/gpurun_out/${1:-r04k}
mkdir -p $OUT
stop_on_fault() { case $1 in 0|1) return 0;; *) echo "step exited $1: stopping"; exit $1;; esac; }
timeout -k 10 600 python3 -u -m pytest -q -x -rf --timeout 120 --timeout-method thread tests/test_gpu_fp8.py -m gpu > $OUT/pytest.log 2>&1
s=$?; tail -8 $OUT/pytest.log; [ $s -eq 0 ] || exit $s
timeout -k 10 300 python3 tools/sol_forward.py imagenet512_uvit_huge 100 5 fp8 > $OUT/sol_h4.log 2>&1
s=$?; cat $OUT/sol_h4.log; stop_on_fault $s
echo done
