#!/bin/bash
# Sampling-configuration speed of light: lanes 2 / 1 at B = 50, algo 11 / 7, no-epilogue timing mode.
OUT=${GRAFT_REPO_ROOT:-.}/gpurun_out/${1:-r04e}
mkdir -p $OUT
stop_on_fault() { case $1 in 0|1) return 0;; *) echo "step exited $1: stopping"; exit $1;; esac; }
timeout -k 10 400 python3 tools/sol_lanes.py imagenet256_uvit_large 50 2 2 > $OUT/sol_lanes2.log 2>&1
s=$?; cat $OUT/sol_lanes2.log; stop_on_fault $s
timeout -k 10 400 python3 tools/sol_lanes.py imagenet256_uvit_large 50 1 2 > $OUT/sol_lanes1.log 2>&1
s=$?; cat $OUT/sol_lanes1.log; stop_on_fault $s
echo done
