#!/bin/bash
# rocprofv3 evidence for the bench line (run on the GPU box from the repo root):
#   1. kernel trace + stats of the bench command itself (graph-captured sampling + decode)
#   2. separate PMC passes (FETCH_SIZE, WRITE_SIZE) over one eager CFG forward at the bench batch, for the
#      HBM traffic of every kernel (MI355X_MICROARCH.md §HBM: FETCH_SIZE x 2 for 16-B streaming reads)
# Usage: tools/profile_bench.sh TAG [extra bench args...]
set -e
TAG=${1:-r01}; shift || true
OUT=${GRAFT_REPO_ROOT:-.}/gpurun_out/prof_$TAG
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp && cd - > /dev/null
timeout -k 10 500 rocprofv3 --kernel-trace --stats -d $OUT/kt -o run --output-format csv -- python3 bench.py --steps 2 --warmup 1 --cpu-baseline off "$@" > $OUT/bench_kt.log 2>&1
echo "kernel trace done"
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d $OUT/fetch -o run --output-format csv -- python3 tools/time_forward.py imagenet256_uvit_large 190 2 > $OUT/fetch.log 2>&1
echo "fetch pass done"
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d $OUT/write -o run --output-format csv -- python3 tools/time_forward.py imagenet256_uvit_large 190 2 > $OUT/write.log 2>&1
echo "write pass done"
