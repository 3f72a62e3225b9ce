#!/bin/bash
# rocprofv3 evidence for one bench line (run on the GPU box from the repo root):
#   1. kernel trace + stats of the bench command itself (graph-captured sampling + decode)
#   2. separate PMC passes (FETCH_SIZE, WRITE_SIZE) over one eager CFG forward at the bench batch, for the
#      HBM traffic of every kernel (MI355X_MICROARCH.md §HBM: FETCH_SIZE x 2 for 16-B streaming reads)
# Usage: tools/profile_bench.sh TAG [CONFIG [BATCH [PRECISION]]]   (then: python tools/summarize_prof.py TAG ...)
set -e
TAG=${1:-r03}
CONFIG=${2:-imagenet256_uvit_large}
BATCH=${3:-50}
PREC=${4:-}
ROWS=$((2 * BATCH))
OUT=${GRAFT_REPO_ROOT:-.}/gpurun_out/prof_${TAG}_${CONFIG}
mkdir -p $OUT
export TMPDIR=/tmp
PARGS=""
[ -n "$PREC" ] && PARGS="--precision $PREC"
timeout -k 10 500 rocprofv3 --kernel-trace --stats -d $OUT/kt -o run --output-format csv -- python3 bench.py --config $CONFIG --batch $BATCH --steps 2 --warmup 1 --cpu-baseline off $PARGS > $OUT/bench_kt.log 2>&1
echo "kernel trace done"; tail -1 $OUT/bench_kt.log | cut -c1-200
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d $OUT/fetch -o run --output-format csv -- python3 tools/time_forward.py $CONFIG $ROWS 2 ${PREC:-bf16} > $OUT/fetch.log 2>&1
echo "fetch pass done"
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d $OUT/write -o run --output-format csv -- python3 tools/time_forward.py $CONFIG $ROWS 2 ${PREC:-bf16} > $OUT/write.log 2>&1
echo "write pass done"
# summarise on the box (raw traces can exceed gpurun's 64 MiB copy-back), keep the summaries + logs only
SUM=${GRAFT_REPO_ROOT:-.}/gpurun_out/prof_summaries
mkdir -p $SUM
PDM_PROF_DST=$SUM python3 tools/summarize_prof.py $TAG $CONFIG $BATCH ${PREC:-bf16} > /dev/null
cp $OUT/bench_kt.log $SUM/${TAG}_${CONFIG}_bench_kt.log
rm -rf $OUT
echo "summarised into $SUM"
