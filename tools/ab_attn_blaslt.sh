set -e
OUT=$GRAFT_REPO_ROOT/gpurun_out/ab1
mkdir -p $OUT
timeout -k 10 120 python3 tools/attn_bench.py 190 258 16 64 4,11 > $OUT/attn190.log 2>&1; tail -4 $OUT/attn190.log
timeout -k 10 120 python3 tools/attn_bench.py 100 258 16 64 4,11 > $OUT/attn100.log 2>&1; tail -4 $OUT/attn100.log
timeout -k 10 120 python3 tools/attn_bench.py 128 590 8 64 4,11 > $OUT/attn590.log 2>&1; tail -4 $OUT/attn590.log
timeout -k 10 120 python3 tools/attn_bench.py 128 334 8 64 4,11 > $OUT/attn334.log 2>&1; tail -4 $OUT/attn334.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $OUT/bl -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/blaslt_probe.py 190 > $OUT/blaslt.log 2>&1
cat $OUT/blaslt.log | grep TF
