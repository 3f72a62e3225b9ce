set -e
OUT=$GRAFT_REPO_ROOT/gpurun_out/$1
mkdir -p $OUT
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_train.py -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
timeout -k 10 300 python3 tools/train_bench.py --batch 64 > $OUT/bench64.log 2>&1
tail -1 $OUT/bench64.log
timeout -k 10 300 python3 tools/train_bench.py --batch 128 > $OUT/bench128.log 2>&1
tail -1 $OUT/bench128.log
timeout -k 10 300 python3 tools/train_bench.py --batch 128 --lanes 1 > $OUT/bench128_l1.log 2>&1
tail -1 $OUT/bench128_l1.log
timeout -k 10 300 python3 tools/train_bench.py --batch 127 > $OUT/bench127.log 2>&1
tail -1 $OUT/bench127.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/kt -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/train_bench.py --batch 64 --steps 2 --warmup 1 > $OUT/kt.log 2>&1
echo prof done
