#!/bin/bash
# t2i injection second output: kernel + t2i parity tests, the injection shapes, the t2i bench (A/B vs the previous
# library kept in ab/) -- one GPU step at a time, each under its own limit
OUT=${GRAFT_REPO_ROOT:-.}/gpurun_out/${1:-r05g}
mkdir -p $OUT
timeout -k 10 300 python3 -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu \
  tests/test_gpu_kernels.py -k "gather_second_output or pair_grouped" tests/test_gpu_t2i.py tests/test_gpu_configs.py \
  > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -3 $OUT/pytest.log
timeout -k 10 200 python3 tools/inject_bench.py 0,1,7 > $OUT/inject.log 2>&1 || exit 1
cat $OUT/inject.log
timeout -k 10 400 python3 bench.py --config mscoco_uvit_small --steps 3 --warmup 1 --cpu-baseline off > $OUT/bench_t2i.log 2>&1 || exit 1
tail -1 $OUT/bench_t2i.log
echo done
