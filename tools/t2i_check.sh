#!/bin/bash
# t2i forward change check: t2i / config / full-size parity GPU tests, then the t2i bench at HEAD~ (ab/) vs the tree
set -e
OUT=gpurun_out/${1:-t2i}
mkdir -p $OUT
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_t2i.py tests/test_gpu_configs.py tests/test_fullsize_golden.py > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
for i in 1 2; do
  PDM_LIB_PATH=ab/libpdm_head.so timeout -k 10 300 python3 bench.py --config mscoco_uvit_small --cpu-baseline off > $OUT/bench_head_$i.log 2>&1
  timeout -k 10 300 python3 bench.py --config mscoco_uvit_small --cpu-baseline off > $OUT/bench_new_$i.log 2>&1
done
for f in $OUT/bench_*.log; do echo "$f $(grep -o '"value": [0-9.]*' $f | head -1)"; done
