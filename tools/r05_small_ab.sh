#!/bin/bash
# small-kernel change check: sampler / forward / t2i / config GPU tests, then the default bench and the t2i bench for
# ab/libpdm_head.so vs the tree (alternating).  Usage: TAG
set -e
OUT=gpurun_out/${1:-smallab}
mkdir -p $OUT
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_sample.py tests/test_gpu_uvit.py tests/test_gpu_t2i.py tests/test_gpu_configs.py > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
for i in 1 2; do
  PDM_LIB_PATH=ab/libpdm_head.so timeout -k 10 300 python3 bench.py --cpu-baseline off > $OUT/bench_head_$i.log 2>&1
  timeout -k 10 300 python3 bench.py --cpu-baseline off > $OUT/bench_new_$i.log 2>&1
done
for i in 1; do
  PDM_LIB_PATH=ab/libpdm_head.so timeout -k 10 300 python3 bench.py --config mscoco_uvit_small --cpu-baseline off > $OUT/t2i_head_$i.log 2>&1
  timeout -k 10 300 python3 bench.py --config mscoco_uvit_small --cpu-baseline off > $OUT/t2i_new_$i.log 2>&1
done
for f in $OUT/bench_*.log $OUT/t2i_*.log; do echo "$f $(grep -o '"value": [0-9.]*' $f | head -1) $(grep -o '"sample_50nfe": [0-9.]*' $f)"; done
