#!/bin/bash
# training-step change check: the out-of-place residual kernel tests + training GPU tests, then the L/2 training
# bench at B = 128 for ab/libpdm_head.so (built by tools/ab_build.sh) vs the tree, interleaved.  Usage: TAG
set -e
OUT=gpurun_out/${1:-trab}
mkdir -p $OUT
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_kernels.py -k "residual_f32 or gemm_algos" > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
timeout -k 10 500 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_train.py > $OUT/pytest_train.log 2>&1 || { tail -40 $OUT/pytest_train.log; exit 1; }
tail -2 $OUT/pytest_train.log
for i in 1 2; do
  PDM_LIB_PATH=ab/libpdm_head.so timeout -k 10 300 python3 tools/train_bench.py --batch 128 > $OUT/head_$i.log 2>&1
  timeout -k 10 300 python3 tools/train_bench.py --batch 128 > $OUT/new_$i.log 2>&1
done
for f in $OUT/head_*.log $OUT/new_*.log; do echo "$f $(tail -1 $f | grep -o '"value": [0-9.]*')"; done
