#!/bin/bash
# GEMM epilogue change check: kernel + fp8 + forward GPU tests, then the epilogue cost table.  Usage: TAG
set -e
OUT=gpurun_out/${1:-qg}
mkdir -p $OUT
timeout -k 10 500 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
  tests/test_gpu_kernels.py tests/test_gpu_fp8.py tests/test_gpu_uvit.py > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -3 $OUT/pytest.log
timeout -k 10 200 python3 tools/epi_cost.py 50 > $OUT/epi_50.log 2>&1
timeout -k 10 200 python3 tools/epi_cost.py 100 > $OUT/epi_100.log 2>&1
cat $OUT/epi_50.log $OUT/epi_100.log
