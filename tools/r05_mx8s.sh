#!/bin/bash
# MXFP8 persistent GEMM check: fp8 GEMM / forward tests (timeout-guarded, stop at the first failure), then the H/4 qkv
# shape per build under rocprof, then the H/4 bench for ab/libpdm_head.so vs the tree.  Usage: TAG
OUT=gpurun_out/${1:-mx8s}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_fp8.py > $OUT/pytest.log 2>&1
s=$?; tail -3 $OUT/pytest.log; [ $s -eq 0 ] || exit $s
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $OUT/kt -o run --output-format csv -- python3 -u -m pytest -x -q -m gpu tests/test_gpu_fp8.py -k "persistent_vs_tile and 12900" > /dev/null 2>&1 || exit 1
grep -h "gemm" $OUT/kt/run_kernel_stats.csv | cut -c1-140
for i in 1 2; do
  PDM_LIB_PATH=ab/libpdm_head.so timeout -k 10 400 python3 bench.py --config imagenet512_uvit_huge --cpu-baseline off > $OUT/h4_head_$i.log 2>&1 || exit 1
  timeout -k 10 400 python3 bench.py --config imagenet512_uvit_huge --cpu-baseline off > $OUT/h4_new_$i.log 2>&1 || exit 1
done
for f in $OUT/h4_*.log; do echo "$f $(grep -o '"value": [0-9.]*' $f | head -1) $(grep -o '"sample_50nfe": [0-9.]*' $f)"; done
