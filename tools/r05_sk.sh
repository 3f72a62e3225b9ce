#!/bin/bash
# Round 5, first stream-K checks: new / changed tests, then the per-GEMM and forward A/B.  Each GPU step has its own
# limit; a fault or a time limit ends the script.
OUT=${GRAFT_REPO_ROOT:-.}/gpurun_out/${1:-r05a}
mkdir -p $OUT
stop_on_fault() { case $1 in 0|1) return 0;; *) echo "step exited $1: stopping"; exit $1;; esac; }
timeout -k 10 500 python3 -u -m pytest -x -v -rf --timeout 200 --timeout-method thread \
  tests/test_gpu_streamk.py "tests/test_gpu_kernels.py::test_gemm_pair_grouped_vs_separate" \
  tests/test_gpu_configs.py::test_full_t2i_forward_grouped_rows_vs_oracle -m gpu > $OUT/pytest.log 2>&1
s=$?; tail -25 $OUT/pytest.log; stop_on_fault $s
[ $s -ne 0 ] && exit 1
timeout -k 10 300 python3 tools/sk_bench.py imagenet256_uvit_large 100 > $OUT/sk_l2_100.log 2>&1
s=$?; cat $OUT/sk_l2_100.log; stop_on_fault $s
timeout -k 10 300 python3 tools/sk_bench.py imagenet256_uvit_huge 100 > $OUT/sk_h2_100.log 2>&1
s=$?; cat $OUT/sk_h2_100.log; stop_on_fault $s
timeout -k 10 300 python3 tools/sk_bench.py imagenet256_uvit_large 50 > $OUT/sk_l2_50.log 2>&1
s=$?; cat $OUT/sk_l2_50.log; stop_on_fault $s
echo done
