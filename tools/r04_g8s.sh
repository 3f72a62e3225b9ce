#!/bin/bash
# Persistent GEMM (algo 11) first GPU pass: kernel parity tests, then epilogue-cost and forward A/B vs algo 7.
OUT=${GRAFT_REPO_ROOT:-.}/gpurun_out/${1:-r04c}
mkdir -p $OUT
stop_on_fault() { case $1 in 0|1) return 0;; *) echo "step exited $1: stopping"; exit $1;; esac; }
timeout -k 10 600 python3 -u -m pytest -x -q -rf --timeout 300 --timeout-method thread tests/test_gpu_kernels.py \
  -m gpu -k "persistent or residual_bf16 or layernorm_consumer or gelu_activation or (gemm_algos and 11)" > $OUT/pytest.log 2>&1
s=$?; tail -15 $OUT/pytest.log; stop_on_fault $s
[ $s -ne 0 ] && exit 1
for a in 11 7; do
  timeout -k 10 300 python3 tools/epi_cost.py 100 1024 $a > $OUT/epi_cost_a$a.log 2>&1
  s=$?; cat $OUT/epi_cost_a$a.log; stop_on_fault $s
done
timeout -k 10 300 python3 tools/sol_forward.py imagenet256_uvit_large 100 5 > $OUT/sol_l2.log 2>&1
s=$?; cat $OUT/sol_l2.log; stop_on_fault $s
echo done
