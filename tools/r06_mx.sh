#!/bin/bash
# Round 6: persistent MXFP8 residual GEMM (H/4 proj) -- fp8 tests, the per-GEMM A/B, and the H/4 bench line A/B
set -o pipefail
O=gpurun_out/r06j; mkdir -p $O
timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_fp8.py > $O/pytest_fp8.txt 2>&1 || exit 1
timeout -k 10 200 python tools/mx_res_bench.py 50,100 > $O/mx_res_bench.txt 2>&1 || exit 1
for r in 1 2; do
  for lib in ab/libpdm_mxres0.so panopticdiffusionmodels_amd/libpdm.so; do
    PDM_LIB_PATH=$lib timeout -k 10 300 python bench.py --config imagenet512_uvit_huge --steps 3 --warmup 1 --cpu-baseline off > $O/bench_h4_$(basename $lib .so)_$r.json 2>$O/bench_h4_err.txt || exit 1
  done
done
