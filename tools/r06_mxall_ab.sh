#!/bin/bash
# persistent MXFP8 GEMM on every MXFP8 shape from 4096 rows (ab/libpdm_mxall.so) vs the tree: fp8 tests on the
# variant, per-shape qkv timings, then the H/4 bench alternating
set -o pipefail
O=gpurun_out/r06ma; mkdir -p $O
PDM_LIB_PATH=ab/libpdm_mxall.so timeout -k 10 400 python -u -m pytest -x -q --timeout 250 --timeout-method thread \
  tests/test_gpu_fp8.py tests/test_gpu_benchbatch.py tests/test_fullsize_golden.py -m gpu > $O/pytest.txt 2>&1 || exit 1
timeout -k 10 200 python3 tools/mx_qkv_bench.py 25,50,100 2>&1 | grep -v amdgpu.ids > $O/mx_qkv.txt || exit 1
for r in 1 2 3; do
  for lib in panopticdiffusionmodels_amd/libpdm.so ab/libpdm_mxall.so; do
    PDM_LIB_PATH=$lib timeout -k 10 200 python3 bench.py --config imagenet512_uvit_huge --steps 3 --warmup 1 --cpu-baseline off > $O/h4_$(basename $lib .so)_$r.txt 2>&1 || exit 1
  done
done
