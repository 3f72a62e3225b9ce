#!/bin/bash
# residual rows requested before the epilogue's rejoin barrier (ab/libpdm_early.so) vs the HEAD library
# (ab/libpdm_base.so): GEMM tests on the variant, residual GEMM shapes, epilogue stamps, default bench
set -o pipefail
O=gpurun_out/r06er; mkdir -p $O
PDM_LIB_PATH=ab/libpdm_early.so timeout -k 10 400 python -u -m pytest -x -q --timeout 250 --timeout-method thread \
  tests/test_gpu_kernels.py tests/test_gpu_streamk.py tests/test_gpu_fp8.py tests/test_gpu_t2i.py -k "gemm or mx or streamk or fp8 or t2i" > $O/pytest.txt 2>&1 || exit 1
for r in 1 2; do
  for lib in ab/libpdm_base.so ab/libpdm_early.so; do
    echo "== $lib rows 50" >> $O/shapes.txt
    PDM_LIB_PATH=$lib timeout -k 10 120 python tools/g8s_diag.py 50 2>&1 | grep -v amdgpu.ids >> $O/shapes.txt || exit 1
  done
done
for r in 1 2; do
  for lib in ab/libpdm_base.so ab/libpdm_early.so; do
    PDM_LIB_PATH=$lib timeout -k 10 200 python3 bench.py --steps 3 --warmup 1 --cpu-baseline off > $O/l2_$(basename $lib .so)_$r.txt 2>&1 || exit 1
  done
done
