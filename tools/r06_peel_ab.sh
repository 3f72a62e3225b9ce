#!/bin/bash
set -o pipefail
O=gpurun_out/r06p; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 250 --timeout-method thread tests/test_gpu_kernels.py tests/test_gpu_streamk.py tests/test_gpu_fp8.py -k "gemm or mx or streamk or fp8" > $O/pytest.txt 2>&1 || exit 1
for lib in ab/libpdm_dual.so panopticdiffusionmodels_amd/libpdm.so ab/libpdm_dual.so panopticdiffusionmodels_amd/libpdm.so; do
  echo "== $lib rows 50" >> $O/shapes.txt
  PDM_LIB_PATH=$lib timeout -k 10 120 python tools/g8s_diag.py 50 2>&1 | grep -v amdgpu.ids >> $O/shapes.txt || exit 1
done
for r in 1 2; do
  for lib in ab/libpdm_dual.so panopticdiffusionmodels_amd/libpdm.so; do
    PDM_LIB_PATH=$lib timeout -k 10 300 python3 bench.py --steps 4 --warmup 1 --cpu-baseline off > $O/ab_$(basename $lib .so)_$r.txt 2>&1 || exit 1
  done
done
