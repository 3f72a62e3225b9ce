#!/bin/bash
# Same-box A/B of library builds (dev tool): GEMM parity tests on every variant, then per-shape GEMM times at rows 50
# and the default bench, alternating the libraries.  tools/ab_libs.sh OUTDIR LIB [LIB ...]
set -o pipefail
O=gpurun_out/$1; shift; mkdir -p $O
for lib in "$@"; do
  PDM_LIB_PATH=$lib timeout -k 10 400 python -u -m pytest -x -q --timeout 250 --timeout-method thread \
    tests/test_gpu_kernels.py tests/test_gpu_streamk.py tests/test_gpu_fp8.py -k "gemm or mx or streamk or fp8" \
    > $O/pytest_$(basename $lib .so).txt 2>&1 || exit 1
done
for r in 1 2; do
  for lib in "$@"; do
    echo "== $lib rows 50" >> $O/shapes.txt
    PDM_LIB_PATH=$lib timeout -k 10 120 python tools/g8s_diag.py 50 2>&1 | grep -v amdgpu.ids >> $O/shapes.txt || exit 1
  done
done
for r in 1 2; do
  for lib in "$@"; do
    PDM_LIB_PATH=$lib timeout -k 10 300 python3 bench.py --steps 4 --warmup 1 --cpu-baseline off \
      > $O/ab_$(basename $lib .so)_$r.txt 2>&1 || exit 1
  done
done
