#!/bin/bash
# Round 6: refill-order variants (PDM_G8S_SCHED=2/3 builds) vs the working tree: GEMM tests on each variant, then
# alternating per-shape timings at the bench's rows
set -o pipefail
O=gpurun_out/r06i; mkdir -p $O
for v in xs2 xs3; do
  PDM_LIB_PATH=ab/libpdm_$v.so timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_kernels.py -k "gemm_persistent or residual or layernorm_consumer" > $O/pytest_$v.txt 2>&1 || exit 1
done
for r in 1 2; do
  for lib in panopticdiffusionmodels_amd/libpdm.so ab/libpdm_xs2.so ab/libpdm_xs3.so; do
    for rows in 100 50; do
      echo "== $lib rows $rows" >> $O/ab.txt
      PDM_LIB_PATH=$lib timeout -k 10 120 python tools/g8s_diag.py $rows 2>&1 | grep -v amdgpu.ids >> $O/ab.txt || exit 1
    done
  done
done
