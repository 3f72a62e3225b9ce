#!/bin/bash
# Round 6: interleaved-refill schedule (PDM_G8S_SCHED=1 build) vs production: GEMM tests on the variant, then
# alternating per-shape timings at the bench's rows
set -o pipefail
O=gpurun_out/r06e; mkdir -p $O
V=${1:-isched}
PDM_LIB_PATH=ab/libpdm_$V.so timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_kernels.py -k "gemm" > $O/pytest_$V.txt 2>&1 || exit 1
for r in 1 2; do
  for lib in panopticdiffusionmodels_amd/libpdm.so ab/libpdm_$V.so; do
    for rows in 100 50; do
      echo "== $lib rows $rows" >> $O/ab_$V.txt
      PDM_LIB_PATH=$lib timeout -k 10 120 python tools/g8s_diag.py $rows 2>&1 | grep -v amdgpu.ids >> $O/ab_$V.txt || exit 1
    done
  done
done
