#!/bin/bash
# Round 6: what bounds gemm8s's main loop -- forward epilogue / no epilogue on the production build and on the
# -DPDM_G8S_DIAG builds (1 no DMA refills, 2 no fragment reads, 3 neither, 4 no MFMAs, 5 no DMA + no MFMA)
set -o pipefail
O=gpurun_out/r06c; mkdir -p $O
for rows in 100 50; do
  for lib in panopticdiffusionmodels_amd/libpdm.so ab/libpdm_diag1.so ab/libpdm_diag2.so ab/libpdm_diag3.so ab/libpdm_diag4.so ab/libpdm_diag5.so; do
    echo "== $lib rows $rows" >> $O/g8s_diag.txt
    PDM_LIB_PATH=$lib timeout -k 10 120 python tools/g8s_diag.py $rows 2>&1 | grep -v amdgpu.ids >> $O/g8s_diag.txt || exit 1
  done
done
