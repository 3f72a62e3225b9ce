#!/bin/bash
set -o pipefail
O=gpurun_out/r06n; mkdir -p $O
for r in 1 2 3; do
  for lib in panopticdiffusionmodels_amd/libpdm.so ab/libpdm_nodual.so; do
    echo "== $lib rows 50" >> $O/ab.txt
    PDM_LIB_PATH=$lib timeout -k 10 120 python tools/g8s_diag.py 50 2>&1 | grep -v amdgpu.ids >> $O/ab.txt || exit 1
  done
done
