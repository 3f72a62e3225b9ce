#!/bin/bash
# experiment: half the persistent bf16-output workgroups (blockIdx & 8: half of every XCD) start 6.4k / 12.8k cycles
# late (ab/libpdm_ds1 / ds2) so the epilogue store bursts of the two halves alternate
set -o pipefail
O=gpurun_out/r06ds; mkdir -p $O
for r in 1 2; do
  for lib in panopticdiffusionmodels_amd/libpdm.so ab/libpdm_ds1.so ab/libpdm_ds2.so; do
    echo "== $lib" >> $O/shapes.txt
    PDM_LIB_PATH=$lib timeout -k 10 120 python tools/g8s_diag.py 50 2>&1 | grep "qkv" >> $O/shapes.txt || exit 1
  done
done
for lib in panopticdiffusionmodels_amd/libpdm.so ab/libpdm_ds1.so ab/libpdm_ds2.so; do
  PDM_LIB_PATH=$lib timeout -k 10 200 python3 bench.py --steps 3 --warmup 1 --cpu-baseline off > $O/l2_$(basename $lib .so).txt 2>&1 || exit 1
done
