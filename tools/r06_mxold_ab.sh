#!/bin/bash
# H/4 bench: the tree vs the tree with gemm_mx_kernel's refills back behind the lgkmcnt wait (ab/libpdm_mxold.so)
set -o pipefail
O=gpurun_out/r06mx; mkdir -p $O
for r in 1 2 3; do
  for lib in panopticdiffusionmodels_amd/libpdm.so ab/libpdm_mxold.so; do
    PDM_LIB_PATH=$lib timeout -k 10 200 python3 bench.py --config imagenet512_uvit_huge --steps 3 --warmup 1 --cpu-baseline off > $O/h4_$(basename $lib .so)_$r.txt 2>&1 || exit 1
  done
done
