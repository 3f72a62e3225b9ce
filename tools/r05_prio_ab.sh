#!/bin/bash
# MFMA-phase priority A/B: head (s_setprio around every GEMM's MFMA phases) vs the tree (none in the persistent
# kernel) vs ab/libpdm_tile0.so (none in any GEMM).  Usage: TAG
OUT=gpurun_out/${1:-prio}
mkdir -p $OUT
bench() {   # name lib config
  PDM_LIB_PATH=$2 timeout -k 10 400 python3 bench.py --config $3 --cpu-baseline off > $OUT/$3_$1.log 2>&1 || exit 1
}
for i in 1 2; do
  bench head_$i ab/libpdm_head.so imagenet256_uvit_large
  bench tree_$i panopticdiffusionmodels_amd/libpdm.so imagenet256_uvit_large
done
bench head ab/libpdm_head.so imagenet512_uvit_huge
bench tree panopticdiffusionmodels_amd/libpdm.so imagenet512_uvit_huge
bench tile0 ab/libpdm_tile0.so imagenet512_uvit_huge
bench head ab/libpdm_head.so mscoco_uvit_small
bench tree panopticdiffusionmodels_amd/libpdm.so mscoco_uvit_small
for f in $OUT/*.log; do echo "$f $(grep -o '"value": [0-9.]*' $f | head -1) $(grep -o '"sample_50nfe": [0-9.]*, "decode": [0-9.]*' $f)"; done
