#!/bin/bash
# SQ counters of the persistent GEMM before (round-5 library, ab/libpdm_head.so) and after round 6 (the tree): qkv
# (LN consumer) and proj (residual) shapes at rows 50 (the bench's lanes), full epilogue
set -o pipefail
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/r06sq; mkdir -p $O
for tag in r5 r6; do
  if [ $tag = r6 ]; then export PDM_LIB_PATH=panopticdiffusionmodels_amd/libpdm.so; else export PDM_LIB_PATH=ab/libpdm_head.so; fi
  for shp in "qkv 12900 3072 1024 0" "proj 12900 1024 1024 3"; do
    set -- $shp
    timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $O/$tag/$1/kt -o run --output-format csv -- python3 tools/gemm_one.py 11 $2 $3 $4 $5 30 > /dev/null 2>&1 || exit 1
    timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_WAIT_INST_LDS -d $O/$tag/$1/p1 -o run --output-format csv -- python3 tools/gemm_one.py 11 $2 $3 $4 $5 10 > /dev/null 2>&1 || exit 1
    timeout -s KILL 90 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE GRBM_COUNT -d $O/$tag/$1/p2 -o run --output-format csv -- python3 tools/gemm_one.py 11 $2 $3 $4 $5 10 > /dev/null 2>&1 || exit 1
  done
done
echo done
