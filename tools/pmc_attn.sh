#!/bin/bash
# PMC passes on one attention structure (run on the GPU box).  Usage: tools/pmc_attn.sh ALGO TAG
set -e
A=$1; TAG=$2
OUT=$GRAFT_REPO_ROOT/gpurun_out/pmc_$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $OUT/kt -o run --output-format csv -- python3 tools/attn_one.py $A > /dev/null 2>&1
timeout -k 10 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_INSTS_VALU -d $OUT/p1 -o run --output-format csv -- python3 tools/attn_one.py $A 190 258 16 64 3 > /dev/null 2>&1
timeout -k 10 120 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE GRBM_COUNT -d $OUT/p2 -o run --output-format csv -- python3 tools/attn_one.py $A 190 258 16 64 3 > /dev/null 2>&1
echo pmc_done $TAG
