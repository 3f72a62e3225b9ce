#!/bin/bash
# PMC passes on one GEMM shape (run on the GPU box).  Usage: tools/pmc_gemm.sh ALGO M N K EPI TAG
set -e
A=$1; M=$2; N=$3; K=$4; E=$5; TAG=$6
OUT=$GRAFT_REPO_ROOT/gpurun_out/pmc_$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $OUT/kt -o run --output-format csv -- python3 tools/gemm_one.py $A $M $N $K $E 20 > /dev/null 2>&1
timeout -k 10 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_WAIT_INST_LDS -d $OUT/p1 -o run --output-format csv -- python3 tools/gemm_one.py $A $M $N $K $E 5 > /dev/null 2>&1
timeout -k 10 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE GRBM_COUNT -d $OUT/p2 -o run --output-format csv -- python3 tools/gemm_one.py $A $M $N $K $E 5 > /dev/null 2>&1
timeout -k 10 120 rocprofv3 --pmc FETCH_SIZE -d $OUT/p3 -o run --output-format csv -- python3 tools/gemm_one.py $A $M $N $K $E 5 > /dev/null 2>&1
timeout -k 10 120 rocprofv3 --pmc WRITE_SIZE -d $OUT/p4 -o run --output-format csv -- python3 tools/gemm_one.py $A $M $N $K $E 5 > /dev/null 2>&1
echo pmc_done $TAG
