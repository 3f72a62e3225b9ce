#!/bin/bash
# Round 6: SQ / GRBM counters of gemm8s's main loop (qkv shape at rows 100, no epilogue) on the production build and on
# the MFMA-only (diag3) / loads-only (diag4) builds: clock vs pipeline
set -o pipefail
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/r06d; mkdir -p $O
export PDM_DBG=16
for tag in prod diag3 diag4; do
  if [ $tag = prod ]; then export PDM_LIB_PATH=panopticdiffusionmodels_amd/libpdm.so; else export PDM_LIB_PATH=ab/libpdm_$tag.so; fi
  timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $O/$tag/kt -o run --output-format csv -- python3 tools/gemm_one.py 11 25800 3072 1024 0 30 > /dev/null 2>&1 || exit 1
  timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_WAIT_INST_LDS -d $O/$tag/p1 -o run --output-format csv -- python3 tools/gemm_one.py 11 25800 3072 1024 0 10 > /dev/null 2>&1 || exit 1
  timeout -s KILL 90 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE GRBM_COUNT -d $O/$tag/p2 -o run --output-format csv -- python3 tools/gemm_one.py 11 25800 3072 1024 0 10 > /dev/null 2>&1 || exit 1
done
echo done
