#!/bin/bash
# GEMM L2-miss traffic vs tile order (is the 5-6.5x operand FETCH of qkv / fc1 costing time?):
# per raster, kernel trace + FETCH_SIZE + TCC hit / miss of the persistent GEMM at rows 100 (M = 25,800), plain bf16.
# Usage: TAG
OUT=$GRAFT_REPO_ROOT/gpurun_out/${1:-rtraffic}
mkdir -p $OUT
export TMPDIR=/tmp
for S in "3072 1024" "4096 1024" "1024 4096"; do
  set -- $S
  for R in 1 8 32; do
    T=$OUT/n$1_k$2_r$R
    PDM_RASTER=$R timeout -s KILL 60 rocprofv3 --kernel-trace --stats -d $T/kt -o run --output-format csv -- python3 tools/gemm_one.py 11 25800 $1 $2 0 20 > /dev/null 2>&1 || { echo "kt fail $S $R"; exit 1; }
    PDM_RASTER=$R timeout -s KILL 60 rocprofv3 --pmc FETCH_SIZE -d $T/fetch -o run --output-format csv -- python3 tools/gemm_one.py 11 25800 $1 $2 0 5 > /dev/null 2>&1 || { echo "fetch fail $S $R"; exit 1; }
    PDM_RASTER=$R timeout -s KILL 60 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum -d $T/hit -o run --output-format csv -- python3 tools/gemm_one.py 11 25800 $1 $2 0 5 > /dev/null 2>&1 || { echo "hit fail $S $R"; exit 1; }
    echo "done N=$1 K=$2 raster=$R"
  done
done
