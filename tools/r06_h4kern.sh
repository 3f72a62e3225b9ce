#!/bin/bash
# per-kernel time of the H/4 MXFP8 forward at the bench's lane rows (50), round-5 library vs the tree
set -o pipefail
export TMPDIR=/tmp
O=${GRAFT_REPO_ROOT:-.}/gpurun_out/r06h4; mkdir -p $O
for lib in ab/libpdm_head.so panopticdiffusionmodels_amd/libpdm.so; do
  t=$(basename $lib .so)
  PDM_LIB_PATH=$lib timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/kt_$t -o run --output-format csv -- python3 tools/time_forward.py imagenet512_uvit_huge 50 5 fp8 > $O/tf_$t.txt 2>&1 || exit 1
  cp $O/kt_$t/*/run_kernel_stats.csv $O/stats_$t.csv 2>/dev/null || find $O/kt_$t -name "*kernel_stats.csv" -exec cp {} $O/stats_$t.csv \;
  rm -rf $O/kt_$t
done
