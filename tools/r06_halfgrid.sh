#!/bin/bash
# experiment: residual GEMMs of at most one round of tiles on half the workgroups (ab/libpdm_halfgrid.so) vs the tree
set -o pipefail
O=gpurun_out/r06hg; mkdir -p $O
for r in 1 2; do
  for lib in ab/libpdm_base.so ab/libpdm_halfgrid.so; do
    echo "== $lib rows 50" >> $O/shapes.txt
    PDM_LIB_PATH=$lib timeout -k 10 120 python tools/g8s_diag.py 50 2>&1 | grep -E "proj|fc2|skip" >> $O/shapes.txt || exit 1
    PDM_LIB_PATH=$lib timeout -k 10 200 python3 bench.py --steps 3 --warmup 1 --cpu-baseline off > $O/l2_$(basename $lib .so)_$r.txt 2>&1 || exit 1
  done
done
