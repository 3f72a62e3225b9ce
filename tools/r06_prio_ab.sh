#!/bin/bash
# MFMA-block priority variants of the persistent GEMM on the round-6 loop: per-block setprio (base), none (prio1),
# none + the younger half at priority 1 throughout (prio2, MI355X_MICROARCH / guide T5 static form)
set -o pipefail
O=gpurun_out/r06pr; mkdir -p $O
for r in 1 2; do
  for lib in ab/libpdm_base.so ab/libpdm_prio1.so ab/libpdm_prio2.so; do
    echo "== $lib rows 50" >> $O/shapes.txt
    PDM_LIB_PATH=$lib timeout -k 10 120 python tools/g8s_diag.py 50 2>&1 | grep -v amdgpu.ids >> $O/shapes.txt || exit 1
    PDM_LIB_PATH=$lib timeout -k 10 200 python3 bench.py --steps 3 --warmup 1 --cpu-baseline off > $O/l2_$(basename $lib .so)_$r.txt 2>&1 || exit 1
  done
done
