#!/bin/bash
# Same-box bench A/B of library builds, alternating (dev tool): tools/ab_bench.sh OUTDIR "BENCH ARGS" LIB [LIB ...]
set -o pipefail
O=gpurun_out/$1; ARGS=$2; shift 2; mkdir -p $O
for r in 1 2; do
  for lib in "$@"; do
    PDM_LIB_PATH=$lib timeout -k 10 300 python3 bench.py --steps 4 --warmup 1 --cpu-baseline off $ARGS \
      > $O/ab_$(basename $lib .so)_$r.txt 2>&1 || exit 1
  done
done
