#!/bin/bash
# L/2 (configs[1]) throughput vs per-GPU batch, one bench line per batch (SURVEY.md §8d "B=50 (sweep 8..256)")
# Usage: [LANES=k] tools/batch_sweep.sh OUTDIR [batches...]
OUT=${1:-gpurun_out/sweep}; shift
LANES=${LANES:-1}
mkdir -p $OUT
for B in ${@:-8 16 32 50 64 95 128 190}; do
  timeout -k 10 400 python3 bench.py --batch $B --lanes $LANES --steps 2 --warmup 1 --cpu-baseline off > $OUT/bench_b${B}_l$LANES.log 2>&1 || exit $?
  python3 -c "import json,sys; d=json.loads(open('$OUT/bench_b${B}_l$LANES.log').read().strip().splitlines()[-1]); print('B=%d lanes=%d %.2f img/s gemm %.1f TF/s frac %.3f e2e %.3f' % ($B, $LANES, d['value'], d['roofline']['achieved'], d['roofline']['frac'], d['end_to_end']['frac_of_peak']))"
done
