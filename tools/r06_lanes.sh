#!/bin/bash
# lanes sweep on the round-6 tree (default bench, B = 50): 1 / 2 / 3 lanes, and decode lanes 1 / 2 / 3
set -o pipefail
O=gpurun_out/r06lanes; mkdir -p $O
for l in 2 3 1 2; do
  timeout -k 10 300 python3 bench.py --steps 3 --warmup 1 --cpu-baseline off --lanes $l > $O/l2_lanes${l}_$RANDOM.txt 2>&1 || exit 1
done
for dl in 1 3; do
  timeout -k 10 300 python3 bench.py --steps 3 --warmup 1 --cpu-baseline off --decode-lanes $dl > $O/l2_declanes$dl.txt 2>&1 || exit 1
done
for l in 2 3; do
  timeout -k 10 300 python3 bench.py --config imagenet512_uvit_huge --steps 3 --warmup 1 --cpu-baseline off --lanes $l > $O/h4_lanes$l.txt 2>&1 || exit 1
done
