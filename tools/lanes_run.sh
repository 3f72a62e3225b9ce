#!/bin/bash
# lanes A/B on every bench config + L/2 batch sweep at 1-4 lanes.  Usage: tools/lanes_run.sh TAG
set -e
OUT=gpurun_out/${1:-lanes}
mkdir -p $OUT
for L in 1 2; do
  timeout -k 10 400 python3 bench.py --config mscoco_uvit_small --batch 64 --lanes $L --steps 2 --warmup 1 --cpu-baseline off > $OUT/t2i_b64_l$L.log 2>&1
  tail -c 300 $OUT/t2i_b64_l$L.log | grep -o '"value": [0-9.]*' | sed "s/^/t2i B=64 lanes=$L /"
  timeout -k 10 400 python3 bench.py --config imagenet256_uvit_huge --batch 50 --lanes $L --steps 2 --warmup 1 --cpu-baseline off > $OUT/h2_b50_l$L.log 2>&1
  grep -o '"value": [0-9.]*' $OUT/h2_b50_l$L.log | head -1 | sed "s/^/H2 B=50 lanes=$L /"
  timeout -k 10 400 python3 bench.py --config imagenet512_uvit_huge --batch 50 --lanes $L --steps 2 --warmup 1 --cpu-baseline off > $OUT/h4_b50_l$L.log 2>&1
  grep -o '"value": [0-9.]*' $OUT/h4_b50_l$L.log | head -1 | sed "s/^/H4 B=50 lanes=$L /"
done
LANES=3 bash tools/batch_sweep.sh $OUT/sweep 50 96 > $OUT/sweep_l3.txt 2>&1; cat $OUT/sweep_l3.txt
LANES=4 bash tools/batch_sweep.sh $OUT/sweep 64 100 128 > $OUT/sweep_l4.txt 2>&1; cat $OUT/sweep_l4.txt
LANES=2 bash tools/batch_sweep.sh $OUT/sweep 8 16 32 190 > $OUT/sweep_l2.txt 2>&1; cat $OUT/sweep_l2.txt
