#!/bin/bash
# Lanes sweep of the bench lines with the persistent GEMM (each 3 timed steps, no CPU baseline).
OUT=${GRAFT_REPO_ROOT:-.}/gpurun_out/${1:-r04s}
mkdir -p $OUT
stop_on_fault() { case $1 in 0|1) return 0;; *) echo "step exited $1: stopping"; exit $1;; esac; }
run() {   # name, args...
  local n=$1; shift
  timeout -k 10 300 python3 bench.py --steps 3 --warmup 1 --cpu-baseline off "$@" > $OUT/$n.log 2>&1
  local s=$?; echo "$n: $(tail -1 $OUT/$n.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d.get("breakdown_ms_per_step"))' 2>/dev/null)"
  stop_on_fault $s
}
for l in 1 2 3 4; do run l2_lanes$l --lanes $l; done
run l2_b64_l2 --batch 64 --lanes 2
run l2_b64_l4 --batch 64 --lanes 4
for l in 1 2 3; do run t2i_lanes$l --config mscoco_uvit_small --lanes $l; done
run t2i_b64_l2 --config mscoco_uvit_small --batch 64 --lanes 2
for l in 2 3; do run h4_lanes$l --config imagenet512_uvit_huge --lanes $l; done
echo done
