#!/bin/bash
# Lane-stream priority A/B (sampler.LANE_STREAM_PRIORITY via PDM_LANE_PRIORITY): the plain bench and the bench under
# torch.distributed.run at world 1 with HIP's default 4 hardware queues kept, each at priority -1 (high) and 0
# (normal); then the epilogue cost decomposition of the L/2 GEMMs at the bench's rows 100.
OUT=${GRAFT_REPO_ROOT:-.}/gpurun_out/${1:-r04b}
mkdir -p $OUT
stop_on_fault() { case $1 in 0|1) return 0;; *) echo "step exited $1: stopping"; exit $1;; esac; }
port=29520
for prio in -1 0; do
  PDM_LANE_PRIORITY=$prio timeout -k 10 300 python3 bench.py --steps 3 --warmup 1 --cpu-baseline off \
    > $OUT/plain_p$prio.log 2>&1
  s=$?; echo "plain prio $prio: $(tail -1 $OUT/plain_p$prio.log | cut -c1-330)"; stop_on_fault $s
  port=$((port + 1))
  PDM_LANE_PRIORITY=$prio PDM_KEEP_HW_QUEUES=1 GPU_MAX_HW_QUEUES=4 timeout -k 10 400 python3 -m torch.distributed.run \
    --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port $port bench.py --gpus 1 --steps 3 --warmup 1 \
    --cpu-baseline off > $OUT/torchrun_q4_p$prio.log 2>&1
  s=$?; echo "torchrun q4 prio $prio: $(tail -1 $OUT/torchrun_q4_p$prio.log | cut -c1-330)"; stop_on_fault $s
done
timeout -k 10 300 python3 tools/epi_cost.py 100 > $OUT/epi_cost_rows100.log 2>&1
s=$?; cat $OUT/epi_cost_rows100.log; stop_on_fault $s
echo done
