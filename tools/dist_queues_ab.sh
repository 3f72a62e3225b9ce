#!/bin/bash
# HIP hardware-queue A/B of bench.py under torch.distributed.run at world size 1 (4 vs 8 queues)
mkdir -p gpurun_out/dist3
for Q in 4 8; do
  PDM_KEEP_HW_QUEUES=1 GPU_MAX_HW_QUEUES=$Q timeout -k 10 400 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 2951$Q bench.py --gpus 1 --steps 2 --warmup 1 > gpurun_out/dist3/torchrun_q$Q.log 2>&1
done
for f in gpurun_out/dist3/*.log; do
  python3 -c "import json,sys; l=[x for x in open(sys.argv[1]) if x.startswith('{')][-1]; j=json.loads(l); print(sys.argv[1], j['value'], j['breakdown_ms_per_step']['sample_50nfe'])" $f
done
