#!/bin/bash
# the bench under torch.distributed.run at world size 1 (the driver's N > 1 launch form) on one GPU
set -o pipefail
O=gpurun_out/r06dist; mkdir -p $O
timeout -k 10 400 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 1 --steps 3 --warmup 1 > $O/torchrun_w1.txt 2>&1 || exit 1
