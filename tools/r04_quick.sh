#!/bin/bash
# Round-4 first checks on the GPU box: the new / changed tests, the configs[0] bench line, the lanes under the
# default 4 HIP hardware queues (torchrun, world 1).  Every GPU step has its own limit; a fault ends the script.
OUT=${GRAFT_REPO_ROOT:-.}/gpurun_out/${1:-r04a}
mkdir -p $OUT
stop_on_fault() { case $1 in 0|1) return 0;; *) echo "step exited $1: stopping"; exit $1;; esac; }
timeout -k 10 600 python3 -u -m pytest -x -q -rf --timeout 300 --timeout-method thread \
  tests/test_fullsize_golden.py tests/test_gpu_train.py::test_train_label_out_of_range_raises \
  tests/test_gpu_fp8.py::test_fp8_lanes_recapture_after_precision_switch tests/test_gpu_sample.py \
  -m gpu > $OUT/pytest.log 2>&1
s=$?; tail -15 $OUT/pytest.log; stop_on_fault $s
timeout -k 10 300 python3 bench.py --config cifar10_uvit_small --steps 5 --warmup 2 > $OUT/bench_cifar.log 2>&1
s=$?; tail -2 $OUT/bench_cifar.log; stop_on_fault $s
PDM_KEEP_HW_QUEUES=1 GPU_MAX_HW_QUEUES=4 timeout -k 10 400 python3 -m torch.distributed.run --nnodes=1 \
  --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29514 bench.py --gpus 1 --steps 3 --warmup 1 \
  --cpu-baseline off > $OUT/torchrun_q4.log 2>&1
s=$?; tail -2 $OUT/torchrun_q4.log | cut -c1-400; stop_on_fault $s
timeout -k 10 300 python3 tools/sol_forward.py imagenet256_uvit_large 100 5 > $OUT/sol_l2.log 2>&1
s=$?; cat $OUT/sol_l2.log; stop_on_fault $s
echo done
