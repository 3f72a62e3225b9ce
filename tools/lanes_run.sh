set -e
mkdir -p gpurun_out/r03u
timeout -k 10 300 python -u -m pytest tests/test_gpu_sample.py tests/test_gpu_configs.py -m gpu -x -q --timeout 250 --timeout-method thread > gpurun_out/r03u/pytest.log 2>&1
for L in 1 2; do
  timeout -k 10 400 python3 bench.py --config mscoco_uvit_small --batch 64 --lanes $L --steps 2 --warmup 1 --cpu-baseline off > gpurun_out/r03u/t2i_l$L.log 2>&1
  timeout -k 10 400 python3 bench.py --config imagenet256_uvit_huge --batch 95 --lanes $L --steps 2 --warmup 1 --cpu-baseline off > gpurun_out/r03u/h2_l$L.log 2>&1
  timeout -k 10 400 python3 bench.py --config imagenet512_uvit_huge --batch 95 --lanes $L --steps 2 --warmup 1 --cpu-baseline off > gpurun_out/r03u/h4_l$L.log 2>&1
done
LANES=2 bash tools/batch_sweep.sh gpurun_out/r03u/sweep 8 16 32 190 > gpurun_out/r03u/sweep_l2.txt 2>&1
LANES=3 bash tools/batch_sweep.sh gpurun_out/r03u/sweep 50 95 > gpurun_out/r03u/sweep_l3.txt 2>&1
LANES=1 bash tools/batch_sweep.sh gpurun_out/r03u/sweep 8 16 32 190 > gpurun_out/r03u/sweep_l1.txt 2>&1
