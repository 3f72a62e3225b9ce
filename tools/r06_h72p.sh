set -o pipefail
mkdir -p gpurun_out/r06h72
for r in 50 100; do
  timeout -k 10 120 python3 tools/attn_bench.py $r 258 16 72 0,14 2>&1 | grep -v amdgpu.ids >> gpurun_out/r06h72/h72.txt || exit 1
  timeout -k 10 120 python3 tools/attn_bench.py $r 258 16 64 0,11,2 2>&1 | grep -v amdgpu.ids >> gpurun_out/r06h72/v3.txt || exit 1
done
