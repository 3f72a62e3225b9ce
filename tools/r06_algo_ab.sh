set -o pipefail
mkdir -p gpurun_out/r06al
for r in 50 100; do
  timeout -k 10 200 python3 tools/forward_algo_ab.py imagenet512_uvit_huge $r fp8 0,11,7 2>&1 | grep -v amdgpu.ids >> gpurun_out/r06al/h4.txt || exit 1
done
