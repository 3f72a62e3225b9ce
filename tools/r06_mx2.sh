set -o pipefail
mkdir -p gpurun_out/r06v
timeout -k 10 200 python3 tools/mx_res_bench.py 25,50,100 1152,1152 2>&1 | grep -v amdgpu.ids > gpurun_out/r06v/mx_res.txt || exit 1
timeout -k 10 200 python3 tools/mx_res_bench.py 25,50,100 1152,4608 2>&1 | grep -v amdgpu.ids >> gpurun_out/r06v/mx_res.txt || exit 1
