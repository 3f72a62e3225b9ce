set -o pipefail
mkdir -p gpurun_out/r06r
for r in 50 100; do timeout -k 10 120 python tools/g8s_diag.py $r 2>&1 | grep -v amdgpu.ids >> gpurun_out/r06r/nostore.txt || exit 1; done
