set -o pipefail
mkdir -p gpurun_out/r06es
for r in 50 100; do
  PDM_LIB_PATH=ab/libpdm_eseg.so timeout -k 10 150 python3 tools/g8s_eseg.py $r 2>&1 | grep -v amdgpu.ids >> gpurun_out/r06es/eseg.txt || exit 1
done
