#!/bin/bash
# A/B of the refill-before-lgkmcnt order in the tile GEMMs (gemm8d, gemm8t, gemm_mx_kernel) + division-free conv addressing: parity tests on the
# variant, then decode / H/4 / default bench timings alternating with the committed library (ab/libpdm_head7.so)
set -o pipefail
O=gpurun_out/r06w; mkdir -p $O
PDM_LIB_PATH=ab/libpdm_conv2.so timeout -k 10 500 python -u -m pytest -x -q --timeout 250 --timeout-method thread \
  tests/test_gpu_kernels.py tests/test_gpu_fp8.py tests/test_gpu_decoder.py tests/test_gpu_streamk.py > $O/pytest.txt 2>&1 || exit 1
for r in 1 2; do
  for lib in ab/libpdm_head7.so ab/libpdm_conv2.so; do
    t=$(basename $lib .so)
    PDM_LIB_PATH=$lib timeout -k 10 120 python3 tools/decode_bench.py 25 32 2>&1 | grep -v amdgpu.ids >> $O/dec256_$t.txt || exit 1
    PDM_LIB_PATH=$lib timeout -k 10 120 python3 tools/decode_bench.py 25 64 2>&1 | grep -v amdgpu.ids >> $O/dec512_$t.txt || exit 1
    PDM_LIB_PATH=$lib timeout -k 10 200 python3 bench.py --steps 3 --warmup 1 --cpu-baseline off > $O/l2_${t}_$r.txt 2>&1 || exit 1
    PDM_LIB_PATH=$lib timeout -k 10 200 python3 bench.py --config imagenet512_uvit_huge --steps 3 --warmup 1 --cpu-baseline off > $O/h4_${t}_$r.txt 2>&1 || exit 1
  done
done
