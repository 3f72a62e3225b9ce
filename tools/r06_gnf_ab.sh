#!/bin/bash
# GroupNorm partials from the producing epilogues: decoder / kernel GPU tests, then decode timings with the fusion
# on and off (pdm_decoder_set_gn_fusion) and the default / H/4 bench against the committed library
set -o pipefail
O=gpurun_out/r06g2; mkdir -p $O
timeout -k 10 500 python -u -m pytest -x -q --timeout 250 --timeout-method thread tests/test_gpu_decoder.py \
  tests/test_gpu_kernels.py tests/test_gpu_output.py > $O/pytest.txt 2>&1 || exit 1
for r in 1 2; do
  for lib in ab/libpdm_base.so panopticdiffusionmodels_amd/libpdm.so; do
    t=$(basename $lib .so)
    PDM_LIB_PATH=$lib timeout -k 10 120 python3 tools/decode_bench.py 25 32 2>&1 | grep -v amdgpu.ids >> $O/dec256_$t.txt || exit 1
    PDM_LIB_PATH=$lib timeout -k 10 120 python3 tools/decode_bench.py 25 64 2>&1 | grep -v amdgpu.ids >> $O/dec512_$t.txt || exit 1
    PDM_LIB_PATH=$lib timeout -k 10 200 python3 bench.py --steps 3 --warmup 1 --cpu-baseline off > $O/l2_${t}_$r.txt 2>&1 || exit 1
    PDM_LIB_PATH=$lib timeout -k 10 200 python3 bench.py --config imagenet512_uvit_huge --steps 3 --warmup 1 --cpu-baseline off > $O/h4_${t}_$r.txt 2>&1 || exit 1
  done
done
