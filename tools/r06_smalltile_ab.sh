#!/bin/bash
# the 128 x 128 tile for GEMMs with fewer 256-tiles than half the CUs (ab/libpdm_smalltile.so) vs the tree: t2i /
# config GPU tests on the variant, then the t2i and default benches alternating
set -o pipefail
O=gpurun_out/r06st; mkdir -p $O
PDM_LIB_PATH=ab/libpdm_smalltile.so timeout -k 10 500 python -u -m pytest -x -q --timeout 250 --timeout-method thread \
  tests/test_gpu_t2i.py tests/test_gpu_configs.py tests/test_gpu_kernels.py tests/test_gpu_benchbatch.py > $O/pytest.txt 2>&1 || exit 1
for r in 1 2 3; do
  for lib in panopticdiffusionmodels_amd/libpdm.so ab/libpdm_smalltile.so; do
    t=$(basename $lib .so)
    PDM_LIB_PATH=$lib timeout -k 10 200 python3 bench.py --config mscoco_uvit_small --steps 3 --warmup 1 --cpu-baseline off > $O/t2i_${t}_$r.txt 2>&1 || exit 1
  done
done
for lib in panopticdiffusionmodels_amd/libpdm.so ab/libpdm_smalltile.so; do
  PDM_LIB_PATH=$lib timeout -k 10 200 python3 bench.py --steps 3 --warmup 1 --cpu-baseline off > $O/l2_$(basename $lib .so).txt 2>&1 || exit 1
done
