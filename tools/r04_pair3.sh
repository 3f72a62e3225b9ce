#!/bin/bash
# Split one-problem / grouped kernels: GEMM + t2i tests, then L/2 and t2i forwards vs the pre-grouping lib.
OUT=${GRAFT_REPO_ROOT:-.}/gpurun_out/${1:-r04z}
mkdir -p $OUT
stop_on_fault() { case $1 in 0|1) return 0;; *) echo "step exited $1: stopping"; exit $1;; esac; }
timeout -k 10 900 python3 -u -m pytest -x -q -rf --timeout 300 --timeout-method thread tests/test_gpu_kernels.py tests/test_gpu_fp8.py tests/test_gpu_configs.py tests/test_fullsize_golden.py \
  -m gpu -k "gemm or mx or mscoco or t2i" > $OUT/pytest.log 2>&1
s=$?; tail -2 $OUT/pytest.log; [ $s -ne 0 ] && exit $s
for r in 1 2 3 4; do
  for lib in ab/libpdm_head.so panopticdiffusionmodels_amd/libpdm.so; do
    n=$(basename $lib .so)
    PDM_LIB_PATH=$lib timeout -k 10 200 python3 tools/time_forward.py imagenet256_uvit_large 100 10 >> $OUT/l2_fwd_$n.log 2>&1
    s=$?; stop_on_fault $s
  done
done
PDM_LIB_PATH=panopticdiffusionmodels_amd/libpdm.so timeout -k 10 200 python3 tools/time_forward.py mscoco_uvit_small 32 20 > $OUT/t2i_fwd.log 2>&1
grep -H ms/forward $OUT/*.log
echo done
