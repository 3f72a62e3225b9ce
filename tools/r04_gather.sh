#!/bin/bash
# t2i injection GEMM (row gather) on the persistent kernel: t2i parity tests, then the t2i forward A/B vs HEAD's lib.
OUT=${GRAFT_REPO_ROOT:-.}/gpurun_out/${1:-r04o}
mkdir -p $OUT
stop_on_fault() { case $1 in 0|1) return 0;; *) echo "step exited $1: stopping"; exit $1;; esac; }
timeout -k 10 600 python3 -u -m pytest -x -q -rf --timeout 300 --timeout-method thread tests/test_gpu_configs.py tests/test_fullsize_golden.py \
  -m gpu -k "mscoco or t2i" > $OUT/pytest.log 2>&1
s=$?; tail -4 $OUT/pytest.log; [ $s -ne 0 ] && exit $s
for r in 1 2 3; do
  for lib in ab/libpdm_head.so panopticdiffusionmodels_amd/libpdm.so; do
    PDM_LIB_PATH=$lib timeout -k 10 200 python3 tools/time_forward.py mscoco_uvit_small 48 20 >> $OUT/t2i_$(basename $lib .so).log 2>&1
    s=$?; stop_on_fault $s
  done
done
tail -3 $OUT/t2i_libpdm_head.log $OUT/t2i_libpdm.log
echo done
