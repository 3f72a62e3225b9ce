#!/bin/bash
# Dh 72 attention variants (round 5): HEAD (algo 7), tree h72 (7) / h72p (14), builtin-V^T-read build (7 / 14)
OUT=${GRAFT_REPO_ROOT:-.}/gpurun_out/${1:-r05e}
mkdir -p $OUT
stop_on_fault() { case $1 in 0|1) return 0;; *) echo "step exited $1: stopping"; exit $1;; esac; }
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_kernels.py \
  -k "h72" > $OUT/pytest.log 2>&1
s=$?; tail -2 $OUT/pytest.log; stop_on_fault $s; [ $s -ne 0 ] && exit 1
for S in "100 258 16 72 7,8,9,14,15,16" "50 258 16 72 7,8,9,14"; do
  for L in ab/libpdm_head.so panopticdiffusionmodels_amd/libpdm.so ab/libpdm_vbuiltin.so; do
    PDM_LIB_PATH=$L timeout -k 10 120 python3 tools/attn_bench.py $S 2>&1 | grep -v amdgpu.ids | sed "s|^|$L |" | tee -a $OUT/attn.log
    s=${PIPESTATUS[0]}; stop_on_fault $s
  done
done
