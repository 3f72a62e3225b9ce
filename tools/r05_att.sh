#!/bin/bash
# Attention change check (round 5): attention / forward / full-size parity GPU tests, then attn_bench at the bench's
# shapes for ab/libpdm_head.so vs the tree (interleaved libraries), then the default bench for both.  Usage: TAG
OUT=${GRAFT_REPO_ROOT:-.}/gpurun_out/${1:-r05att}
mkdir -p $OUT
stop_on_fault() { case $1 in 0|1) return 0;; *) echo "step exited $1: stopping"; exit $1;; esac; }
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_kernels.py \
  -k attention > $OUT/pytest.log 2>&1
s=$?; tail -3 $OUT/pytest.log; stop_on_fault $s; [ $s -ne 0 ] && exit 1
for S in "100 258 16 64 4,11,12,13" "50 258 16 64 4,11" "190 258 16 64 4,11" "100 258 16 72 7,14,15,16" "50 258 16 72 7,14" "32 334 8 64 4,11" "32 590 8 64 4,11"; do
  for L in ab/libpdm_head.so panopticdiffusionmodels_amd/libpdm.so; do
    PDM_LIB_PATH=$L timeout -k 10 120 python3 tools/attn_bench.py $S 2>&1 | grep -v amdgpu.ids | sed "s|^|$L |" | tee -a $OUT/attn.log
    s=${PIPESTATUS[0]}; stop_on_fault $s
  done
done
for i in 1 2; do
  PDM_LIB_PATH=ab/libpdm_head.so timeout -k 10 300 python3 bench.py --cpu-baseline off > $OUT/bench_head_$i.log 2>&1
  s=$?; stop_on_fault $s
  timeout -k 10 300 python3 bench.py --cpu-baseline off > $OUT/bench_new_$i.log 2>&1
  s=$?; stop_on_fault $s
done
for f in $OUT/bench_*.log; do echo "$f $(grep -o '"value": [0-9.]*' $f | head -1) $(grep -o '"sample_50nfe": [0-9.]*' $f | head -1)"; done
