#!/bin/bash
# Round-6 final validation on one MI355X.  Part A: GPU suite, smoke, the default bench line (with its CPU baseline),
# a same-box A/B of the default bench against the round-5 library (ab/libpdm_head.so, built from c170268).  Part B:
# every other config's bench line with its CPU baseline.  Usage: TAG A|B
TAG=${1:-r06f}; PART=${2:-A}
OUT=${GRAFT_REPO_ROOT:-.}/gpurun_out/$TAG
mkdir -p $OUT
stop_on_fault() { case $1 in 0|1) return 0;; *) echo "step exited $1: stopping"; exit $1;; esac; }
if [ "$PART" = A ]; then
  timeout -k 10 700 python3 -u -m pytest -q -rf --timeout 300 --timeout-method thread tests -m gpu > $OUT/pytest.txt 2>&1
  s=$?; tail -4 $OUT/pytest.txt; stop_on_fault $s
  timeout -k 10 200 python3 -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.txt 2>&1
  s=$?; tail -3 $OUT/smoke.txt; stop_on_fault $s
  timeout -k 10 300 python3 bench.py --steps 5 --warmup 2 > $OUT/bench.txt 2>&1
  s=$?; tail -1 $OUT/bench.txt | cut -c1-300; stop_on_fault $s
  for r in 1 2; do
    for lib in ab/libpdm_head.so panopticdiffusionmodels_amd/libpdm.so; do
      PDM_LIB_PATH=$lib timeout -k 10 200 python3 bench.py --steps 4 --warmup 1 --cpu-baseline off > $OUT/ab_$(basename $lib .so)_$r.txt 2>&1
      s=$?; stop_on_fault $s
    done
  done
else
  for c in imagenet256_uvit_huge imagenet512_uvit_huge mscoco_uvit_small cifar10_uvit_small; do
    timeout -k 10 300 python3 bench.py --config $c --steps 3 --warmup 1 > $OUT/bench_$c.txt 2>&1
    s=$?; tail -1 $OUT/bench_$c.txt | cut -c1-260; stop_on_fault $s
  done
  for lib in ab/libpdm_head.so panopticdiffusionmodels_amd/libpdm.so; do
    for c in imagenet256_uvit_huge imagenet512_uvit_huge mscoco_uvit_small; do
      PDM_LIB_PATH=$lib timeout -k 10 200 python3 bench.py --config $c --steps 3 --warmup 1 --cpu-baseline off > $OUT/ab_$(basename $lib .so)_$c.txt 2>&1
      s=$?; stop_on_fault $s
    done
  done
fi
echo done
