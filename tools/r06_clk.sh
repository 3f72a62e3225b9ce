#!/bin/bash
set -o pipefail
O=gpurun_out/r06f; mkdir -p $O
for lib in clk clk3 clk4 clk; do
  echo "== $lib" >> $O/clk.txt
  PDM_LIB_PATH=ab/libpdm_$lib.so timeout -k 10 120 python tools/g8s_clock.py 100 2>&1 | grep -v amdgpu.ids >> $O/clk.txt || exit 1
done
