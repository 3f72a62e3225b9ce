#!/bin/bash
set -o pipefail
O=gpurun_out/r06g; mkdir -p $O
for rows in 100 50; do
  echo "== clk rows $rows" >> $O/clk.txt
  PDM_LIB_PATH=ab/libpdm_clk.so timeout -k 10 120 python tools/g8s_clock.py $rows 2>&1 | grep -v amdgpu.ids >> $O/clk.txt || exit 1
done
