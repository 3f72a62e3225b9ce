#!/bin/bash
# kernel trace of the decode after the round-6 decoder changes (25-image chunks, 256^2 and 512^2)
set -o pipefail
export TMPDIR=/tmp
O=${GRAFT_REPO_ROOT:-.}/gpurun_out/r06k2; mkdir -p $O
for lat in 32 64; do
  timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/kt$lat -o run --output-format csv -- python3 tools/decode_bench.py 25 $lat > $O/dec$lat.txt 2>&1 || exit 1
  find $O/kt$lat -name "*kernel_stats.csv" -exec cp {} $O/dec${lat}_kernel_stats.csv \;
  rm -rf $O/kt$lat
done
