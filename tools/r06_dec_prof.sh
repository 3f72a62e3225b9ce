#!/bin/bash
# Round 6: where the KL-f8 decode spends its time (kernel trace of 25-image chunks at 256^2 and 512^2)
set -o pipefail
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/r06k; mkdir -p $O
timeout -k 10 200 python3 tools/decode_bench.py 25 32 > $O/dec256.txt 2>&1 || exit 1
timeout -k 10 200 python3 tools/decode_bench.py 25 64 > $O/dec512.txt 2>&1 || exit 1
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/kt256 -o run --output-format csv -- python3 tools/decode_bench.py 25 32 > /dev/null 2>&1 || exit 1
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/kt512 -o run --output-format csv -- python3 tools/decode_bench.py 25 64 > /dev/null 2>&1 || exit 1
echo done
