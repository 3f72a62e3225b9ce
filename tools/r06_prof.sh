#!/bin/bash
# Round-6 rocprof evidence: kernel trace + FETCH / WRITE passes of the default, t2i and H/4 benches
set -o pipefail
bash tools/profile_bench.sh r06p imagenet256_uvit_large 50 || exit 1
bash tools/profile_bench.sh r06p mscoco_uvit_small 32 || exit 1
bash tools/profile_bench.sh r06p imagenet512_uvit_huge 50 fp8 || exit 1
