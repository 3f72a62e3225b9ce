#!/bin/bash
# rocprof evidence (kernel trace + FETCH / WRITE) for the non-default bench configs at the round-4 HEAD
TAG=${1:-r04final}
bash tools/profile_bench.sh $TAG imagenet256_uvit_huge 50 || exit $?
bash tools/profile_bench.sh $TAG imagenet512_uvit_huge 50 fp8 || exit $?
bash tools/profile_bench.sh $TAG mscoco_uvit_small 32 || exit $?
echo done
