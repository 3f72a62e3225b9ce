# rocprof evidence for every bench config (tools/profile_bench.sh), tag = $1 (default r03a)
set -e
TAG=${1:-r03a}
bash tools/profile_bench.sh $TAG imagenet256_uvit_large 95
bash tools/profile_bench.sh $TAG imagenet256_uvit_huge 95
bash tools/profile_bench.sh $TAG imagenet512_uvit_huge 95 fp8
bash tools/profile_bench.sh $TAG mscoco_uvit_small 64
