# rocprof evidence for every bench config at the bench defaults (tools/profile_bench.sh), tag = $1
set -e
TAG=${1:-r03w}
bash tools/profile_bench.sh $TAG imagenet256_uvit_large 50
bash tools/profile_bench.sh $TAG imagenet256_uvit_huge 50
bash tools/profile_bench.sh $TAG imagenet512_uvit_huge 50 fp8
bash tools/profile_bench.sh $TAG mscoco_uvit_small 50
