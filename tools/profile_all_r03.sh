set -e
bash tools/profile_bench.sh r03a imagenet256_uvit_large 95
bash tools/profile_bench.sh r03a imagenet256_uvit_huge 95
bash tools/profile_bench.sh r03a imagenet512_uvit_huge 95 fp8
bash tools/profile_bench.sh r03a mscoco_uvit_small 64
