#!/bin/bash
# rocprof evidence for the H/2 and CIFAR bench lines of the round-6 tree
set -o pipefail
bash tools/profile_bench.sh r06z imagenet256_uvit_huge 50 || exit 1
bash tools/profile_bench.sh r06z cifar10_uvit_small 4 || exit 1
