#!/bin/bash
# PMC passes over the GEMM tile policies on the U-ViT shapes (run on the GPU box from the repo root).
set -e
export TMPDIR=/tmp
bash tools/pmc_gemm.sh 5 49152 4096 4096 0 a5big
bash tools/pmc_gemm.sh 5 49020 1024 4096 2 a5fc2
bash tools/pmc_gemm.sh 4 49152 4096 4096 0 a4big
