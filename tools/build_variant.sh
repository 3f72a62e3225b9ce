#!/bin/bash
# Build the WORKING TREE's libpdm.so with extra compiler flags into ab/libpdm_<tag>.so (in-tree, git-ignored, travels
# to the GPU box) for same-box A/B or diagnostic runs:  tools/build_variant.sh TAG "-DPDM_G8S_DIAG"
set -e
TAG=$1; EXTRA=$2
ROOT=$(git rev-parse --show-toplevel)
TMP=$(mktemp -d)
mkdir -p $TMP/include $TMP/panopticdiffusionmodels_amd/csrc $ROOT/ab
cp $ROOT/include/pdm.h $TMP/include/
cp $ROOT/panopticdiffusionmodels_amd/csrc/*.hip $ROOT/panopticdiffusionmodels_amd/csrc/*.h $ROOT/panopticdiffusionmodels_amd/csrc/Makefile $TMP/panopticdiffusionmodels_amd/csrc/
make -s -j8 -C $TMP/panopticdiffusionmodels_amd/csrc OUT=$ROOT/ab/libpdm_$TAG.so EXTRA="$EXTRA"
rm -rf $TMP
echo "built ab/libpdm_$TAG.so (working tree, EXTRA=$EXTRA)"
