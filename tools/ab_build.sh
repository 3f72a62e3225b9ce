#!/bin/bash
# Build libpdm.so of another git revision into ab/libpdm_<tag>.so (in-tree, git-ignored, travels to the GPU box)
# for same-box A/B timing:  PDM_LIB_PATH=ab/libpdm_<tag>.so python3 tools/attn_bench.py ...
# Usage: tools/ab_build.sh REV TAG
set -e
REV=${1:-HEAD}; TAG=${2:-head}
ROOT=$(git rev-parse --show-toplevel)
TMP=$(mktemp -d)
mkdir -p $TMP/include $TMP/panopticdiffusionmodels_amd/csrc $ROOT/ab
git -C $ROOT show $REV:include/pdm.h > $TMP/include/pdm.h
for f in $(git -C $ROOT ls-tree --name-only $REV panopticdiffusionmodels_amd/csrc/); do
  git -C $ROOT show $REV:$f > $TMP/$f
done
make -s -j8 -C $TMP/panopticdiffusionmodels_amd/csrc OUT=$ROOT/ab/libpdm_$TAG.so
rm -rf $TMP
echo "built ab/libpdm_$TAG.so from $REV"
