#!/bin/bash
# Development: build tools/score_lab from the sources of git revision $1 into tools/score_lab_ref
# (A/B timing of the working tree against a committed kernel in one GPU run)
set -e
REV=${1:-HEAD}
TMP=$(mktemp -d)
mkdir -p $TMP/src/factors_of_serendipity_recommendation_amd/csrc $TMP/src/include $TMP/src/tools
for f in score_topk.hip misc.hip stratify.hip wave_topk.h lgx_common.h; do
  git show $REV:factors_of_serendipity_recommendation_amd/csrc/$f > $TMP/src/factors_of_serendipity_recommendation_amd/csrc/$f
done
git show $REV:include/lgx.h > $TMP/src/include/lgx.h
cp tools/score_lab.hip $TMP/src/tools/score_lab.hip
C=$TMP/src/factors_of_serendipity_recommendation_amd/csrc
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -I$C -I$TMP/src/include -Wno-unused-result \
    $TMP/src/tools/score_lab.hip $C/misc.hip $C/stratify.hip -o tools/score_lab_ref
rm -rf $TMP
