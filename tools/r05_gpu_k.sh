#!/bin/bash
# round 5, GPU step K: the stamped lab build with the full path split (drop_masked / drain inserts /
# direct inserts, rescans and wave-serial drain steps) at the evaluation shapes.
set -o pipefail
OUT=gpurun_out/r05k
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python -u tools/score_stats.py --only eval > $OUT/score_stats.txt 2>&1 || { tail -30 $OUT/score_stats.txt; exit 1; }
grep -v amdgpu.ids $OUT/score_stats.txt
