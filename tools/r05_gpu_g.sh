#!/bin/bash
# round 5, GPU step G: refined cycle breakdown (stamped lab build); variants of the fp32 walk against
# this build at the evaluation shapes (random tables: eval_probe; propagated tables: route_probe):
# v1 = the early waves' refill at the top of the iteration (fp32); v3 = v1 + fp32 score floors over
# each split's first eighth; v4 = list rows padded to a conflict-free stride (if present).
set -o pipefail
OUT=gpurun_out/r05g
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u tools/score_stats.py --only eval > $OUT/score_stats.txt 2>&1 || { tail -30 $OUT/score_stats.txt; exit 1; }
grep -v amdgpu.ids $OUT/score_stats.txt
LIBS="factors_of_serendipity_recommendation_amd/liblgx.so tools/_ab/liblgx_v1.so tools/_ab/liblgx_v3.so"
[ -f tools/_ab/liblgx_v4.so ] && LIBS="$LIBS tools/_ab/liblgx_v4.so"
for rep in 1 2; do
  for lib in $LIBS; do
    echo "== $lib" >> $OUT/eval_probe.txt
    timeout -k 10 300 python -u tools/eval_probe.py --f32 --lib $lib >> $OUT/eval_probe.txt 2>&1 || { tail -30 $OUT/eval_probe.txt; exit 1; }
  done
done
grep -v amdgpu.ids $OUT/eval_probe.txt
for lib in $LIBS; do
  echo "== $lib" >> $OUT/route_probe.txt
  timeout -k 10 600 python -u tools/route_probe.py --lib $lib >> $OUT/route_probe.txt 2>&1 || { tail -30 $OUT/route_probe.txt; exit 1; }
done
grep -v amdgpu.ids $OUT/route_probe.txt
