#!/bin/bash
# round 5, GPU step G: refined cycle breakdown (stamped lab build); the fp32 8-wave walk with the early
# waves' refill at the top of the iteration (v1) against this build.
set -o pipefail
OUT=gpurun_out/r05g
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u tools/score_stats.py --only eval > $OUT/score_stats.txt 2>&1 || { tail -30 $OUT/score_stats.txt; exit 1; }
grep -v amdgpu.ids $OUT/score_stats.txt
for rep in 1 2; do
  for lib in factors_of_serendipity_recommendation_amd/liblgx.so tools/_ab/liblgx_v1.so; do
    echo "== $lib" >> $OUT/eval_probe.txt
    timeout -k 10 300 python -u tools/eval_probe.py --f32 --lib $lib >> $OUT/eval_probe.txt 2>&1 || { tail -30 $OUT/eval_probe.txt; exit 1; }
  done
done
grep -v amdgpu.ids $OUT/eval_probe.txt
