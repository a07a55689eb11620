#!/bin/bash
# round 5, GPU step J: the 8-wave fp32 walk at d = 128 with 4 deferred slots per lane (a 3-buffer ring
# fits) against this build (12 slots, 2 buffers): eval_probe + route_probe, alternating.
set -o pipefail
OUT=gpurun_out/r05j
mkdir -p $OUT
export TMPDIR=/tmp
for rep in 1 2; do
  for lib in factors_of_serendipity_recommendation_amd/liblgx.so tools/_ab/liblgx_e2.so; do
    echo "== $lib" >> $OUT/eval_probe.txt
    timeout -k 10 300 python -u tools/eval_probe.py --f32 --only amazon --lib $lib >> $OUT/eval_probe.txt 2>&1 || { tail -30 $OUT/eval_probe.txt; exit 1; }
  done
done
grep -v amdgpu.ids $OUT/eval_probe.txt
for lib in factors_of_serendipity_recommendation_amd/liblgx.so tools/_ab/liblgx_e2.so; do
  echo "== $lib" >> $OUT/route_probe.txt
  timeout -k 10 600 python -u tools/route_probe.py --lib $lib >> $OUT/route_probe.txt 2>&1 || { tail -30 $OUT/route_probe.txt; exit 1; }
done
grep -v amdgpu.ids $OUT/route_probe.txt | grep -v "threshold [0-9]*:"
