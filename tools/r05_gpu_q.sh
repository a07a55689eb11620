#!/bin/bash
# round 5, GPU step Q: staggered LDS walks with only the late half staging the tiles
# (tools/_ab/liblgx_ls.so) against the round-5 base with the f4 stagger (tools/_ab/liblgx_r05f4.so):
# bf16 C5 call at 262144 users and the fp32 Amazon-book shape, alternating.
set -o pipefail
OUT=gpurun_out/r05q
mkdir -p $OUT
export TMPDIR=/tmp
for rep in 1 2; do
  for lib in tools/_ab/liblgx_r05f4.so tools/_ab/liblgx_ls.so; do
    echo "== $lib" >> $OUT/c5.txt
    timeout -k 10 300 python -u tools/score_traffic.py --users 262144 --calls 3 --lib $lib >> $OUT/c5.txt 2>&1 || { tail -30 $OUT/c5.txt; exit 1; }
    echo "== $lib" >> $OUT/eval_probe.txt
    timeout -k 10 300 python -u tools/eval_probe.py --f32 --only amazon --lib $lib >> $OUT/eval_probe.txt 2>&1 || { tail -30 $OUT/eval_probe.txt; exit 1; }
  done
done
grep -v amdgpu.ids $OUT/c5.txt
grep -v amdgpu.ids $OUT/eval_probe.txt
