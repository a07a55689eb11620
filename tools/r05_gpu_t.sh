#!/bin/bash
# round 5, GPU step T: rescans over whole 8-key groups without bounds tests + a 2-read tail
# (tools/_ab/liblgx_rg.so) against the current build (tools/_ab/liblgx_r05f4.so): eval shapes (fp32,
# random and propagated tables) and the bf16 C5 call, alternating.
set -o pipefail
OUT=gpurun_out/r05t
mkdir -p $OUT
export TMPDIR=/tmp
for rep in 1 2; do
  for lib in tools/_ab/liblgx_r05f4.so tools/_ab/liblgx_rg.so; do
    echo "== $lib" >> $OUT/eval_probe.txt
    timeout -k 10 300 python -u tools/eval_probe.py --f32 --lib $lib >> $OUT/eval_probe.txt 2>&1 || { tail -30 $OUT/eval_probe.txt; exit 1; }
    echo "== $lib" >> $OUT/c5.txt
    timeout -k 10 300 python -u tools/score_traffic.py --users 262144 --calls 3 --lib $lib >> $OUT/c5.txt 2>&1 || { tail -30 $OUT/c5.txt; exit 1; }
    echo "== $lib" >> $OUT/route_probe.txt
    timeout -k 10 600 python -u tools/route_probe.py --lib $lib >> $OUT/route_probe.txt 2>&1 || { tail -30 $OUT/route_probe.txt; exit 1; }
  done
done
grep -v amdgpu.ids $OUT/eval_probe.txt
grep -v amdgpu.ids $OUT/c5.txt
grep -v amdgpu.ids $OUT/route_probe.txt | grep -v "threshold [0-9]*:"
