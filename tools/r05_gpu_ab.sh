#!/bin/bash
# round 5, GPU step AB: the Amazon-book shape on the 4-wave fp32 walk (16 deferred slots, score
# floors; scratch build tools/_ab/liblgx_w4.so with the 8-wave walk disabled) against the current
# build (8 waves, 12 slots): eval_probe + route_probe, alternating.
set -o pipefail
OUT=gpurun_out/r05ab
mkdir -p $OUT
export TMPDIR=/tmp
for rep in 1 2; do
  for lib in tools/_ab/liblgx_r05e.so tools/_ab/liblgx_w4.so; do
    echo "== $lib" >> $OUT/eval_probe.txt
    timeout -k 10 300 python -u tools/eval_probe.py --f32 --only amazon --lib $lib >> $OUT/eval_probe.txt 2>&1 || { tail -30 $OUT/eval_probe.txt; exit 1; }
    echo "== $lib" >> $OUT/route_probe.txt
    timeout -k 10 600 python -u tools/route_probe.py --lib $lib >> $OUT/route_probe.txt 2>&1 || { tail -30 $OUT/route_probe.txt; exit 1; }
  done
done
grep -v amdgpu.ids $OUT/eval_probe.txt
grep -v amdgpu.ids $OUT/route_probe.txt | grep -v "threshold [0-9]*:" | grep -v "^gowalla\|981 dense"
