#!/bin/bash
# round 5, GPU step L: one-round-trip rescans (k <= 24 where the registers allow) + the drain's
# prefetched pending slots (tools/_ab/liblgx_rs1.so = this tree's build) against the round's
# evidence build (tools/_ab/liblgx_r05base.so): eval shapes (fp32) and the bf16 C5 call, alternating.
set -o pipefail
OUT=gpurun_out/r05l
mkdir -p $OUT
export TMPDIR=/tmp
for rep in 1 2; do
  for lib in tools/_ab/liblgx_r05base.so tools/_ab/liblgx_rs1.so; do
    echo "== $lib" >> $OUT/eval_probe.txt
    timeout -k 10 300 python -u tools/eval_probe.py --f32 --lib $lib >> $OUT/eval_probe.txt 2>&1 || { tail -30 $OUT/eval_probe.txt; exit 1; }
    echo "== $lib" >> $OUT/c5.txt
    timeout -k 10 300 python -u tools/score_traffic.py --users 262144 --calls 3 --lib $lib >> $OUT/c5.txt 2>&1 || { tail -30 $OUT/c5.txt; exit 1; }
  done
done
grep -v amdgpu.ids $OUT/eval_probe.txt
grep -v amdgpu.ids $OUT/c5.txt
for lib in tools/_ab/liblgx_r05base.so tools/_ab/liblgx_rs1.so; do
  echo "== $lib" >> $OUT/route_probe.txt
  timeout -k 10 600 python -u tools/route_probe.py --lib $lib >> $OUT/route_probe.txt 2>&1 || { tail -30 $OUT/route_probe.txt; exit 1; }
done
grep -v amdgpu.ids $OUT/route_probe.txt | grep -v "threshold [0-9]*:"
