#!/bin/bash
# round 5, GPU step AA: the fp32 floor window at the Gowalla shape -- the split's first quarter
# (tools/_ab/liblgx_fw4.so) and sixteenth (liblgx_fw16.so) against the eighth (liblgx_r05e.so, the
# current build): route_probe + eval_probe, rotating.
set -o pipefail
OUT=gpurun_out/r05aa
mkdir -p $OUT
export TMPDIR=/tmp
for rep in 1 2; do
  for lib in tools/_ab/liblgx_r05e.so tools/_ab/liblgx_fw4.so tools/_ab/liblgx_fw16.so; do
    echo "== $lib" >> $OUT/eval_probe.txt
    timeout -k 10 300 python -u tools/eval_probe.py --f32 --only gowalla --lib $lib >> $OUT/eval_probe.txt 2>&1 || { tail -30 $OUT/eval_probe.txt; exit 1; }
    echo "== $lib" >> $OUT/route_probe.txt
    timeout -k 10 600 python -u tools/route_probe.py --lib $lib >> $OUT/route_probe.txt 2>&1 || { tail -30 $OUT/route_probe.txt; exit 1; }
  done
done
grep -v amdgpu.ids $OUT/eval_probe.txt
grep -v amdgpu.ids $OUT/route_probe.txt | grep -v "threshold [0-9]*:" | grep -v "^amazon\|737 dense"
