#!/bin/bash
# round 5, GPU step AD: 8 mask searches in lockstep instead of 4 in the 4-wave fp32 walk up to
# d = 128 (scratch build tools/_ab/liblgx_ks.so) against the current build: the Gowalla route.
set -o pipefail
OUT=gpurun_out/r05ad
mkdir -p $OUT
export TMPDIR=/tmp
for rep in 1 2 3; do
  for lib in tools/_ab/liblgx_r05e.so tools/_ab/liblgx_ks.so; do
    echo "== $lib" >> $OUT/route_probe.txt
    timeout -k 10 600 python -u tools/route_probe.py --lib $lib >> $OUT/route_probe.txt 2>&1 || { tail -30 $OUT/route_probe.txt; exit 1; }
  done
done
grep -v amdgpu.ids $OUT/route_probe.txt | grep -v "threshold [0-9]*:" | grep -v "^amazon\|737 dense"
