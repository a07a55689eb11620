#!/bin/bash
# round 5, GPU step N: 64 parked mask suspects per (user, split, half) (tools/_ab/liblgx_p64.so)
# against the round's evidence build (32), route_probe on propagated tables, alternating.
set -o pipefail
OUT=gpurun_out/r05n
mkdir -p $OUT
export TMPDIR=/tmp
for rep in 1 2; do
  for lib in tools/_ab/liblgx_r05base.so tools/_ab/liblgx_p64.so; do
    echo "== $lib" >> $OUT/route_probe.txt
    timeout -k 10 600 python -u tools/route_probe.py --lib $lib >> $OUT/route_probe.txt 2>&1 || { tail -30 $OUT/route_probe.txt; exit 1; }
  done
done
grep -v amdgpu.ids $OUT/route_probe.txt | grep -v "threshold [0-9]*:"
