#!/bin/bash
# round 5, GPU step AG: the dense-route threshold with the dense route beside the fused launch
set -o pipefail
OUT=gpurun_out/r05ag
mkdir -p $OUT
export TMPDIR=/tmp
for rep in 1 2; do
  timeout -k 10 600 python -u tools/route_probe.py >> $OUT/route_probe.txt 2>&1 || { tail -30 $OUT/route_probe.txt; exit 1; }
done
grep -v amdgpu.ids $OUT/route_probe.txt
