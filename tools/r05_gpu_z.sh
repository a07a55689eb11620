#!/bin/bash
# round 5, GPU step Z: 16 deferred slots per lane in the 4-wave fp32 walk at d <= 128 (scratch build
# tools/_ab/liblgx_p16.so) against the current build (tools/_ab/liblgx_r05d.so, 12): the Gowalla
# shape (eval_probe + route_probe), alternating; then the fp32 scoring tests on the variant.
set -o pipefail
OUT=gpurun_out/r05z
mkdir -p $OUT
export TMPDIR=/tmp
for rep in 1 2; do
  for lib in tools/_ab/liblgx_r05d.so tools/_ab/liblgx_p16.so; do
    echo "== $lib" >> $OUT/eval_probe.txt
    timeout -k 10 300 python -u tools/eval_probe.py --f32 --only gowalla --lib $lib >> $OUT/eval_probe.txt 2>&1 || { tail -30 $OUT/eval_probe.txt; exit 1; }
    echo "== $lib" >> $OUT/route_probe.txt
    timeout -k 10 600 python -u tools/route_probe.py --lib $lib >> $OUT/route_probe.txt 2>&1 || { tail -30 $OUT/route_probe.txt; exit 1; }
  done
done
grep -v amdgpu.ids $OUT/eval_probe.txt
grep -v amdgpu.ids $OUT/route_probe.txt | grep -v "threshold [0-9]*:"
