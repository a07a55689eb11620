#!/bin/bash
# round 5, GPU step Y: on a deferred-slot overflow only the lane half holding the overflowing lane
# takes the exact path (tools/_ab/liblgx_ph.so = this tree's build) against the current build
# (tools/_ab/liblgx_r05d.so): the whole GPU suite on the new build first, then eval shapes and the
# bf16 C5 call, alternating.
set -o pipefail
OUT=gpurun_out/r05y
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest_gpu.txt 2>&1 || { tail -40 $OUT/pytest_gpu.txt; exit 1; }
tail -2 $OUT/pytest_gpu.txt
for rep in 1 2; do
  for lib in tools/_ab/liblgx_r05d.so tools/_ab/liblgx_ph.so; do
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
