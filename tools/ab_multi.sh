#!/bin/bash
# A/B/C... of liblgx.so builds on the evaluation shapes only (tools/route_probe.py), alternating
# builds, two rounds:  bash tools/ab_multi.sh OUTDIR lib1 lib2 [lib3 ...]
set -o pipefail
OUT=$1; shift
for rep in 1 2; do
  for lib in "$@"; do
    n=$(basename "$lib" .so)_$rep
    GPU_STEP_TAIL=0 bash tools/gpu_step.sh "$OUT" "route_$n" 300 python -u tools/route_probe.py --lib "$lib" || exit 1
    echo "$n: $(grep -h 'the rule' "$OUT/route_$n.txt" | head -1 | sed 's/\[.*//')"
  done
done
