#!/bin/bash
# A/B of two liblgx.so builds on the evaluation shapes (tools/route_probe.py: the evaluator's route at
# the Gowalla / Amazon-book shapes) and the fp32 / bf16 C5 scoring shapes (tools/score_probe.py), alternating
# builds, two rounds; then the fp32 scoring tests on build B.
#   bash tools/ab_eval.sh OUTDIR libA libB [score users]
set -o pipefail
OUT=$1; A=$2; B=$3; SU=${4:-262144}
for rep in 1 2; do
  for lib in "$A" "$B"; do
    n=$(basename "$lib" .so)_$rep
    GPU_STEP_TAIL=3 bash tools/gpu_step.sh "$OUT" "route_$n" 300 python -u tools/route_probe.py --lib "$lib" || exit 1
    grep -h "the rule" "$OUT/route_$n.txt"
    GPU_STEP_TAIL=1 bash tools/gpu_step.sh "$OUT" "score_$n" 300 python -u tools/score_probe.py "$SU" f32 --lib "$lib" || exit 1
    GPU_STEP_TAIL=1 bash tools/gpu_step.sh "$OUT" "score16_$n" 300 python -u tools/score_probe.py 262144 bf16 --lib "$lib" || exit 1
  done
done
