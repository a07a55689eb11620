#!/bin/bash
# round 5, GPU step C (via gpurun): fold-out / evaluator tests after the streamed truth lists; where
# the evaluation-shape top-k spends its time on propagated tables (mask_probe); the fold-out probe;
# the evaluation rows; the N=2 bench rehearsal started WITHOUT an external launcher (bench.py spawns
# its two ranks; gloo, both on this one GPU).  The first failure ends the script.
set -o pipefail
OUT=gpurun_out/r05c
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_topk_eval.py \
    tests/test_gpu_parity.py -k "foldout or batch_test or column_mean or kat or procedure" \
    > $OUT/pytest.txt 2>&1 || { tail -60 $OUT/pytest.txt; exit 1; }
tail -2 $OUT/pytest.txt
timeout -k 10 300 python -u tools/foldout_probe.py > $OUT/foldout_probe.txt 2>&1 || { tail -30 $OUT/foldout_probe.txt; exit 1; }
cat $OUT/foldout_probe.txt
timeout -k 10 600 python -u tools/mask_probe.py > $OUT/mask_probe.txt 2>&1 || { tail -30 $OUT/mask_probe.txt; exit 1; }
cat $OUT/mask_probe.txt
timeout -k 10 600 python -u tools/bench_rows.py --only eval_c1,eval_c3 --out $OUT/rows_eval.json > $OUT/rows_eval.log 2>&1 || { tail -30 $OUT/rows_eval.log; exit 1; }
python3 -c "
import json
for r in json.load(open('$OUT/rows_eval.json'))['rows']:
    print(r['row'][:50], r['gpu_ms'] if 'gpu_ms' in r else '', r.get('phases_ms'), r['roofline'].get('launch_ms'), r['roofline'].get('frac'))
"
LGX_BENCH_BACKEND=gloo timeout -k 10 900 python -u bench.py --gpus 2 --steps 2 --warmup 1 --extra-steps 1 --score-steps 1 \
    --no-cpu-baseline > $OUT/bench_n2_gloo_selflaunch.json 2> $OUT/bench_n2_gloo_selflaunch.log || { tail -40 $OUT/bench_n2_gloo_selflaunch.log; exit 1; }
cat $OUT/bench_n2_gloo_selflaunch.json
