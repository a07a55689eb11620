#!/bin/bash
# round 5, GPU step D: the evaluator's dense route for long masks -- tests, then the evaluation rows.
set -o pipefail
OUT=gpurun_out/r05d
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_topk_eval.py \
    tests/test_gpu_parity.py -k "foldout or batch_test or column_mean or kat or procedure or dropin" \
    > $OUT/pytest.txt 2>&1 || { tail -60 $OUT/pytest.txt; exit 1; }
tail -2 $OUT/pytest.txt
timeout -k 10 600 python -u tools/bench_rows.py --only eval_c1,eval_c3 --out $OUT/rows_eval.json > $OUT/rows_eval.log 2>&1 || { tail -30 $OUT/rows_eval.log; exit 1; }
python3 -c "
import json
for r in json.load(open('$OUT/rows_eval.json'))['rows']:
    print(r['row'][:50], r['gpu_ms'] if 'gpu_ms' in r else '', r.get('phases_ms'), r['roofline'].get('launch_ms'), r['roofline'].get('frac'), r['roofline'].get('kernel'))
"
