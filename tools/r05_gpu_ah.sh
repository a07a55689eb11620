#!/bin/bash
# round 5, GPU step AH: the dense-route threshold at the floor while the fused walk leaves CUs idle:
# evaluator tests, route_probe, evaluation rows
set -o pipefail
OUT=gpurun_out/r05ah
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_topk_eval.py tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread > $OUT/pytest.txt 2>&1 || { tail -40 $OUT/pytest.txt; exit 1; }
tail -2 $OUT/pytest.txt
timeout -k 10 600 python -u tools/bench_rows.py --only eval_c1,eval_c3 --out $OUT/rows_eval.json > $OUT/rows_eval.log 2>&1 || { tail -30 $OUT/rows_eval.log; exit 1; }
python3 -c "
import json
for r in json.load(open('$OUT/rows_eval.json'))['rows']:
    print(r['row'][:70], '|', round(r.get('gpu_ms', 0), 3), '|', r['roofline'].get('kernel', '')[-90:], '|', {k: round(v, 3) for k, v in r.get('phases_ms', {}).items()})
"
