#!/bin/bash
# round 5: every SURVEY §8 row not in bench.py, on the final library (tools/bench_rows.py)
set -o pipefail
OUT=gpurun_out/r05_evidence
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 1000 python -u tools/bench_rows.py --out $OUT/rows.json > $OUT/rows.log 2>&1 || { tail -30 $OUT/rows.log; exit 1; }
python3 -c "
import json
for r in json.load(open('$OUT/rows.json'))['rows']:
    print(r['row'][:70], '|', round(r.get('gpu_ms', 0), 3), '|', r['roofline'].get('frac'))
"
