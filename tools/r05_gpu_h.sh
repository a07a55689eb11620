#!/bin/bash
# round 5, GPU step H: the whole GPU suite with fp32 floors at the evaluation shapes; the route probe
# and the evaluation rows on this build.  The first failure ends the script.
set -o pipefail
OUT=gpurun_out/r05h
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/pytest_gpu.txt 2>&1 \
    || { tail -60 $OUT/pytest_gpu.txt; exit 1; }
tail -2 $OUT/pytest_gpu.txt
timeout -k 10 600 python -u tools/route_probe.py > $OUT/route_probe.txt 2>&1 || { tail -30 $OUT/route_probe.txt; exit 1; }
grep -v amdgpu.ids $OUT/route_probe.txt
timeout -k 10 300 python -u tools/eval_probe.py --f32 > $OUT/eval_probe.txt 2>&1 || { tail -30 $OUT/eval_probe.txt; exit 1; }
grep -v amdgpu.ids $OUT/eval_probe.txt
timeout -k 10 600 python -u tools/bench_rows.py --only eval_c1,eval_c3 --out $OUT/rows_eval.json > $OUT/rows_eval.log 2>&1 || { tail -30 $OUT/rows_eval.log; exit 1; }
python3 -c "
import json
for r in json.load(open('$OUT/rows_eval.json'))['rows']:
    print(r['row'][:50], r['gpu_ms'] if 'gpu_ms' in r else '', r.get('phases_ms'), r['roofline'].get('launch_ms'), r['roofline'].get('frac'), r['roofline'].get('kernel'))
"
