#!/bin/bash
# round 5, GPU step E: fp32 plan (4 vs 8 waves, split penalty) and the dense route -- tests, the route
# probe at several thresholds, the evaluation rows.  The first failure ends the script.
set -o pipefail
OUT=gpurun_out/r05e
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_topk_eval.py \
    tests/test_gpu_score_f32.py tests/test_gpu_pinned.py tests/test_gpu_parity.py \
    -k "not full_size and not c3_amazon and not eigenvector" > $OUT/pytest.txt 2>&1 || { tail -60 $OUT/pytest.txt; exit 1; }
tail -2 $OUT/pytest.txt
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
