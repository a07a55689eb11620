#!/bin/bash
# round 5, GPU step AC: the N>1 path on the final build, two ranks on one GPU over gloo, started by
# bench.py itself (no external launcher)
set -o pipefail
OUT=gpurun_out/r05ac
mkdir -p $OUT
export TMPDIR=/tmp
LGX_BENCH_BACKEND=gloo timeout -k 10 900 python -u bench.py --gpus 2 --steps 2 --warmup 1 > $OUT/bench_n2.json 2> $OUT/bench_n2.log || { tail -30 $OUT/bench_n2.log; exit 1; }
python3 -c "
import json
b = json.loads(open('$OUT/bench_n2.json').read().strip().splitlines()[-1])
print(b['n_gpus'], b['process_group'], round(b['value'] / 1e9, 3), 'G edges/s', b['ms_per_step'], 'ms/step')
print('phases', b.get('phases_ms'))
"
