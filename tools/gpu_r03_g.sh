#!/bin/bash
# round-3: 12 deferred slots in the bf16 LDS kernel -- scoring tests, then the scoring legs
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests/test_gpu_pinned.py tests/test_gpu_parity.py tests/test_gpu_topk_eval.py tests/test_gpu_score_f32.py tests/test_gpu_stratify.py tests/test_gpu_candidates.py -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_g.txt 2>&1 || { tail -60 gpurun_out/pytest_g.txt; exit 1; }
tail -3 gpurun_out/pytest_g.txt
timeout -k 10 300 python -u bench.py --no-propagation --no-cpu-baseline > gpurun_out/bench_score_g.json 2> gpurun_out/bench_score_g.err || { tail -20 gpurun_out/bench_score_g.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/bench_score_g.json')); [print(k, d[k]['ms_per_step'], d[k]['roofline']['frac']) for k in ('scoring','scoring_bf16')]"
