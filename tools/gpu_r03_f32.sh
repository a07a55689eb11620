#!/bin/bash
# round-3: the fp32 LDS scoring kernel -- its tests, then the scoring legs of the bench
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_score_f32.py tests/test_gpu_pinned.py -k "f32 or c5 or fp32" -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_f32.txt 2>&1 || { tail -60 gpurun_out/pytest_f32.txt; exit 1; }
tail -3 gpurun_out/pytest_f32.txt
timeout -k 10 300 python -u bench.py --no-propagation --no-cpu-baseline > gpurun_out/bench_score.json 2> gpurun_out/bench_score.err || { tail -20 gpurun_out/bench_score.err; exit 1; }
cat gpurun_out/bench_score.json
timeout -k 10 300 python -u tools/f4_e2e.py > gpurun_out/f4_e2e.txt 2>&1 || { tail -20 gpurun_out/f4_e2e.txt; exit 1; }
cat gpurun_out/f4_e2e.txt
