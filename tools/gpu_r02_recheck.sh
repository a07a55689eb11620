#!/bin/bash
# round-2 re-entry: the rebuilt tree's GPU tests, smoke and default bench line
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.txt 2>&1 || { tail -40 gpurun_out/pytest_gpu.txt; exit 1; }
tail -2 gpurun_out/pytest_gpu.txt
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.txt 2>&1 || { cat gpurun_out/smoke.txt; exit 1; }
cat gpurun_out/smoke.txt
timeout -k 10 600 python -u bench.py > gpurun_out/bench_r02.json 2> gpurun_out/bench_r02.err || { tail -20 gpurun_out/bench_r02.err; exit 1; }
cat gpurun_out/bench_r02.json
