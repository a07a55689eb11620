#!/bin/bash
# round-3: column-blocked item rows -- tests, then the propagation legs of the bench
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_colblock.py tests/test_gpu_parity.py tests/test_gpu_pinned.py -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_d.txt 2>&1 || { tail -60 gpurun_out/pytest_d.txt; exit 1; }
tail -3 gpurun_out/pytest_d.txt
timeout -k 10 600 python -u bench.py --steps 10 --warmup 3 --no-scoring --no-cpu-baseline > gpurun_out/bench_d.json 2> gpurun_out/bench_d.err || { tail -20 gpurun_out/bench_d.err; exit 1; }
cat gpurun_out/bench_d.json
