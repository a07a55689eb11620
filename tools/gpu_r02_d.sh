#!/bin/bash
# round-2 run D: scoring DMA-wave lab, full GPU tests, default bench line
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 tools/score_lab 131072 > gpurun_out/lab8.txt 2>&1 || { cat gpurun_out/lab8.txt; exit 1; }
cat gpurun_out/lab8.txt
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.txt 2>&1 || { tail -40 gpurun_out/pytest_gpu.txt; exit 1; }
tail -3 gpurun_out/pytest_gpu.txt
timeout -k 10 600 python -u bench.py > gpurun_out/bench_r02.json 2> gpurun_out/bench_r02.err || { tail -20 gpurun_out/bench_r02.err; exit 1; }
cat gpurun_out/bench_r02.json
