#!/bin/bash
# round-3: the new / changed GPU tests first, then the full GPU suite, then the default bench line
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_stratify.py tests/test_gpu_pinned.py tests/test_gpu_distributed.py -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_new.txt 2>&1 || { tail -60 gpurun_out/pytest_new.txt; exit 1; }
tail -3 gpurun_out/pytest_new.txt
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.txt 2>&1 || { tail -40 gpurun_out/pytest_gpu.txt; exit 1; }
tail -3 gpurun_out/pytest_gpu.txt
timeout -k 10 600 python -u bench.py --steps 20 --warmup 5 > gpurun_out/bench_r03a.json 2> gpurun_out/bench_r03a.err || { tail -20 gpurun_out/bench_r03a.err; exit 1; }
cat gpurun_out/bench_r03a.json
