#!/bin/bash
# round-3: full GPU suite on the f32-LDS build, f4 end to end with component times
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.txt 2>&1 || { tail -60 gpurun_out/pytest_gpu.txt; exit 1; }
tail -3 gpurun_out/pytest_gpu.txt
timeout -k 10 300 python -u tools/f4_e2e.py > gpurun_out/f4_e2e.txt 2>&1 || { tail -20 gpurun_out/f4_e2e.txt; exit 1; }
cat gpurun_out/f4_e2e.txt
