#!/bin/bash
# round-3: min / max mode + select margin -- their tests, f4 phases and end to end
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_score_f32.py tests/test_gpu_stratify.py tests/test_gpu_candidates.py -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_c.txt 2>&1 || { tail -60 gpurun_out/pytest_c.txt; exit 1; }
tail -3 gpurun_out/pytest_c.txt
timeout -k 10 240 python -u tools/f4_phases.py > gpurun_out/f4_phases.txt 2>&1 || { tail -20 gpurun_out/f4_phases.txt; exit 1; }
cat gpurun_out/f4_phases.txt
timeout -k 10 300 python -u tools/f4_e2e.py > gpurun_out/f4_e2e.txt 2>&1 || { tail -20 gpurun_out/f4_e2e.txt; exit 1; }
cat gpurun_out/f4_e2e.txt
