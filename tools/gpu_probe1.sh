#!/bin/bash
# round-2 probe 1: GPU tests, FETCH_SIZE calibration, SpMM phase split
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.txt 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/pytest_gpu.txt; exit 1; }
tail -3 gpurun_out/pytest_gpu.txt
bash tools/fetch_calib.sh r02 || exit 1
cat gpurun_out/calib_r02/timing.txt
timeout -k 10 400 python -u tools/spmm_probe.py --phase --blocks 4 --hot 16384,131072 > gpurun_out/spmm_probe_phase.txt 2>&1 || exit 1
cat gpurun_out/spmm_probe_phase.txt
