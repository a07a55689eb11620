#!/bin/bash
# round-2 GPU run A: full GPU tests, calibration (timing + PMC), bench line, rocprof profile
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.txt 2>&1 || { tail -40 gpurun_out/pytest_gpu.txt; exit 1; }
tail -3 gpurun_out/pytest_gpu.txt
bash tools/fetch_calib.sh r02 || exit 1
python tools/calib_summary.py r02 > /dev/null || exit 1
timeout -k 10 600 python -u bench.py > gpurun_out/bench_r02.json 2> gpurun_out/bench_r02.err || { tail -20 gpurun_out/bench_r02.err; exit 1; }
cat gpurun_out/bench_r02.json
bash tools/profile_round.sh r02 > gpurun_out/profile.txt 2>&1 || { tail -20 gpurun_out/profile.txt; exit 1; }
echo "[round2a] done"
