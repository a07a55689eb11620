#!/bin/bash
# a round's evidence on the final library (tools/gpu_evidence.sh, via gpurun): GPU tests, smoke,
# rocprof (kernel trace + PMC bytes, tools/profile_round.sh) and the
# bench line carrying this build's traffic
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.txt 2>&1 || { tail -40 gpurun_out/pytest_gpu.txt; exit 1; }
tail -2 gpurun_out/pytest_gpu.txt
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.txt 2>&1 || { cat gpurun_out/smoke.txt; exit 1; }
cat gpurun_out/smoke.txt
bash tools/profile_round.sh ${1:-r03} > gpurun_out/profile.txt 2>&1 || { tail -20 gpurun_out/profile.txt; exit 1; }
tail -2 gpurun_out/profile.txt
cat gpurun_out/prof_${1:-r03}/bench_with_traffic.json | head -c 1500
