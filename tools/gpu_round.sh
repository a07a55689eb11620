# Round-end GPU check on the box (gpurun): GPU tests, smoke, rocprof profile of the bench
#   gpurun --timeout 1200 -- bash tools/gpu_round.sh
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.txt 2>&1 || exit 1
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.txt 2>&1 || exit 1
bash tools/profile_round.sh r01 > gpurun_out/profile.txt 2>&1 || exit 1
