set -o pipefail
mkdir -p gpurun_out
bash tools/_ab.sh tools/liblgx_BLOOM3.so tools/liblgx_EPIFIRST.so || exit 1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.txt 2>&1 || exit 1
