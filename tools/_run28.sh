set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_training.py -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_train.txt 2>&1 || exit 1
timeout -k 10 300 python -u tools/bench_rows.py --only f2b --out gpurun_out/rows_f2b_fused.json > gpurun_out/rows_f2b_fused.txt 2>&1 || exit 1
