set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_training.py tests/test_gpu_stratify.py -x -v --timeout 200 --timeout-method thread > gpurun_out/train_tests.txt 2>&1 || { tail -40 gpurun_out/train_tests.txt; exit 1; }
tail -3 gpurun_out/train_tests.txt
timeout -k 10 300 python -u tools/f2b_diag.py > gpurun_out/f2b_diag.txt 2>&1 || { cat gpurun_out/f2b_diag.txt; exit 1; }
cat gpurun_out/f2b_diag.txt
timeout -k 10 300 python -u tools/bench_rows.py --only f4,f2b --out gpurun_out/rows_f.json > gpurun_out/rows_f.log 2>&1 || { tail -20 gpurun_out/rows_f.log; exit 1; }
grep -o '"note": "[^"]*"' gpurun_out/rows_f.json; grep -o '"gpu_ms": [0-9.]*' gpurun_out/rows_f.json
