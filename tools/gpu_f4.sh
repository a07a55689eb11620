set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_stratify.py -x -q --timeout 200 --timeout-method thread > gpurun_out/strat_tests.txt 2>&1 || { tail -40 gpurun_out/strat_tests.txt; exit 1; }
tail -2 gpurun_out/strat_tests.txt
timeout -k 10 300 python -u tools/bench_rows.py --only f4 --out gpurun_out/rows_f4.json > gpurun_out/rows_f4.log 2>&1 || { tail -20 gpurun_out/rows_f4.log; exit 1; }
cat gpurun_out/rows_f4.json
