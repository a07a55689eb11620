set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_stratify.py tests/test_gpu_candidates.py -x -q --timeout 200 --timeout-method thread -k "dense or strat or fused or Rating or candidates" > gpurun_out/dense_tests.txt 2>&1 || { tail -40 gpurun_out/dense_tests.txt; exit 1; }
tail -2 gpurun_out/dense_tests.txt
timeout -k 10 300 python -u tools/bench_rows.py --only a6,f4 --out gpurun_out/rows_a6.json > gpurun_out/rows_a6.log 2>&1 || { tail -20 gpurun_out/rows_a6.log; exit 1; }
grep -o '"gpu_ms": [0-9.]*\|"frac": [0-9.]*\|"note": "[^"]*"' gpurun_out/rows_a6.json
