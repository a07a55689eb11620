set -o pipefail
mkdir -p gpurun_out
rm -f gpurun_out/ab.txt
for r in 1 2; do
for b in score_lab score_lab_ref; do
  echo "== $b" >> gpurun_out/ab.txt
  timeout -k 10 200 tools/$b 131072 >> gpurun_out/ab.txt 2>&1 || { cat gpurun_out/ab.txt; exit 1; }
done
done
cat gpurun_out/ab.txt
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_pinned.py tests/test_gpu_topk_eval.py -x -q --timeout 200 --timeout-method thread -k "score or topk or kat or Test or procedure or full_sweep" > gpurun_out/score_tests.txt 2>&1 || { tail -40 gpurun_out/score_tests.txt; exit 1; }
tail -2 gpurun_out/score_tests.txt
