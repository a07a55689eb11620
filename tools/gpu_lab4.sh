set -o pipefail
mkdir -p gpurun_out
for b in score_lab score_lab_m1 score_lab_m2; do
  timeout -k 10 200 tools/$b 131072 >> gpurun_out/lab4.txt 2>&1 || { cat gpurun_out/lab4.txt; exit 1; }
done
cat gpurun_out/lab4.txt
