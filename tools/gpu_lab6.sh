set -o pipefail
mkdir -p gpurun_out
rm -f gpurun_out/lab6.txt
for b in score_lab_m1 score_lab_m2; do
  timeout -k 10 200 tools/$b 131072 >> gpurun_out/lab6.txt 2>&1 || { cat gpurun_out/lab6.txt; exit 1; }
done
timeout -k 10 200 tools/score_lab 1000000 >> gpurun_out/lab6.txt 2>&1 || { cat gpurun_out/lab6.txt; exit 1; }
cat gpurun_out/lab6.txt
