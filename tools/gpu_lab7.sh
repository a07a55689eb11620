set -o pipefail
mkdir -p gpurun_out
rm -f gpurun_out/lab7.txt
timeout -k 10 200 tools/score_lab_m3 131072 >> gpurun_out/lab7.txt 2>&1 || { cat gpurun_out/lab7.txt; exit 1; }
cat gpurun_out/lab7.txt
