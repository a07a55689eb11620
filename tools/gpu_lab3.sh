set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 tools/score_lab 131072 > gpurun_out/lab3.txt 2>&1 || { cat gpurun_out/lab3.txt; exit 1; }
cat gpurun_out/lab3.txt
