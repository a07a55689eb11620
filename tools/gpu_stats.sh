set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 tools/score_stats 131072 1 > gpurun_out/stats.txt 2>&1 || { cat gpurun_out/stats.txt; exit 1; }
cat gpurun_out/stats.txt
timeout -k 10 300 tools/score_lab 131072 > gpurun_out/lab.txt 2>&1 || { cat gpurun_out/lab.txt; exit 1; }
cat gpurun_out/lab.txt
