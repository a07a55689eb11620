set -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 python -u tools/spmm_probe.py --blocks "" --hot 2048,8192,32768 > gpurun_out/probe_hot.txt 2>&1
