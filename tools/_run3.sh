set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q -k "score or topk or kat" --timeout 200 --timeout-method thread > gpurun_out/pt3.txt 2>&1 || exit 1
ABL_B=131072,1000000 timeout -k 10 300 python -u tools/score_ablation.py > gpurun_out/stag.txt 2>&1 || exit 1
LGX_SCORE_NOSTAGGER=1 ABL_B=131072,1000000 timeout -k 10 300 python -u tools/score_ablation.py > gpurun_out/nostag.txt 2>&1 || exit 1
timeout -k 10 400 python -u tools/spmm_probe.py > gpurun_out/probe_base.txt 2>&1 || exit 1
timeout -k 10 400 python -u tools/spmm_probe.py --lib tools/liblgx_nt.so --blocks 8 > gpurun_out/probe_nt.txt 2>&1
