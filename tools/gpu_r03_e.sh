#!/bin/bash
# round-3: f32 MFMA interleave -- scoring tests + scoring legs; N=2 rehearsal of the bench (gloo,
# two ranks on one GPU) on the amazon shape and on C4
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_score_f32.py tests/test_gpu_pinned.py tests/test_gpu_stratify.py -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_e.txt 2>&1 || { tail -60 gpurun_out/pytest_e.txt; exit 1; }
tail -3 gpurun_out/pytest_e.txt
timeout -k 10 300 python -u bench.py --no-propagation --no-cpu-baseline > gpurun_out/bench_score_e.json 2> gpurun_out/bench_score_e.err || { tail -20 gpurun_out/bench_score_e.err; exit 1; }
cat gpurun_out/bench_score_e.json
LGX_BENCH_BACKEND=gloo timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --config synth10m --no-scoring --no-cpu-baseline --steps 2 --warmup 1 --extra-steps 2 > gpurun_out/bench_n2_rehearsal.json 2> gpurun_out/bench_n2_rehearsal.err || { tail -30 gpurun_out/bench_n2_rehearsal.err; exit 1; }
head -c 3000 gpurun_out/bench_n2_rehearsal.json; echo
