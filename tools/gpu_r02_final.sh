#!/bin/bash
# round-2 final GPU evidence: GPU tests, smoke, N>1 bench rehearsal (gloo, 2 ranks on one GPU),
# rocprof (bench + PMC traffic), the §8 rows
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.txt 2>&1 || { tail -40 gpurun_out/pytest_gpu.txt; exit 1; }
tail -2 gpurun_out/pytest_gpu.txt
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.txt 2>&1 || { cat gpurun_out/smoke.txt; exit 1; }
cat gpurun_out/smoke.txt
LGX_BENCH_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --config amazon --no-scoring --no-cpu-baseline --no-fp32 --steps 3 --warmup 1 > gpurun_out/bench_n2_rehearsal.json 2> gpurun_out/bench_n2_rehearsal.err || { tail -30 gpurun_out/bench_n2_rehearsal.err; exit 1; }
head -c 600 gpurun_out/bench_n2_rehearsal.json; echo
bash tools/profile_round.sh r02 > gpurun_out/profile.txt 2>&1 || { tail -20 gpurun_out/profile.txt; exit 1; }
tail -2 gpurun_out/profile.txt
timeout -k 10 900 python -u tools/bench_rows.py --out gpurun_out/rows.json > gpurun_out/rows.log 2>&1 || { tail -20 gpurun_out/rows.log; exit 1; }
tail -2 gpurun_out/rows.log
