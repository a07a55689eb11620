set -o pipefail
mkdir -p gpurun_out
LGX_BENCH_BACKEND=gloo timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --config amazon --no-cpu-baseline --steps 3 --warmup 1 --score-users 20000 --score-items 100000 > gpurun_out/bench_n2_rehearsal.json 2> gpurun_out/bench_n2_rehearsal.err || { tail -30 gpurun_out/bench_n2_rehearsal.err; exit 1; }
grep "\[bench\]" gpurun_out/bench_n2_rehearsal.err | head; head -c 700 gpurun_out/bench_n2_rehearsal.json; echo
timeout -k 10 300 python -u -m pytest tests/test_gpu_distributed.py -x -q --timeout 200 --timeout-method thread > gpurun_out/dist_tests.txt 2>&1 || { tail -30 gpurun_out/dist_tests.txt; exit 1; }
tail -2 gpurun_out/dist_tests.txt
