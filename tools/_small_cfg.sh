# propagation bench lines for BASELINE configs[0..2] (Gowalla / ML-1M / Amazon-book shapes) with the CPU baseline beside each
set -o pipefail
mkdir -p gpurun_out
: > gpurun_out/bench_small_cpu.json
for C in gowalla ml1m amazon; do
timeout -k 10 300 python -u bench.py --config $C --no-scoring --steps 20 --warmup 5 >> gpurun_out/bench_small_cpu.json 2>> gpurun_out/bench_small_cpu.log || exit 1
done
