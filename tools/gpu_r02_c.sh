#!/bin/bash
# round-2 run C: C4 world=8 shard probe on one GPU
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u tools/shard_probe.py > gpurun_out/shard_probe.json 2> gpurun_out/shard_probe.err || { tail -20 gpurun_out/shard_probe.err; exit 1; }
cat gpurun_out/shard_probe.err gpurun_out/shard_probe.json
