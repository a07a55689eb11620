#!/bin/bash
# round 5, GPU step R: the dense route's chunk size and threshold at the evaluation shapes
set -o pipefail
OUT=gpurun_out/r05r
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 500 python -u tools/chunk_probe.py > $OUT/chunk_probe.txt 2>&1 || { tail -30 $OUT/chunk_probe.txt; exit 1; }
grep -v amdgpu.ids $OUT/chunk_probe.txt
