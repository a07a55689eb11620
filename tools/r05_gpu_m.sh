#!/bin/bash
# round 5, GPU step M: every test user through the dense route at the evaluation shapes
set -o pipefail
OUT=gpurun_out/r05m
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python -u tools/dense_probe.py > $OUT/dense_probe.txt 2>&1 || { tail -30 $OUT/dense_probe.txt; exit 1; }
grep -v amdgpu.ids $OUT/dense_probe.txt
