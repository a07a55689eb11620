#!/bin/bash
# FETCH_SIZE calibration on the GPU box (gpurun), from the repo root:
#   bash tools/fetch_calib.sh r02      -> gpurun_out/calib_r02/{timing.txt, fetch/, hitmiss/}
# then python tools/calib_summary.py r02 -> profiles/r02_fetch_calibration.json
set -eo pipefail
TAG=${1:?usage: tools/fetch_calib.sh <tag>}
ROOT=$(pwd)
OUT=$ROOT/gpurun_out/calib_$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
BIN=$ROOT/tools/fetch_calib
timeout -k 10 120 "$BIN" 3 > "$OUT/timing.txt"
cd /tmp
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/fetch" -o run -- "$BIN" 1 > /dev/null 2> "$OUT/fetch.log"
timeout -s KILL 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --output-format csv -d "$OUT/hitmiss" -o run -- "$BIN" 1 > /dev/null 2> "$OUT/hitmiss.log"
echo "[calib] done"
