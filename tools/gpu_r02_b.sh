#!/bin/bash
# round-2 run B: FETCH_SIZE calibration (with the gather sweep), degree-renumbering probe, PMC profile
set -o pipefail
mkdir -p gpurun_out
bash tools/fetch_calib.sh r02 || exit 1
timeout -k 10 400 python -u tools/renum_probe.py > gpurun_out/renum_default.txt 2>&1 || { cat gpurun_out/renum_default.txt; exit 1; }
cat gpurun_out/renum_default.txt
bash tools/profile_round.sh r02 > gpurun_out/profile.txt 2>&1 || { tail -20 gpurun_out/profile.txt; exit 1; }
echo "[r02b] done"
