#!/bin/bash
# round-2 probe 2: gather ceilings by table size; degree-ordered numbering and nt cold gathers
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 120 tools/fetch_calib 2 > gpurun_out/calib_sweep.txt 2>&1 || exit 1
cat gpurun_out/calib_sweep.txt
timeout -k 10 300 python -u tools/renum_probe.py > gpurun_out/renum_default.txt 2>&1 || exit 1
cat gpurun_out/renum_default.txt
timeout -k 10 300 python -u tools/renum_probe.py --lib tools/liblgx_ntcold.so --cuts 16384:16384,131072:131072,1048576:262144,0:0 > gpurun_out/renum_ntcold.txt 2>&1 || exit 1
cat gpurun_out/renum_ntcold.txt
