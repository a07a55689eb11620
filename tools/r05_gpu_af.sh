#!/bin/bash
# round 5, GPU step AF: the whole GPU suite and smoke on the final tree
set -o pipefail
OUT=gpurun_out/r05af
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest_gpu.txt 2>&1 || { tail -40 $OUT/pytest_gpu.txt; exit 1; }
tail -2 $OUT/pytest_gpu.txt
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.txt 2>&1 || { cat $OUT/smoke.txt; exit 1; }
grep -v amdgpu.ids $OUT/smoke.txt
