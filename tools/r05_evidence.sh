#!/bin/bash
# round 5's evidence on the final library (via gpurun): the whole GPU suite, smoke, rocprof (kernel
# trace + PMC bytes of the bench workload: tools/profile_round.sh), the bench line carrying this
# build's traffic, and the per-row measurements (tools/bench_rows.py).  The first failure ends it.
set -o pipefail
OUT=gpurun_out/r05_evidence
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/pytest_gpu.txt 2>&1 \
    || { tail -40 $OUT/pytest_gpu.txt; exit 1; }
tail -2 $OUT/pytest_gpu.txt
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.txt 2>&1 || { cat $OUT/smoke.txt; exit 1; }
cat $OUT/smoke.txt
bash tools/profile_round.sh r05 > $OUT/profile.txt 2>&1 || { tail -20 $OUT/profile.txt; exit 1; }
tail -2 $OUT/profile.txt
head -c 1500 gpurun_out/prof_r05/bench_with_traffic.json
