#!/bin/bash
# round 5, GPU step V: the column mean with two blocks in flight and 16-B LDS reads
# (tools/_ab/liblgx_cm.so) against the final evidence build (tools/_ab/liblgx_r05c.so): the
# batch_test rows (a8 phases), alternating; then the parity tests on the new build.
set -o pipefail
OUT=gpurun_out/r05v
mkdir -p $OUT
export TMPDIR=/tmp
for rep in 1 2; do
  for lib in tools/_ab/liblgx_r05c.so tools/_ab/liblgx_cm.so; do
    n=$(basename $lib .so)_$rep
    timeout -k 10 300 python -u tools/bench_rows.py --only eval_c1,eval_c3 --lib $lib --out $OUT/$n.json > $OUT/$n.log 2>&1 || { tail -30 $OUT/$n.log; exit 1; }
  done
done
python3 - <<'PY'
import json, glob
for f in sorted(glob.glob("gpurun_out/r05v/*.json")):
    for r in json.load(open(f))["rows"]:
        if r["row"].startswith("a8"):
            print(f.split("/")[-1], r["row"][:40], round(r["gpu_ms"], 3), {k: round(v, 3) for k, v in r["phases_ms"].items()})
PY
timeout -k 10 200 python -u tools/cm_probe.py --lib tools/_ab/liblgx_cm.so > $OUT/cm_probe.txt 2>&1 || { tail -30 $OUT/cm_probe.txt; exit 1; }
grep -v amdgpu.ids $OUT/cm_probe.txt
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread > $OUT/pytest.txt 2>&1 || { tail -30 $OUT/pytest.txt; exit 1; }
tail -2 $OUT/pytest.txt
