#!/bin/bash
# round 5, GPU step P: f4's label walk (strat_label_lds) with staggered wave halves
# (tools/_ab/liblgx_lst.so) against the round's evidence build: bench_rows f4, alternating; then the
# stratification tests on the new build.
set -o pipefail
OUT=gpurun_out/r05p
mkdir -p $OUT
export TMPDIR=/tmp
for rep in 1 2; do
  for lib in tools/_ab/liblgx_r05base.so tools/_ab/liblgx_lst.so; do
    n=$(basename $lib .so)_$rep
    timeout -k 10 300 python -u tools/bench_rows.py --only f4 --lib $lib --out $OUT/$n.json > $OUT/$n.log 2>&1 || { tail -30 $OUT/$n.log; exit 1; }
  done
done
python - <<'PY'
import json, glob
for f in sorted(glob.glob("gpurun_out/r05p/*.json")):
    d = json.load(open(f))
    for r in d["rows"]:
        print(f.split("/")[-1], f"{r['gpu_ms']:.3f} ms |", r.get("note", "")[:200])
PY
timeout -k 10 600 python -u -m pytest tests/test_gpu_stratify.py -x -q --timeout 300 --timeout-method thread > $OUT/pytest.txt 2>&1 || { tail -30 $OUT/pytest.txt; exit 1; }
tail -3 $OUT/pytest.txt
