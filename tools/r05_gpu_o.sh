#!/bin/bash
# round 5, GPU step O: the dense-score walk with staggered wave halves (tools/_ab/liblgx_dst.so:
# late waves store tile t-1 after the barrier, early waves stage the tiles; 2 waves per SIMD above
# 8 chunks) against the round's evidence build: bench_rows a6 (+a9), alternating.
set -o pipefail
OUT=gpurun_out/r05o
mkdir -p $OUT
export TMPDIR=/tmp
for rep in 1 2; do
  for lib in tools/_ab/liblgx_r05base.so tools/_ab/liblgx_dst.so; do
    n=$(basename $lib .so)_$rep
    timeout -k 10 300 python -u tools/bench_rows.py --only a6 --lib $lib --out $OUT/$n.json > $OUT/$n.log 2>&1 || { tail -30 $OUT/$n.log; exit 1; }
  done
done
python - <<'PY'
import json, glob
for f in sorted(glob.glob("gpurun_out/r05o/*.json")):
    d = json.load(open(f))
    print(f.split("/")[-1], " | ".join(f"{r['row'][:40]}: {r['gpu_ms']:.3f} ms" + (f" ({r['note'].split('raw scores')[1][:40]})" if 'raw scores' in r.get('note','') else "") for r in d["rows"]))
PY
