#!/bin/bash
# round 5, GPU step B (via gpurun): the whole GPU suite on this build; evaluation-shape probes (round-4
# library vs this one); the fold-out / users'-mean probe; the bf16 C5 traffic and time of this build
# against the dynamic XCD rotation variant.  Every GPU step has its own time limit; the first failure
# ends the script.
set -o pipefail
OUT=gpurun_out/r05b
mkdir -p $OUT
NEW=factors_of_serendipity_recommendation_amd/liblgx.so
OLD=tools/_ab/liblgx_r04.so
DYN=tools/_ab/liblgx_dyn.so
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
    > $OUT/pytest_gpu.txt 2>&1 || { tail -60 $OUT/pytest_gpu.txt; exit 1; }
tail -2 $OUT/pytest_gpu.txt
for lib in $OLD $NEW; do
  echo "== $lib" >> $OUT/eval_probe.txt
  timeout -k 10 300 python -u tools/eval_probe.py --f32 --lib $lib >> $OUT/eval_probe.txt 2>&1 || { tail -30 $OUT/eval_probe.txt; exit 1; }
  echo "== $lib" >> $OUT/order_probe.txt
  timeout -k 10 600 python -u tools/order_probe.py --lib $lib >> $OUT/order_probe.txt 2>&1 || { tail -30 $OUT/order_probe.txt; exit 1; }
done
cat $OUT/eval_probe.txt $OUT/order_probe.txt
timeout -k 10 300 python -u tools/foldout_probe.py > $OUT/foldout_probe.txt 2>&1 || { tail -30 $OUT/foldout_probe.txt; exit 1; }
cat $OUT/foldout_probe.txt
for lib in $NEW $DYN; do
  n=$(basename $lib .so)
  timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "score_topk" --output-format csv \
      -d $OUT/fetch1m_$n -o run -- python3 tools/score_traffic.py --lib $lib --users 1000000 --calls 1 \
      > $OUT/fetch1m_$n.json 2> $OUT/fetch1m_$n.log || { tail -20 $OUT/fetch1m_$n.log; exit 1; }
  python3 tools/fetch_sum.py $OUT/fetch1m_$n 2 >> $OUT/fetch1m_summary.jsonl
  rm -rf $OUT/fetch1m_$n
done
for rep in 1 2; do
  for lib in $NEW $DYN; do
    timeout -k 10 180 python3 tools/score_traffic.py --lib $lib --users 1000000 --calls 2 >> $OUT/score_ab.jsonl 2>> $OUT/score_ab.log \
        || { tail -20 $OUT/score_ab.log; exit 1; }
  done
done
cat $OUT/fetch1m_summary.jsonl $OUT/score_ab.jsonl
timeout -k 10 600 python -u tools/bench_rows.py --only eval_c1,eval_c3 --out $OUT/rows_eval.json > $OUT/rows_eval.log 2>&1 || { tail -30 $OUT/rows_eval.log; exit 1; }
python3 -c "
import json
for r in json.load(open('$OUT/rows_eval.json'))['rows']:
    print(r['row'][:50], r.get('phases_ms'), r['roofline'].get('launch_ms'), r['roofline'].get('frac'))
"
