#!/bin/bash
# round 5, GPU step A (via gpurun): the tests touched by the 8-wave fp32 walk, the exact users' mean
# and the one-FMA label estimate; the evaluation-shape probes and the f4 row on both builds (round-4
# library vs this one, alternating); the evaluation rows; the fp32 world-8 shard probe.  Every GPU
# step has its own time limit; the first failure ends the script.
set -o pipefail
OUT=gpurun_out/r05a
mkdir -p $OUT
NEW=factors_of_serendipity_recommendation_amd/liblgx.so
OLD=tools/_ab/liblgx_r04.so
# bf16 C5 scoring at the bench's 1M users: L2-miss bytes (FETCH_SIZE, its own pass per build) of the
# round-3 final, round-4 final and this build
export TMPDIR=/tmp
for lib in tools/_ab/liblgx_r03.so $OLD $NEW; do
  n=$(basename $lib .so)
  timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "score_topk" --output-format csv \
      -d $OUT/fetch1m_$n -o run -- python3 tools/score_traffic.py --lib $lib --users 1000000 --calls 1 \
      > $OUT/fetch1m_$n.json 2> $OUT/fetch1m_$n.log || { tail -20 $OUT/fetch1m_$n.log; exit 1; }
  python3 tools/fetch_sum.py $OUT/fetch1m_$n 2 >> $OUT/fetch1m_summary.jsonl
  rm -rf $OUT/fetch1m_$n
done
cat $OUT/fetch1m_summary.jsonl
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
    tests/test_gpu_score_f32.py tests/test_gpu_topk_eval.py tests/test_gpu_stratify.py tests/test_gpu_sigmoid.py \
    "tests/test_gpu_parity.py::test_batch_test_both_flags_vs_oracle" \
    "tests/test_gpu_parity.py::test_column_mean_is_numpy_mean_bit_for_bit" \
    tests/test_gpu_pinned.py -k "not full_size and not c3_amazon and not c1_gowalla" \
    > $OUT/pytest.txt 2>&1 || { tail -60 $OUT/pytest.txt; exit 1; }
tail -3 $OUT/pytest.txt
FLOOR=tools/_ab/liblgx_f32floor.so
for rep in 1 2; do
  for lib in $OLD $NEW $FLOOR; do
    echo "== $lib rep $rep" >> $OUT/eval_probe.txt
    timeout -k 10 300 python -u tools/eval_probe.py --f32 --lib $lib >> $OUT/eval_probe.txt 2>&1 || { tail -30 $OUT/eval_probe.txt; exit 1; }
  done
  for lib in $OLD $NEW; do
    timeout -k 10 300 python -u tools/bench_rows.py --only f4 --lib $lib --out $OUT/rows_f4_$(basename $lib .so)_$rep.json \
        >> $OUT/rows_f4.log 2>&1 || { tail -30 $OUT/rows_f4.log; exit 1; }
  done
done
cat $OUT/eval_probe.txt
for lib in $OLD $NEW $FLOOR; do
  echo "== $lib" >> $OUT/order_probe.txt
  timeout -k 10 600 python -u tools/order_probe.py --lib $lib >> $OUT/order_probe.txt 2>&1 || { tail -30 $OUT/order_probe.txt; exit 1; }
done
cat $OUT/order_probe.txt
timeout -k 10 600 python -u tools/bench_rows.py --only eval_c1,eval_c3 --out $OUT/rows_eval.json > $OUT/rows_eval.log 2>&1 || { tail -30 $OUT/rows_eval.log; exit 1; }
timeout -k 10 900 python -u tools/shard_probe.py --dtype f32 > $OUT/shard_probe_world8_f32.json 2> $OUT/shard_probe.log || { tail -30 $OUT/shard_probe.log; exit 1; }
cat $OUT/shard_probe_world8_f32.json
