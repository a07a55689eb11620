#!/bin/bash
# deferred-slot depth and ring depth A/B on the C5 shape (131072 users x 1M items, d=256, top-20)
set -o pipefail
mkdir -p gpurun_out
out=gpurun_out/lab_pend.txt
rm -f $out
for v in ${LAB_VARIANTS:-score_lab score_lab_nb2 score_lab_p8 score_lab_p12}; do
  echo "== $v" >> $out
  timeout -k 10 200 tools/$v 131072 >> $out 2>&1 || { cat $out; exit 1; }
  LAB_STAGES=16384,32768,65536,131072,262144,524288 timeout -k 10 200 tools/$v 131072 >> $out 2>&1 || { cat $out; exit 1; }
done
cat $out
