#!/bin/bash
# Collect a round's rocprofv3 evidence for the default bench workload.  Run ON THE GPU BOX from the
# repo root (gpurun); the summary lands in gpurun_out/prof_<tag>/summary/ (copy it into profiles/)
#   1. plain bench (the JSON line, with CPU baselines)
#   2. --kernel-trace --stats under the bench (per-kernel durations)
#   3. --pmc FETCH_SIZE and 4. --pmc WRITE_SIZE, separate passes (MI355X_MICROARCH.md HBM recipe)
#   5. --pmc MFMA busy / SQ busy cycles of the bf16 scoring walk (its own pass)
#   6. plain bench again, with the PMC bytes of this build in its line
set -eo pipefail
TAG=${1:?usage: tools/profile_round.sh <tag, e.g. r01>}
ROOT=$(pwd)
OUT=$ROOT/gpurun_out/prof_$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
ARGS="--steps 3 --warmup 1 --extra-steps 2 --score-steps 1 --no-cpu-baseline"
KRE='spmm_segments|spmm_fixup|score_topk_bf16_lds|score_topk_f32_lds|score_topk_finalize'
echo "[profile] plain bench"
timeout -k 10 900 python3 "$ROOT/bench.py" > "$OUT/bench.json" 2> "$OUT/bench.log"
cd /tmp
echo "[profile] kernel trace"
timeout -k 10 900 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o run -- \
    python3 "$ROOT/bench.py" $ARGS > "$OUT/bench_under_rocprof.json" 2> "$OUT/trace.log"
echo "[profile] FETCH_SIZE"
timeout -k 10 900 rocprofv3 --pmc FETCH_SIZE --output-format csv --kernel-include-regex "$KRE" -d "$OUT/fetch" -o run -- \
    python3 "$ROOT/bench.py" $ARGS > /dev/null 2> "$OUT/fetch.log"
echo "[profile] WRITE_SIZE"
timeout -k 10 900 rocprofv3 --pmc WRITE_SIZE --output-format csv --kernel-include-regex "$KRE" -d "$OUT/write" -o run -- \
    python3 "$ROOT/bench.py" $ARGS > /dev/null 2> "$OUT/write.log"
echo "[profile] MFMA busy of the bf16 scoring walk"
timeout -k 10 600 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv \
    --kernel-include-regex score_topk_bf16_lds -d "$OUT/mfma" -o run -- \
    python3 "$ROOT/bench.py" --no-propagation --no-cpu-baseline --score-steps 1 --score-f32-users 16384 \
    > /dev/null 2> "$OUT/mfma.log"
cd "$ROOT"
python3 tools/pmc_summary.py "$TAG" --src "$OUT" --dst "$OUT/summary" > /dev/null
python3 tools/mfma_busy.py "$OUT/mfma" > "$OUT/summary/${TAG}_scoring_pmc_mfma.txt"
rm -rf "$OUT/trace" "$OUT/fetch" "$OUT/write" "$OUT/mfma"   # raw rocprof output exceeds what gpurun copies back
# 6. the plain bench again, now reading this build's PMC bytes (bench.py takes them from profiles/)
cp "$OUT/summary/${TAG}_synth10m_pmc_traffic.json" "$ROOT/profiles/"
echo "[profile] plain bench with this build's PMC traffic"
timeout -k 10 900 python3 "$ROOT/bench.py" > "$OUT/bench_with_traffic.json" 2> "$OUT/bench_with_traffic.log"
echo "[profile] done"
