# rocprofv3 kernel stats of the Gowalla-shape BPR epoch row (tools/bench_rows.py f2b), stats only
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
LGX_ROWS_F2B_FUSED_ONLY=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_f2b -o f2b --output-format csv -- python3 -u tools/bench_rows.py --only f2b --reps 2 --out gpurun_out/rows_f2b_prof.json > gpurun_out/prof_f2b.txt 2>&1 || exit 1
find gpurun_out/prof_f2b -type f ! -name "*stats*" -delete
