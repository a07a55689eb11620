set -o pipefail
mkdir -p gpurun_out/icache
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc SQC_ICACHE_HITS SQC_ICACHE_MISSES -d $GRAFT_REPO_ROOT/gpurun_out/icache -o ic --output-format csv -- $GRAFT_REPO_ROOT/tools/score_lab 131072 > $GRAFT_REPO_ROOT/gpurun_out/icache/log.txt 2>&1 || { tail -20 $GRAFT_REPO_ROOT/gpurun_out/icache/log.txt; exit 1; }
tail -12 $GRAFT_REPO_ROOT/gpurun_out/icache/log.txt
find $GRAFT_REPO_ROOT/gpurun_out/icache -name "*.csv" | head
