#!/bin/bash
# One GPU step of a gpurun call, bounded and logged (replaces round 5's tools/r05_gpu_*.sh one-offs):
#   bash tools/gpu_step.sh OUTDIR NAME SECONDS command args...
# runs the command under `timeout -k 10 SECONDS`, stdout+stderr into OUTDIR/NAME.txt, prints the
# last lines; a non-zero exit (fault, abort, time limit) is returned, so steps chain with && and
# nothing further runs on the GPU after a failure.
set -o pipefail
OUT=$1; NAME=$2; SECS=$3; shift 3
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 "$SECS" "$@" > "$OUT/$NAME.txt" 2>&1
rc=$?
grep -v amdgpu.ids "$OUT/$NAME.txt" | tail -${GPU_STEP_TAIL:-15}
[ $rc -ne 0 ] && echo "[gpu_step] $NAME failed with exit $rc"
exit $rc
