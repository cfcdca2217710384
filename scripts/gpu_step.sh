#!/bin/bash
# One GPU step on the gpurun box: `scripts/gpu_step.sh NAME SECONDS CMD...` runs CMD under
# `timeout -k 10 SECONDS` with its output in gpurun_out/NAME.log and a heartbeat line in
# gpurun_out/NAME.hb every 30 s (so a long, quiet step is not taken for a hung one).
# Exits with CMD's status; chain steps with && so nothing runs after a failed one.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
name=$1; secs=$2; shift 2
( while sleep 30; do date +%T >> "gpurun_out/$name.hb"; done ) &
hb=$!
timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1
rc=$?
kill $hb 2>/dev/null
echo "[gpu_step] $name rc=$rc"
tail -n 5 "gpurun_out/$name.log"
exit $rc
