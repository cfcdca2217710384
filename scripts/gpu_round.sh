#!/bin/bash
# One GPU-box session: smoke -> gpu tests -> bench -> rocprofv3 kernel trace.
# Each GPU step has its own time limit; a crash/timeout (rc not 0/1) stops the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
MODE=${1:-full}
step() {  # name timeout cmd...
    local name=$1 t=$2; shift 2
    echo "== $name: $*"
    timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
    local rc=$?
    echo "== $name rc=$rc"
    tail -n 4 "gpurun_out/$name.log" | cut -c1-1500
    return $rc
}
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()" || exit $?
step pytest_gpu 900 python -m pytest tests -m gpu -q -x -p no:cacheprovider
rc=$?; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
[ "$MODE" = "tests" ] && exit 0
step bench 600 python bench.py --steps 10 --warmup 2 || exit $?
[ "$MODE" = "bench" ] && exit 0
step rocprof 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- \
    python bench.py --steps 5 --warmup 1 --no-cpu-baseline || exit $?
find gpurun_out/prof -name "*kernel_stats.csv" -exec cp {} gpurun_out/kernel_stats.csv \;
cat gpurun_out/kernel_stats.csv | cut -c1-200
