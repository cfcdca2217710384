#!/bin/bash
# One GPU-box session: smoke -> gpu tests -> small bench -> full bench.
# Each GPU step has its own time limit; a crash/timeout (rc not 0/1) stops the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {  # name timeout cmd...
    local name=$1 t=$2; shift 2
    echo "== $name: $*"
    timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
    local rc=$?
    echo "== $name rc=$rc"
    tail -n 5 "gpurun_out/$name.log"
    return $rc
}
step probe 120 python scripts/probe_device.py
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()" || exit $?
step pytest_gpu 900 python -m pytest tests -m gpu -q -x -p no:cacheprovider
rc=$?; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
step bench_small 300 python bench.py --reads 20000000 --cells 1000 --steps 5 --warmup 1 --no-cpu-baseline || exit $?
step bench 600 python bench.py --steps 5 --warmup 2 || exit $?
