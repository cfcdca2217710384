#!/bin/bash
# Full round on one GPU box: smoke, gpu tests, bench (with CPU baseline),
# rocprofv3 kernel stats, FETCH/WRITE PMC passes -> traffic json.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {
    local name=$1 t=$2; shift 2
    echo "== $name: $*"
    timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
    local rc=$?
    echo "== $name rc=$rc"
    tail -n 3 "gpurun_out/$name.log" | cut -c1-3000
    return $rc
}
SKIP_TESTS=${SKIP_TESTS:-0}
SKIP_PMC=${SKIP_PMC:-0}
BENCH_ARGS=${BENCH_ARGS:-}
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()" || exit $?
if [ "$SKIP_TESTS" = 0 ]; then
    step pytest_gpu 900 python -m pytest tests -m gpu -q -x -p no:cacheprovider
    rc=$?; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
fi
step bench 900 python bench.py $BENCH_ARGS || exit $?
step rocprof 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- \
    python bench.py --steps 5 --warmup 1 --no-cpu-baseline || exit $?
find gpurun_out/prof -name "*kernel_stats.csv" -exec cp {} gpurun_out/kernel_stats.csv \;
[ "$SKIP_PMC" = 0 ] || exit 0
for grp in FETCH_SIZE WRITE_SIZE; do
    step pmc_$grp 400 rocprofv3 --pmc $grp --kernel-include-regex "k_pileup|k_group_a|k_group_b|k_bin_count|k_median" \
        --output-format csv -d gpurun_out/pmc_$grp -o pmc -- python bench.py --steps 2 --warmup 0 --no-cpu-baseline \
        || exit $?
done
python scripts/pmc_traffic.py gpurun_out 200000000 10000 gpurun_out/pmc_traffic.json
