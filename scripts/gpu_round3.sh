#!/bin/bash
# Round 3 measurement pass on one GPU box: the full-size C4/C5 parity tests, a
# 2-rank rehearsal of `bench.py --gpus 2` (both ranks on this GPU, no RCCL), the
# rocprofv3 kernel stats of the default bench, the FETCH/WRITE PMC passes of the
# default layout (-> pmc_traffic.json) and the pileup's HBM read requests by size
# for the 32-byte (quad32) and 64-byte (paired) layouts. Every step has its own
# time limit; the script stops at the first failing step.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
STEPS=${STEPS:-fullsize,rehearse,rocprof,pmc,rdreq}
step() {
    local name=$1 t=$2; shift 2
    echo "== $name: $*"
    timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
    local rc=$?
    echo "== $name rc=$rc"
    tail -n 3 "gpurun_out/$name.log" | cut -c1-3000
    return $rc
}
NB="--no-cpu-baseline --no-check --no-pcie --no-device-paired --no-host-pack"
if [[ $STEPS == *fullsize* ]]; then
    step fullsize 700 python -u -m pytest tests/test_gpu_parity.py -x -v -k "c4 or c5" --timeout 300 \
        --timeout-method thread -p no:cacheprovider || exit $?
fi
if [[ $STEPS == *rehearse* ]]; then
    MGP_BENCH_NO_COMM=1 step rehearse2 300 python -u bench.py --gpus 2 --steps 5 --warmup 2 --no-cpu-baseline \
        || exit $?
fi
if [[ $STEPS == *rocprof* ]]; then
    step rocprof 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- \
        python bench.py --steps 5 --warmup 1 $NB || exit $?
    find gpurun_out/prof -name "*kernel_stats.csv" -exec cp {} gpurun_out/kernel_stats.csv \;
fi
if [[ $STEPS == *pmc* ]]; then
    for grp in FETCH_SIZE WRITE_SIZE; do
        step pmc_$grp 300 rocprofv3 --pmc $grp --kernel-include-regex "k_pileup|k_group_a|k_group_b|k_bin_count|k_median" \
            --output-format csv -d gpurun_out/pmc_$grp -o pmc -- python bench.py --steps 2 --warmup 0 $NB || exit $?
    done
    python scripts/pmc_traffic.py gpurun_out 200000000 10000 gpurun_out/pmc_traffic.json quad32
fi
if [[ $STEPS == *rdreq* ]]; then
    for lay in quad32 paired; do
        step rdreq_$lay 300 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum \
            TCC_EA0_RDREQ_128B_sum --kernel-include-regex "k_pileup" --output-format csv -d gpurun_out/rdreq_$lay \
            -o pmc -- python bench.py --steps 2 --warmup 0 $NB --record-layout $lay || exit $?
    done
    python - <<'PY' > gpurun_out/rdreq.txt
import csv, glob
from collections import defaultdict
for lay in ("quad32", "paired"):
    acc = defaultdict(list)
    for f in glob.glob(f"gpurun_out/rdreq_{lay}/**/*counter_collection.csv", recursive=True):
        for row in csv.DictReader(open(f)):
            acc[row["Counter_Name"]].append(float(row["Counter_Value"]))
    print(lay, {k: f"{sum(v) / len(v):.4g}" for k, v in sorted(acc.items())})
PY
    cat gpurun_out/rdreq.txt
fi
