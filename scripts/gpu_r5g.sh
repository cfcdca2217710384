#!/bin/bash
# Round 5 measurement pass: the whole GPU suite, the default bench line, rocprofv3
# kernel stats of the streamed headline alone and of the resident device leg alone,
# and the FETCH/WRITE PMC passes of each (-> profiles' pmc_traffic_stream.json /
# pmc_traffic.json, which bench.py reads for roofline.traffic).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
V=${V:-r5g}
STEPS=${STEPS:-tests,bench,prof,pmc}
if [[ $STEPS == *tests* ]]; then
    timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
        > gpurun_out/pytest_gpu_$V.log 2>&1 || { tail -20 gpurun_out/pytest_gpu_$V.log; exit 1; }
    tail -2 gpurun_out/pytest_gpu_$V.log
fi
if [[ $STEPS == *bench* ]]; then
    timeout -k 10 400 python -u bench.py > gpurun_out/bench_$V.log 2>&1 || { tail -20 gpurun_out/bench_$V.log; exit 1; }
    tail -c 400 gpurun_out/bench_$V.log
fi
HEAD="--steps 5 --warmup 1 --no-cpu-baseline --no-check --no-pcie --no-device --no-device-paired --no-host-pack --no-e2e"
DEV="--device-only --steps 5 --warmup 1 --no-cpu-baseline --no-check --no-pcie --no-device-paired --no-host-pack --no-e2e"
if [[ $STEPS == *prof* ]]; then
    for leg in head dev; do
        args=$HEAD; [ $leg = dev ] && args=$DEV
        timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/kprof_$leg -o run -- \
            python bench.py $args > gpurun_out/kprof_${leg}_$V.log 2>&1 || { tail -5 gpurun_out/kprof_${leg}_$V.log; exit 1; }
        f=$(find gpurun_out/kprof_$leg -name "*kernel_stats.csv" | head -1)
        cp "$f" gpurun_out/kernel_stats_${leg}_$V.csv
        echo "== $leg"
        python - "$leg" "$V" <<'PY'
import csv, json, sys
leg, V = sys.argv[1], sys.argv[2]
for r in csv.DictReader(open(f"gpurun_out/kernel_stats_{leg}_{V}.csv")):
    if "pileup" in r["Name"] or "group" in r["Name"] or "bin_count" in r["Name"]:
        print(f'{r["Name"].split("(")[0][:40]:40s} calls={r["Calls"]:>5s} avg_ms={float(r["AverageNs"])/1e6:8.4f}')
d = json.loads([l for l in open(f"gpurun_out/kprof_{leg}_{V}.log") if l.startswith("{")][-1])
r = d["roofline"]
print("bench:", {k: r[k] for k in ("achieved", "frac", "avg_launch_ms", "launches_per_step")}, "ms/step", d["ms_per_step"])
PY
    done
fi
if [[ $STEPS == *pmc* ]]; then
    for leg in head dev; do
        args=$HEAD; [ $leg = dev ] && args=$DEV
        for grp in FETCH_SIZE WRITE_SIZE; do
            timeout -s KILL 150 rocprofv3 --pmc $grp --kernel-include-regex "k_pileup|k_group_a|k_group_b|k_bin_count|k_median" \
                --output-format csv -d gpurun_out/pmc_$leg/pmc_$grp -o pmc -- python bench.py $args \
                > gpurun_out/pmc_${leg}_$grp.log 2>&1 || { echo "pmc $leg $grp failed"; tail -3 gpurun_out/pmc_${leg}_$grp.log; exit 1; }
        done
    done
    python scripts/pmc_traffic.py gpurun_out/pmc_head 200000000 10000 gpurun_out/pmc_traffic_stream.json packed > /dev/null
    python scripts/pmc_traffic.py gpurun_out/pmc_dev 200000000 10000 gpurun_out/pmc_traffic.json quad32 > /dev/null
    python -c "import json; [print(f, {k: v for k, v in json.load(open(f)).items() if k in ('pileup','group_a','group_b','hist')}) for f in ('gpurun_out/pmc_traffic_stream.json','gpurun_out/pmc_traffic.json')]"
fi
