#!/bin/bash
# The streamed step's tail (last k_rows_to_host beside k_median / k_tally_reduce) under
# variants of the D2H stream: `scripts/ab_tail.sh NAME "ENV=.. ENV=.." ...` — one
# rocprofv3 kernel-trace run of the headline step per variant; per-kernel averages and
# ms per step into gpurun_out/NAME.txt.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
name=$1; shift
HEAD="--steps 5 --warmup 2 --no-cpu-baseline --no-check --no-pcie --no-device --no-device-paired --no-host-pack --no-e2e"
: > gpurun_out/$name.txt
i=0
for v in "$@"; do
    i=$((i + 1))
    d=gpurun_out/${name}_$i
    rm -rf "$d"
    env $v timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d "$d" -o run -- python3 bench.py $HEAD ${BENCH_ARGS:-} \
        > "$d.log" 2>&1 || { echo "variant $v failed"; tail -5 "$d.log"; exit 1; }
    python3 - "$d" "$v" >> gpurun_out/$name.txt <<'PY'
import csv, glob, json, sys
d, v = sys.argv[1], sys.argv[2]
line = [l for l in open(d + ".log") if l.startswith("{")][-1]
b = json.loads(line)
f = glob.glob(d + "/**/*kernel_stats.csv", recursive=True)[0]
ks = {r["Name"].split("(")[0].split("<")[0].replace("void ", ""): float(r["AverageNs"]) / 1e3 for r in csv.DictReader(open(f))}
keep = {k: round(ks[k], 1) for k in ("k_median", "k_tally_reduce", "k_rows_to_host", "k_pileup", "k_pair_place") if k in ks}
print(json.dumps({"variant": v, "ms_per_step": round(b["ms_per_step"], 2), "value": round(b["value"] / 1e9, 4), "avg_us": keep}))
PY
    tail -1 gpurun_out/$name.txt
done
