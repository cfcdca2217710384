#!/bin/bash
# Round 5: pass B with non-temporal element loads (write traffic of its partial lines).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
bash scripts/ab_bench.sh libmgpileup_gbnt.so > gpurun_out/ab_r5h.txt 2>&1; rc=$?
cat gpurun_out/ab_r5h.txt
[ $rc -eq 0 ] || exit $rc
NB="--device-only --steps 2 --warmup 0 --no-cpu-baseline --no-check --no-pcie --no-device-paired --no-host-pack"
for lib in libmgpileup_gbnt.so; do
    export MGP_LIB=mgatk2_amd/_lib/$lib
    timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "k_group_b" --output-format csv \
        -d gpurun_out/pmcn_$lib/pmc_WRITE_SIZE -o pmc -- python bench.py $NB > gpurun_out/pmcn_$lib.log 2>&1 || { echo "pmc failed"; exit 1; }
    python - "$lib" <<'PY'
import csv, glob, sys
v = [float(r["Counter_Value"]) for f in glob.glob(f"gpurun_out/pmcn_{sys.argv[1]}/**/*counter_collection.csv", recursive=True) for r in csv.DictReader(open(f))]
print(sys.argv[1], "k_group_b WRITE_SIZE per launch (B):", sum(v) / len(v) * 1024)
PY
done
unset MGP_LIB
