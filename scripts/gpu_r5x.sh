#!/bin/bash
# Round 5: pass B carry without its own barrier: parity/stream tests, device step A/B
# (carry0, and no pel stores at all as the floor), pass B's WRITE_SIZE.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
V=${V:-r5x}
timeout -k 10 700 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_stream.py -m gpu -x -q --timeout 600 \
    --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_carry_$V.log 2>&1 \
    || { tail -30 gpurun_out/pytest_carry_$V.log; exit 1; }
tail -2 gpurun_out/pytest_carry_$V.log
for i in 1 2; do bash scripts/ab_bench.sh libmgpileup_carry0.so libmgpileup_nostore.so >> gpurun_out/ab_carry_$V.txt 2>&1 || { cat gpurun_out/ab_carry_$V.txt; exit 1; }; done
cat gpurun_out/ab_carry_$V.txt
DEV="--device-only --steps 3 --warmup 1 --no-cpu-baseline --no-check --no-pcie --no-device-paired --no-host-pack"
for lib in base carry0; do
    unset MGP_LIB
    [ $lib != base ] && export MGP_LIB=mgatk2_amd/_lib/libmgpileup_$lib.so
    timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "k_group_b" --output-format csv \
        -d gpurun_out/pmcw_$lib -o pmc -- python bench.py $DEV > gpurun_out/pmcw_$lib.log 2>&1 || { echo "pmc $lib failed"; tail -3 gpurun_out/pmcw_$lib.log; exit 1; }
    f=$(find gpurun_out/pmcw_$lib -name "*counter_collection.csv" | head -1)
    python - "$f" "$lib" <<'PY'
import csv, sys
v = [float(r["Counter_Value"]) for r in csv.DictReader(open(sys.argv[1])) if r["Counter_Name"] == "WRITE_SIZE"]
print(f"{sys.argv[2]}: k_group_b WRITE_SIZE per dispatch {sum(v) / max(len(v), 1) * 1024 / 1e9:.3f} GB over {len(v)} dispatch rows")
PY
done
