#!/bin/bash
# SQ counters of the pileup kernels for the default library and a variant (MGP_LIB=$1).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
V=${1:?variant}
i=0
while read -r grp; do
    [ -z "$grp" ] && continue
    i=$((i+1))
    for lib in base "$V"; do
        if [ "$lib" = base ]; then unset MGP_LIB; else export MGP_LIB=mgatk2_amd/_lib/$lib; fi
        timeout -k 10 300 rocprofv3 --pmc $grp --kernel-include-regex "k_pileup" --output-format csv \
            -d gpurun_out/sq_${lib}_$i -o pmc -- python bench.py --steps 2 --warmup 0 --no-cpu-baseline \
            > gpurun_out/sq_${lib}_$i.log 2>&1 || exit $?
    done
done <<'GROUPS'
SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS
SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAVES
GROUPS
unset MGP_LIB
for lib in base "$V"; do echo "== $lib"; python scripts/pmc_summary.py "gpurun_out" 2>/dev/null | head -0; done
python - "$V" <<'PY'
import csv, glob, sys
from collections import defaultdict
for lib in ("base", sys.argv[1]):
    acc = defaultdict(lambda: defaultdict(list))
    for f in glob.glob(f"gpurun_out/sq_{lib}_*/**/*counter_collection.csv", recursive=True):
        for row in csv.DictReader(open(f)):
            acc[row["Kernel_Name"].split("(")[0]][row["Counter_Name"]].append(float(row["Counter_Value"]))
    print("==", lib)
    for k, cs in sorted(acc.items()):
        print(" ", k)
        for c, v in sorted(cs.items()):
            print(f"    {c:24s} {sum(v)/len(v):.4g}")
PY
