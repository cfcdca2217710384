#!/bin/bash
# SQ/LDS counter passes for the main kernels (one rocprofv3 --pmc run per group).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
KRE=${KRE:-"k_pileup|k_scatter|k_bin_count"}
ARGS=${ARGS:-"--steps 2 --warmup 0 --no-cpu-baseline"}
i=0
while read -r grp; do
    [ -z "$grp" ] && continue
    i=$((i+1))
    echo "== pmc pass $i: $grp"
    timeout -k 10 400 rocprofv3 --pmc $grp --kernel-include-regex "$KRE" --output-format csv \
        -d gpurun_out/pmc_$i -o pmc -- python bench.py $ARGS > gpurun_out/pmc_$i.log 2>&1
    rc=$?
    echo "== pass $i rc=$rc"
    if [ $rc -ne 0 ]; then exit $rc; fi
done <<'GROUPS'
SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY
SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD
SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAVES
SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_INST_CYCLES_VMEM_WR
GROUPS
python scripts/pmc_summary.py gpurun_out > gpurun_out/pmc_summary.txt 2>&1
cat gpurun_out/pmc_summary.txt
