#!/bin/bash
# PMC counter passes (one counter group per rocprofv3 run; no trace domains mixed in).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
KRE=${KRE:-"k_pileup|k_scatter|k_bin_hist|k_median"}
ARGS=${ARGS:-"--steps 2 --warmup 0 --no-cpu-baseline"}
timeout -k 10 120 rocprofv3 -L > gpurun_out/counters_list.txt 2>&1 || true
i=0
while read -r grp; do
    [ -z "$grp" ] && continue
    i=$((i+1))
    echo "== pmc pass $i: $grp"
    timeout -k 10 400 rocprofv3 --pmc $grp --kernel-include-regex "$KRE" --output-format csv \
        -d gpurun_out/pmc_$i -o pmc -- python bench.py $ARGS > gpurun_out/pmc_$i.log 2>&1
    rc=$?
    echo "== pass $i rc=$rc"
    if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
done <<'GROUPS'
FETCH_SIZE
WRITE_SIZE
SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_LDS_BANK_CONFLICT
TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum
GROUPS
python scripts/pmc_summary.py gpurun_out > gpurun_out/pmc_summary.txt 2>&1
cat gpurun_out/pmc_summary.txt
