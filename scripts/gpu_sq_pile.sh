#!/bin/bash
# SQ counters of k_pileup for the default library and ablation variants (SURVEY.md
# §8 row: what the pileup's skeleton costs). One rocprofv3 --pmc run per counter group
# and library; each variant's counters land in gpurun_out/sqp_<lib>/ and are
# summarised per kernel into gpurun_out/sq_pile_<V>.txt.
#   V=tag bash scripts/gpu_sq_pile.sh [libmgpileup_x.so ...]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
V=${V:-sqp}
NB="--steps 2 --warmup 0 --no-cpu-baseline --no-check --no-pcie --no-device-paired --no-host-pack"
out=gpurun_out/sq_pile_$V.txt
: > "$out"
for lib in base "$@"; do
    unset MGP_LIB
    if [ "$lib" != base ]; then export MGP_LIB=mgatk2_amd/_lib/$lib; fi
    i=0
    while read -r grp; do
        [ -z "$grp" ] && continue
        i=$((i+1))
        timeout -s KILL 120 rocprofv3 --pmc $grp --kernel-include-regex "k_pileup" --output-format csv \
            -d "gpurun_out/sqp_$lib/pmc_$i" -o pmc -- python bench.py $NB > "gpurun_out/sqp_${lib}_$i.log" 2>&1
        rc=$?
        if [ $rc -ne 0 ]; then echo "$lib pass $i rc=$rc"; tail -5 "gpurun_out/sqp_${lib}_$i.log"; exit $rc; fi
    done <<'GROUPS'
SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAVES
SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR
SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE
GROUPS
    echo "== $lib" >> "$out"
    python scripts/pmc_summary.py "gpurun_out/sqp_$lib" >> "$out" 2>&1
done
cat "$out"
