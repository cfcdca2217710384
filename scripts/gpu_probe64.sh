#!/bin/bash
# 64-byte record gathers by allocation kind and load cache policy
# (scripts/probe_gather64.hip): timing pass, then one PMC pass of the fabric
# read-request sizes. Each GPU step has its own time limit.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 240 scripts/probe_gather64 > gpurun_out/probe64.log 2>&1 || exit $?
cat gpurun_out/probe64.log
timeout -s KILL 240 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum \
    TCC_EA0_RDREQ_128B_sum --output-format csv -d gpurun_out/pmc_probe64 -o pmc \
    -- scripts/probe_gather64 > gpurun_out/probe64_pmc.log 2>&1 || exit $?
python scripts/pmc_summary.py gpurun_out > gpurun_out/probe64_pmc.txt
cat gpurun_out/probe64_pmc.txt
