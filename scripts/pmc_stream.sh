#!/bin/bash
# HBM traffic of the streamed headline step's kernels (MI355X guide, HBM section): one
# rocprofv3 PMC pass for FETCH_SIZE and one for WRITE_SIZE (each within the 4 TCC
# counters a pass can hold), then scripts/pmc_traffic.py -> profiles/pmc_traffic_stream.json
# (2 x FETCH_SIZE + WRITE_SIZE per launch; bench.py reads it when reads/cells match).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/pmcs
export TMPDIR=/tmp
K="k_pileup|k_group_a|k_group_b|k_bin_count|k_median"
HEAD="--steps 2 --warmup 1 --no-cpu-baseline --no-check --no-pcie --no-device --no-device-paired --no-host-pack --no-e2e"
for c in FETCH_SIZE WRITE_SIZE; do
    rm -rf gpurun_out/pmcs/pmc_$c
    timeout -s KILL 150 rocprofv3 --pmc $c --kernel-include-regex "$K" --output-format csv \
        -d gpurun_out/pmcs/pmc_$c -o pmc -- python3 bench.py $HEAD > gpurun_out/pmcs/pmc_$c.log 2>&1 || exit $?
done
python3 scripts/pmc_traffic.py gpurun_out/pmcs 200000000 10000 gpurun_out/pmc_traffic_stream.json packed
