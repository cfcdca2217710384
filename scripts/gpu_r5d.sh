#!/bin/bash
# Round 5: host link probe; rows-to-host grid size A/B on the streamed step.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
hipcc --offload-arch=gfx950 -O2 scripts/probe_pcie.hip -o /tmp/probe_pcie && timeout -k 10 120 /tmp/probe_pcie > gpurun_out/pcie_probe_r5d.txt 2>&1
cat gpurun_out/pcie_probe_r5d.txt
bash scripts/ab_stream.sh MGP_ROWS_WG=64 MGP_ROWS_WG=1024 MGP_ROWS_WG=1000000 MGP_ROWS_WG=64,MGP_SEG_MIN_WIN=3 > gpurun_out/abs_r5d.txt 2>&1; rc=$?
cat gpurun_out/abs_r5d.txt
exit $rc
