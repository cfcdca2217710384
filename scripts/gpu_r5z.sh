#!/bin/bash
# Round 5: host link probe with a kernel pulling mapped pinned host memory.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O2 scripts/probe_pcie.hip -o /tmp/probe_pcie || exit 1
timeout -k 10 120 /tmp/probe_pcie > gpurun_out/pcie_probe_r5z.txt 2>&1; rc=$?
cat gpurun_out/pcie_probe_r5z.txt
exit $rc
