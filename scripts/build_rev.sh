#!/bin/bash
# Build the engine library of a git revision as an A/B variant:
#   scripts/build_rev.sh <rev> <out.so> [extra hipcc -D flags...]
set -eu
rev=$1; out=$2; shift 2
d=$(mktemp -d)
mkdir -p "$d/mgatk2_amd/csrc" "$d/include"
for f in mgatk2_amd/csrc/mgp_engine.hip mgatk2_amd/csrc/mgp_synth.hip mgatk2_amd/csrc/mgp_kernels.h include/mgpileup.h; do
    git show "$rev:$f" > "$d/$f"
done
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -w "$@" \
    "$d/mgatk2_amd/csrc/mgp_engine.hip" "$d/mgatk2_amd/csrc/mgp_synth.hip" -o "$out" -lrccl
rm -rf "$d"
