#!/bin/bash
# Build an A/B variant of libmgpileup.so with extra -D flags (experiments only):
#   scripts/build_variant.sh NAME -DMGP_X=1 ...  ->  mgatk2_amd/_lib/libmgpileup_NAME.so
set -eu
cd "$(dirname "$0")/.."
name=$1; shift
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -Wall -Wno-unused-function "$@" \
    mgatk2_amd/csrc/mgp_engine.hip mgatk2_amd/csrc/mgp_synth.hip -o "mgatk2_amd/_lib/libmgpileup_$name.so" -lrccl
