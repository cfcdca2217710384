#!/bin/bash
# Build an A/B variant of libmgpileup.so with extra defines (experiments only):
#   scripts/build_variant.sh NAME MGP_X=1 ...  ->  mgatk2_amd/_lib/libmgpileup_NAME.so
set -eu
cd "$(dirname "$0")/.."
name=$1; shift
python - "$name" "$@" <<'PY'
import sys
from mgatk2_amd.build import LIB_DIR, build_engine
build_engine(force=True, out=LIB_DIR / f"libmgpileup_{sys.argv[1]}.so", defines=tuple(sys.argv[2:]))
PY
