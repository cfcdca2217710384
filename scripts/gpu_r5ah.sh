#!/bin/bash
# Round 5: the multi-device product path with rows fetched per device after the run
# (default) against per-device views of a pinned rows target (MGP_ROWS_TARGET=1): the
# pipeline GPU tests, then C4 txt gzip 1 on 8 contexts of one GPU, alternating.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests/test_pipeline.py -m gpu -x -q --timeout 300 --timeout-method thread \
    -p no:cacheprovider > gpurun_out/pytest_pipe_r5ah.log 2>&1 || { tail -30 gpurun_out/pytest_pipe_r5ah.log; exit 1; }
tail -1 gpurun_out/pytest_pipe_r5ah.log
E="python -u scripts/e2e_bench.py --reads 200000000 --cells 10000 --formats txt --modes stream --gzip-levels 1 --out /tmp/mgp_e2e_c4"
timeout -k 10 400 $E > gpurun_out/e2e_x8_gen.log 2>&1 || { tail -20 gpurun_out/e2e_x8_gen.log; exit 1; }
for i in 1 2; do
    for a in 0 1; do
        MGP_ROWS_TARGET=$a timeout -k 10 200 $E --reuse-bam --devices 0,0,0,0,0,0,0,0 > gpurun_out/e2e_c4x8_rows$a$i.log 2>&1 \
            || { tail -20 gpurun_out/e2e_c4x8_rows$a$i.log; exit 1; }
        python - "$a" "gpurun_out/e2e_c4x8_rows$a$i.log" <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[2]) if l.startswith("{")][-1])["txt_stream"]
print("x8 rows_target", sys.argv[1], {k: d[k] for k in ("wall_s", "bam_ingest", "engine_fetch", "write", "total")})
PY
    done
done
