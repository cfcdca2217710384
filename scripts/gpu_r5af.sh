#!/bin/bash
# Round 5: C4 txt (gzip 1) end to end with the pinned rows target (allocated on a thread
# during the first batches) against rows fetched after the run (MGP_ROWS_TARGET=0).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
E="python -u scripts/e2e_bench.py --reads 200000000 --cells 10000 --formats txt --modes stream --gzip-levels 1 --out /tmp/mgp_e2e_c4"
timeout -k 10 400 $E > gpurun_out/e2e_rows_gen.log 2>&1 || { tail -20 gpurun_out/e2e_rows_gen.log; exit 1; }
for i in 1 2; do
    for a in 1 0; do
        MGP_ROWS_TARGET=$a timeout -k 10 200 $E --reuse-bam > gpurun_out/e2e_rows_$a$i.log 2>&1 || { tail -20 gpurun_out/e2e_rows_$a$i.log; exit 1; }
        python - "$a" "gpurun_out/e2e_rows_$a$i.log" <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[2]) if l.startswith("{")][-1])["txt_stream"]
print("rows_target", sys.argv[1], {k: d[k] for k in ("wall_s", "stream_setup", "stream_first_batch", "bam_ingest", "engine_tail", "engine_fetch", "write", "total")})
PY
    done
done
