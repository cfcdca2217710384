#!/bin/bash
# Round 5: decode pool size (MGP_BAM_DEC_THREADS 12 / 14 / default 16) beside the 16-thread
# inflate pool, C4 txt gzip 1 end to end, alternating.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
E="python -u scripts/e2e_bench.py --reads 200000000 --cells 10000 --formats txt --modes stream --gzip-levels 1 --out /tmp/mgp_e2e_c4"
timeout -k 10 400 $E > gpurun_out/e2e_dec_gen.log 2>&1 || { tail -20 gpurun_out/e2e_dec_gen.log; exit 1; }
for i in 1 2; do
    for t in 12 14 16 20; do
        MGP_BAM_DEC_THREADS=$t timeout -k 10 200 $E --reuse-bam > gpurun_out/e2e_dec_$t$i.log 2>&1 || { tail -20 gpurun_out/e2e_dec_$t$i.log; exit 1; }
        python - "$t" "gpurun_out/e2e_dec_$t$i.log" <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[2]) if l.startswith("{")][-1])["txt_stream"]
print("dec threads", sys.argv[1], {k: d[k] for k in ("wall_s", "bam_ingest", "write")})
PY
    done
done
