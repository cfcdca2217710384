#!/bin/bash
# Round 5: C4 BAM ingest A/B (alternating) of the prefetch's read-ahead and boundary walk
# on threads of their own: AB=WALK (MGP_BAM_WALK_ASYNC) or AB=READ (MGP_BAM_READ_AHEAD).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
V=${V:-r5t}
E="python -u scripts/e2e_bench.py --reads 200000000 --cells 10000 --formats txt --modes stream --gzip-levels 1 --out /tmp/mgp_e2e_c4"
MGP_HOST_PROFILE=1 timeout -k 10 400 $E > gpurun_out/e2e_walk_${V}_gen.log 2>&1 || { tail -20 gpurun_out/e2e_walk_${V}_gen.log; exit 1; }
grep "^\[mgp_bam_stream\]" gpurun_out/e2e_walk_${V}_gen.log | cut -c1-330
for i in 1 2 3; do
    for a in 0 1; do
        env MGP_BAM_${AB:-READ_AHEAD}=$a MGP_HOST_PROFILE=1 timeout -k 10 200 $E --reuse-bam > gpurun_out/e2e_walk_${V}_$a$i.log 2>&1 \
            || { tail -20 gpurun_out/e2e_walk_${V}_$a$i.log; exit 1; }
        echo "async=$a: $(grep -o "open [0-9.]* s; waiting for inflated chunks [0-9.]*\|prefetch: [^;]*\|classify [0-9.]*" gpurun_out/e2e_walk_${V}_$a$i.log | tr '\n' ' ') $(grep -o "'wall_s': [0-9.]*" gpurun_out/e2e_walk_${V}_$a$i.log)"
    done
done
