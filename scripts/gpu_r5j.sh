#!/bin/bash
# Round 5: C5 (1B reads x 100k cells) on one GPU with the round-5 bench: the streamed
# headline at the auto batch (80M reads) and a batch sweep, the resident device step.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
free -g | head -2
timeout -k 10 900 python -u bench.py --reads 1000000000 --cells 100000 --seed $((20251015 + 5)) --steps 3 --warmup 1 \
    --no-cpu-baseline --no-host-pack --no-device-paired --batch-reads auto,16000000,64000000 \
    > gpurun_out/bench_c5_r5j.log 2>&1; rc=$?
python - <<'PY'
import json
l = [x for x in open("gpurun_out/bench_c5_r5j.log") if x.startswith("{")]
if l:
    d = json.loads(l[-1])
    print({k: d[k] for k in ("value", "ms_per_step", "value_device", "device_ms_quad32", "bit_exact")})
    print("stream", d["stream"], "link", d["link"]["h2d_GBps"])
    print("roofline", {k: d["roofline"][k] for k in ("frac", "avg_launch_ms", "launches_per_step")})
    print("dev stages", d["device"]["stage_ms"])
    for leg in d["pcie_pack32"]["legs"] + d["pcie_pack32"].get("sweep_packed", []):
        print(leg)
PY
[ $rc -eq 0 ] || tail -20 gpurun_out/bench_c5_r5j.log
exit $rc
