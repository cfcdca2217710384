#!/bin/bash
# Round 5, first box: the pileup's LDS-conflict ceiling (conflict-free address
# ablation, lane order, plane pitch), and the PCIe-inclusive leg on 64-byte records.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
bash scripts/ab_bench.sh libmgpileup_abl10.so libmgpileup_perm0.so libmgpileup_pad16.so > gpurun_out/ab_r5a.txt 2>&1 || { cat gpurun_out/ab_r5a.txt; exit 1; }
cat gpurun_out/ab_r5a.txt
V=r5a bash scripts/gpu_sq_pile.sh libmgpileup_abl10.so > /dev/null 2>&1 || { echo "sq failed"; exit 1; }
cat gpurun_out/sq_pile_r5a.txt
timeout -k 10 300 python bench.py --record-layout paired --steps 5 --warmup 1 --no-cpu-baseline --no-check \
    --no-host-pack --batch-reads 16000000,4000000,64000000 > gpurun_out/bench_paired_r5a.log 2>&1 || { tail -20 gpurun_out/bench_paired_r5a.log; exit 1; }
python - <<'PY'
import json
d = json.loads([l for l in open("gpurun_out/bench_paired_r5a.log") if l.startswith("{")][-1])
print("paired resident ms/step", d["ms_per_step"], "pcie", d["value_pcie"])
for leg in d["pcie"]["legs"]:
    print(leg)
PY
