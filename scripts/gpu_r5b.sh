#!/bin/bash
# Round 5: the host's memory bandwidth by thread count, the restructured bench
# (streamed 64-byte headline) small then at C4, and the record-check GPU tests.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
g++ -O2 -pthread scripts/probe_hostbw.cpp -o /tmp/probe_hostbw && timeout -k 5 60 /tmp/probe_hostbw > gpurun_out/hostbw_r5b.txt 2>&1
cat gpurun_out/hostbw_r5b.txt
nproc; python -c "import os; print('affinity', len(os.sched_getaffinity(0)))"
timeout -k 10 300 python bench.py --reads 2000000 --cells 500 --steps 3 --warmup 1 --no-cpu-baseline \
    --batch-reads 400000,100000 > gpurun_out/bench_small_r5b.log 2>&1 || { tail -30 gpurun_out/bench_small_r5b.log; exit 1; }
tail -c 3000 gpurun_out/bench_small_r5b.log
timeout -k 10 600 python bench.py > gpurun_out/bench_r5b.log 2>&1 || { tail -30 gpurun_out/bench_r5b.log; exit 1; }
python - <<'PY'
import json
d = json.loads([l for l in open("gpurun_out/bench_r5b.log") if l.startswith("{")][-1])
print({k: d[k] for k in ("value", "ms_per_step", "value_device", "device_ms_quad32", "device_ms_paired", "bit_exact")})
print("roofline", {k: v for k, v in d["roofline"].items() if k != "kernels"})
print("link", d["link"])
print("stream", d["stream"])
print("pcie_pack32", d["pcie_pack32"]["value"], d["pcie_pack32"]["best_batch_reads"])
print("cpu", d["cpu_baseline"]["value"], "host_pack", d["host_pack"])
print("dev roofline", d["device"]["roofline"]["frac"], d["device"]["stage_ms"])
PY
timeout -k 10 300 python -u -m pytest tests/test_gpu_stream.py -x -q -k "records_outside" --timeout 120 \
    --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_rec_r5b.log 2>&1; rc=$?
tail -3 gpurun_out/pytest_rec_r5b.log
exit $rc
