#!/bin/bash
# Round 5 final pass A: the whole GPU suite, smoke(), the default bench line.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
V=${V:-r5fa}
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread -p no:cacheprovider \
    > gpurun_out/pytest_gpu_$V.log 2>&1 || { tail -30 gpurun_out/pytest_gpu_$V.log; exit 1; }
tail -1 gpurun_out/pytest_gpu_$V.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$V.log 2>&1 || { cat gpurun_out/smoke_$V.log; exit 1; }
cat gpurun_out/smoke_$V.log
timeout -k 10 400 python -u bench.py > gpurun_out/bench_$V.log 2>&1 || { tail -20 gpurun_out/bench_$V.log; exit 1; }
grep '^{' gpurun_out/bench_$V.log | python -c "
import json,sys; d=json.loads(sys.stdin.read())
print('value', d['value'], 'ms', d['ms_per_step'], 'bit_exact', d['bit_exact'], 'frac', d['roofline']['frac'], 'traffic', d['roofline']['traffic'])
print('device', d['value_device'], d['device_ms_quad32'], d['device_ms_paired'])
print('e2e', {k: v['wall_s'] for k, v in d['e2e'].items() if isinstance(v, dict)})
print('cpu', d['cpu_baseline']['value'])"
