#!/bin/bash
# Round 5: streaming pileup chunk size A/B (workgroups per one-window launch), then
# the GPU stream tests at the new default.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
bash scripts/ab_stream.sh MGP_PILE_WG_STREAM=625 MGP_PILE_WG_STREAM=1024 MGP_PILE_WG_STREAM=4096 \
    MGP_PILE_WG_STREAM=4096,MGP_SEG_MIN_WIN=2 > gpurun_out/abs_r5e.txt 2>&1; rc=$?
cat gpurun_out/abs_r5e.txt
[ $rc -eq 0 ] || exit $rc
bash scripts/ab_bench.sh libmgpileup_qqs2.so libmgpileup_qqs4.so libmgpileup_qqs8.so libmgpileup_gbxcd.so \
    > gpurun_out/ab_r5e.txt 2>&1; rc=$?
cat gpurun_out/ab_r5e.txt
[ $rc -eq 0 ] || exit $rc
NB="--device-only --steps 2 --warmup 0 --no-cpu-baseline --no-check --no-pcie --no-device-paired --no-host-pack"
for lib in base libmgpileup_gbxcd.so; do
    unset MGP_LIB
    [ "$lib" != base ] && export MGP_LIB=mgatk2_amd/_lib/$lib
    for grp in WRITE_SIZE FETCH_SIZE; do
        timeout -s KILL 120 rocprofv3 --pmc $grp --kernel-include-regex "k_group_b|k_group_a" --output-format csv \
            -d gpurun_out/pmcb_$lib/pmc_$grp -o pmc -- python bench.py $NB > gpurun_out/pmcb_${lib}_$grp.log 2>&1 || { echo "pmc $lib $grp failed"; tail -3 gpurun_out/pmcb_${lib}_$grp.log; exit 1; }
    done
    echo "== $lib"
    python scripts/pmc_traffic.py gpurun_out/pmcb_$lib 200000000 10000 gpurun_out/pmcb_$lib.json quad32 | grep -A3 '"k_group'
done
unset MGP_LIB
timeout -k 10 600 python -u -m pytest tests/test_gpu_stream.py tests/test_abi.py -x -q --timeout 120 --timeout-method thread \
    -p no:cacheprovider > gpurun_out/pytest_stream_r5e.log 2>&1; rc=$?
tail -3 gpurun_out/pytest_stream_r5e.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 700 python -u -m pytest tests/test_gpu_parity.py -x -v -k "eight_cell_shards" --timeout 650 \
    --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_c4x8_r5e.log 2>&1; rc=$?
tail -3 gpurun_out/pytest_c4x8_r5e.log
exit $rc
