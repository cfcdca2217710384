#!/bin/bash
# Round 4 GPU pass: the GPU suite (verbose: one line per test), then the default bench
# line. V names the logs; STEPS picks the parts (suite,bench,fullsize).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
V=${V:-r4}
STEPS=${STEPS:-suite,bench}
has() { [[ ",$STEPS," == *",$1,"* ]]; }  # exact step names, comma-separated
AB=${AB:-}; AB5=${AB5:-}; SQP=${SQP:-}; TK=${TK:-gpu}; DECENV=${DECENV:-}
if has smoke; then
    timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" \
        > gpurun_out/smoke_$V.log 2>&1 || { tail -30 gpurun_out/smoke_$V.log; exit 1; }
    tail -2 gpurun_out/smoke_$V.log
fi
if has suite; then
    timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
        -p no:cacheprovider > gpurun_out/pytest_gpu_$V.log 2>&1 || { tail -30 gpurun_out/pytest_gpu_$V.log; exit 1; }
    tail -3 gpurun_out/pytest_gpu_$V.log
fi
if has sel; then
    # a selection of the GPU suite (TK: pytest -k expression)
    timeout -k 10 600 python -u -m pytest tests -m gpu -x -v -k "$TK" --timeout 300 --timeout-method thread \
        -p no:cacheprovider > gpurun_out/pytest_sel_$V.log 2>&1 || { tail -30 gpurun_out/pytest_sel_$V.log; exit 1; }
    tail -3 gpurun_out/pytest_sel_$V.log
fi
if has fullsize; then
    timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -v -k "full_size" --timeout 300 \
        --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_fullsize_$V.log 2>&1 \
        || { tail -30 gpurun_out/pytest_fullsize_$V.log; exit 1; }
    tail -3 gpurun_out/pytest_fullsize_$V.log
fi
if has e2e3; then
    MGP_HOST_PROFILE=1 timeout -k 10 600 python -u scripts/e2e_bench.py --reads 50000000 --cells 5000 --out /tmp/mgp_e2e \
        > gpurun_out/e2e_c3_$V.json 2> gpurun_out/e2e_c3_$V.log || { tail -30 gpurun_out/e2e_c3_$V.log; exit 1; }
    cat gpurun_out/e2e_c3_$V.log
fi
if has dec; then
    # streamed C3 txt pipeline under decoder variants (DECENV: space-separated NAME=VALUE sets, ',' joins)
    for v in base $DECENV; do
        envset=(); [ "$v" != base ] && IFS=, read -ra envset <<< "$v"
        MGP_HOST_PROFILE=1 timeout -k 10 300 env "${envset[@]}" python -u scripts/e2e_bench.py --reads 50000000 \
            --cells 5000 --out /tmp/mgp_e2e --modes stream --formats txt > gpurun_out/dec_${V}_$v.json \
            2> gpurun_out/dec_${V}_$v.log || { tail -30 gpurun_out/dec_${V}_$v.log; exit 1; }
        echo "== $v"; grep -h "mgp_bam_stream\|txt_stream" gpurun_out/dec_${V}_$v.log | cut -c1-300
    done
fi
if has e2e4x2; then
    # C4 through the pipeline with the cells split over two engine contexts on this GPU (the
    # multi-device streamed path and its host concat of the rows, at scale)
    MGP_HOST_PROFILE=1 timeout -k 10 900 python -u scripts/e2e_bench.py --reads 200000000 --cells 10000 \
        --out /tmp/mgp_e2e4 --modes stream --formats hdf5,txt --devices 0,0 > gpurun_out/e2e_c4x2_$V.json \
        2> gpurun_out/e2e_c4x2_$V.log || { tail -30 gpurun_out/e2e_c4x2_$V.log; exit 1; }
    grep "\[e2e\]" gpurun_out/e2e_c4x2_$V.log | cut -c1-400
fi
if has rehearse; then
    # bench.py --gpus 2 with both ranks on this GPU (no RCCL): the multi-rank bench path
    MGP_BENCH_NO_COMM=1 timeout -k 10 400 python -u bench.py --gpus 2 --steps 5 --warmup 2 --no-cpu-baseline \
        > gpurun_out/rehearse2_$V.log 2>&1 || { tail -30 gpurun_out/rehearse2_$V.log; exit 1; }
    tail -c 1200 gpurun_out/rehearse2_$V.log
fi
if has e2e4; then
    MGP_HOST_PROFILE=1 timeout -k 10 900 python -u scripts/e2e_bench.py --reads 200000000 --cells 10000 --out /tmp/mgp_e2e4 \
        --modes stream --formats txt,hdf5 > gpurun_out/e2e_c4_$V.json 2> gpurun_out/e2e_c4_$V.log \
        || { tail -30 gpurun_out/e2e_c4_$V.log; exit 1; }
    cat gpurun_out/e2e_c4_$V.log
fi
if has c5; then
    # C5 on one GPU with the PCIe-inclusive leg's batch-size sweep (first = reported)
    timeout -k 10 900 python -u bench.py --reads 1000000000 --cells 100000 --steps 5 --warmup 1 \
        --no-cpu-baseline --no-check --no-device-paired --no-host-pack \
        --batch-reads 16000000,1000000,4000000,64000000 > gpurun_out/bench_c5_$V.log 2>&1 \
        || { tail -30 gpurun_out/bench_c5_$V.log; exit 1; }
    tail -c 1500 gpurun_out/bench_c5_$V.log
fi
if has ab; then
    # A/B of engine variants (AB="libmgpileup_x.so ..."), C4 default bench
    bash scripts/ab_bench.sh $AB > gpurun_out/ab_$V.txt 2>&1 || { tail -30 gpurun_out/ab_$V.txt; exit 1; }
    cat gpurun_out/ab_$V.txt
fi
if has abshare; then
    # the same A/B at the 8- and 4-GPU strong-scaling shares of C4 (1250 and 2500 cells per GPU)
    for sh in ${SHARES:-"25000000 1250" "50000000 2500"}; do
        set -- ${sh//_/ }
        BARGS="--reads $1 --cells $2 --steps 20 --warmup 3 --no-cpu-baseline --no-check --no-pcie --no-device-paired --no-host-pack" \
            bash scripts/ab_bench.sh $AB > gpurun_out/abshare_${V}_$2.txt 2>&1 || { tail -30 gpurun_out/abshare_${V}_$2.txt; exit 1; }
        echo "== $2 cells"; cat gpurun_out/abshare_${V}_$2.txt
    done
fi
if has ab5; then
    # the same A/B at C5 on one GPU (AB5="libmgpileup_x.so ..."; MGP_* env variants as ENV:NAME=VALUE)
    BARGS="--reads 1000000000 --cells 100000 --steps 3 --warmup 1 --no-cpu-baseline --no-check --no-pcie --no-device-paired --no-host-pack" \
        bash scripts/ab_bench.sh $AB5 > gpurun_out/ab5_$V.txt 2>&1 || { tail -30 gpurun_out/ab5_$V.txt; exit 1; }
    cat gpurun_out/ab5_$V.txt
fi
if has sqp; then
    # k_pileup SQ counters, default and ablation libraries (SQP="libmgpileup_abl1.so ...")
    V=$V bash scripts/gpu_sq_pile.sh $SQP > gpurun_out/sqp_$V.log 2>&1 || { tail -30 gpurun_out/sqp_$V.log; exit 1; }
    cat gpurun_out/sq_pile_$V.txt
fi
if has prof; then
    # rocprofv3 kernel stats + FETCH/WRITE PMC passes of the default bench (gpu_round3.sh)
    STEPS=rocprof,pmc bash scripts/gpu_round3.sh > gpurun_out/prof_$V.log 2>&1 || { tail -30 gpurun_out/prof_$V.log; exit 1; }
    grep "rc=" gpurun_out/prof_$V.log
fi
if has wr; then
    # output stage on the box's host cores, C3-shaped arrays (no GPU)
    MGP_TXT_PROFILE=1 timeout -k 10 400 python -u scripts/writers_bench.py --cells 5000 \
        > gpurun_out/writers_c3_$V.json 2> gpurun_out/writers_c3_$V.log || { tail -30 gpurun_out/writers_c3_$V.log; exit 1; }
    cat gpurun_out/writers_c3_$V.log
fi
if has bench; then
    timeout -k 10 500 python -u bench.py > gpurun_out/bench_$V.log 2>&1 || { tail -30 gpurun_out/bench_$V.log; exit 1; }
    tail -c 1500 gpurun_out/bench_$V.log
fi
