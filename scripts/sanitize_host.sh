#!/bin/bash
# The host library (libmgphost.so: threaded BGZF/BAM decoder, placement, writers) built
# with AddressSanitizer and, separately, ThreadSanitizer, and the CPU tests that drive
# its threads (whole / streamed / pipelined decode, placement, pack32, txt and HDF5
# tiles) run against each build. CPU only (no GPU code is instrumented).
#   scripts/sanitize_host.sh [asan|tsan ...]   -> /tmp/mgp_san/<mode>.log
set -u
cd "$(dirname "$0")/.."
out=/tmp/mgp_san
mkdir -p $out
SRCS="mgatk2_amd/csrc/host/mgp_bam.cpp mgatk2_amd/csrc/host/mgp_txt.cpp mgatk2_amd/csrc/host/mgp_tiles.cpp
      mgatk2_amd/csrc/host/mgp_bamw.cpp mgatk2_amd/csrc/host/mgp_shard.cpp mgatk2_amd/csrc/host/mgp_place.cpp
      mgatk2_amd/csrc/host/mgp_repack.cpp"
TESTS=${TESTS:-"tests/test_bam.py tests/test_placement.py tests/test_pack32.py tests/test_writers_golden.py
       tests/test_pipeline.py::test_stream_batches_equal_the_whole_decode
       tests/test_pipeline.py::test_stream_pipelined_decode_equals_serial
       tests/test_pipeline.py::test_stream_sharded_routing_host tests/test_pipeline.py::test_pipeline_txt_host"}
# (not the HDF5 pipeline tests: their QC report imports matplotlib, whose extension
# modules abort under the preloaded ASan runtime before any of this library's code runs)
rc=0
for mode in "${@:-asan tsan}"; do
    for m in $mode; do
        case $m in
            asan) flags="-fsanitize=address -fno-omit-frame-pointer"; rt=$(gcc -print-file-name=libasan.so)
                  envs="ASAN_OPTIONS=detect_leaks=0:abort_on_error=1:symbolize=1:log_path=$out/asan.rep" ;;
            tsan) flags="-fsanitize=thread"; rt=$(gcc -print-file-name=libtsan.so)
                  envs="TSAN_OPTIONS=halt_on_error=1:second_deadlock_stack=1:log_path=$out/tsan.rep" ;;
        esac
        lib=$out/libmgphost_$m.so
        rm -f $out/$m.rep.*  # (reports go to files: pytest's output capture would swallow them)
        g++ -O1 -g -std=c++17 -fPIC -shared -Wall -pthread $flags -Iinclude $SRCS -o $lib -lz -ldl || exit 1
        echo "== $m: $lib"
        env MGP_HOST_LIB=$lib LD_PRELOAD=$rt $envs MGP_HOST_THREADS=8 \
            timeout -k 10 1800 python -m pytest $TESTS -q -x -m "not gpu" -p no:cacheprovider > $out/$m.log 2>&1
        r=$?
        tail -3 $out/$m.log
        cat $out/$m.rep.* 2>/dev/null | head -80
        [ $r -ne 0 ] && rc=$r
    done
done
exit $rc
