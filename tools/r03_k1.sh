#!/bin/bash
# Round 3 K1 session on the GPU box: variant 6 timing vs 5, then the K1 parity
# tests.  Every GPU step has its own time limit; a failure ends the script.
set -u
cd "$(dirname "$0")/.."
OUT=gpurun_out/r03
mkdir -p $OUT
export TMPDIR=/tmp
step() {  # name seconds cmd...
    local name=$1 secs=$2
    shift 2
    echo "== $name" >&2
    timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1
    local rc=$?
    echo "== $name rc=$rc" >&2
    tail -n 30 "$OUT/$name.log" >&2
    if [ $rc -ne 0 ]; then exit $rc; fi
}
for s in ${STEPS:-time16 tests}; do
    case $s in
    time16) step k1_time_n16 240 python -u tools/k1_time.py 16 16384 8 6 5 ;;
    timeall) step k1_time_n15 120 python -u tools/k1_time.py 15 16384 8 6 5
             step k1_time_n14 120 python -u tools/k1_time.py 14 16384 8 6 5
             step k1_time_n13 120 python -u tools/k1_time.py 13 16384 8 6 5
             step k1_time_i32 120 python -u tools/k1_time.py 16 16384 4 6 5 ;;
    tests) step k1_tests 400 python -u -m pytest tests/test_k1_variants_gpu.py tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread ;;
    trace) rm -rf $OUT/trace_timed
           BENCH_I32=0 BENCH_OTHER_SCALING=0 step trace_timed 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace_timed -o run -- python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-pmc --no-tto --no-k2 --no-ref-multiblock ;;
    pmc6) step pmc6 300 bash tools/k1_pmc.sh v6_n16 16 4096 8 6 ;;
    rccl) step rccl_tests 300 python -u -m pytest tests/test_rccl_gpu.py tests/test_bench_gpu.py -x -v --timeout 200 --timeout-method thread ;;
    k2phases) step k2_phases 120 python -u tools/k2_phases.py 5 ;;
    k2var) step k2_variants 300 python -u tools/k2_phases.py --variants ;;
    ab) step ab_time 600 bash tools/ab_time.sh ;;
    k2tests) step k2_tests 600 python -u -m pytest tests/test_search_gpu.py tests/test_rccl_gpu.py tests/test_search_cli.py tests/test_tsplib.py -x -q -m gpu --timeout 200 --timeout-method thread ;;
    chaintest) step chain_test 300 python -u -m pytest tests/test_search_gpu.py -k "chained" -x -q --timeout 200 --timeout-method thread ;;
    pyk) step pyk 600 python -u -m pytest tests -m gpu -k "$PYK" -x -q --timeout 200 --timeout-method thread ;;
    gputests) step gpu_tests 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread ;;
    bench) step bench 600 python3 -u bench.py --steps 20 --warmup 3 ;;
    benchk2) step bench_k2 300 python3 -u bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-ref-multiblock --no-tto ;;
    bench2) step bench_2ranks 300 python3 -u bench.py --gpus 2 --steps 10 --warmup 2 --no-k2 ;;
    bench4) step bench_4ranks 400 python3 -u bench.py --gpus 4 --steps 5 --warmup 1 --no-k2 --no-tto ;;
    esac
done
