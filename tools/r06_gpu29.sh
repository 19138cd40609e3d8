#!/bin/bash
# Round-6 check 29: the tail launch at one block per CU at <= 16 cities and
# the fused prologue's per-block seed sum: K2 GPU tests, the 16-city search
# against CHAIN_TAIL_GRID=8 (the previous default), then a bench.py line.
set -u
cd "$(dirname "$0")/.."
OUT=gpurun_out/r06/tail1
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_search_gpu.py tests/test_tsplib.py tests/test_search_cli.py tests/test_rccl_gpu.py tests/test_search_dist.py -m gpu -x -q --timeout 240 --timeout-method thread > $OUT/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 $OUT/tests.log; [ $rc -eq 0 ] || exit $rc
SETS_JSON='[{}, {"CHAIN_TAIL_GRID": 8}, {}, {"CHAIN_TAIL_GRID": 8}, {}, {"CHAIN_TAIL_GRID": 8}]' timeout -k 10 300 python3 tools/k2_16_sweep.py 60 > $OUT/sweep.json 2> $OUT/sweep.err
echo "sweep rc=$?"; cat $OUT/sweep.json
timeout -k 10 500 python3 bench.py > $OUT/bench.json 2> $OUT/bench.err
echo "bench rc=$?"
