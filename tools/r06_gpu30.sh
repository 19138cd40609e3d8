#!/bin/bash
# Round-6 check 30: a level block folding its own few tail children (tail_wide_w
# in expand_kernel, knob CHAIN_TAIL_INBLOCK): K2 GPU tests, then the 16-city
# search against CHAIN_TAIL_INBLOCK=0.
set -u
cd "$(dirname "$0")/.."
OUT=gpurun_out/r06/tailin
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_search_gpu.py tests/test_tsplib.py tests/test_search_cli.py tests/test_rccl_gpu.py tests/test_search_dist.py -m gpu -x -q --timeout 240 --timeout-method thread > $OUT/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 $OUT/tests.log; [ $rc -eq 0 ] || exit $rc
SETS_JSON='[{}, {"CHAIN_TAIL_INBLOCK": 0}, {}, {"CHAIN_TAIL_INBLOCK": 0}, {}, {"CHAIN_TAIL_INBLOCK": 0}]' timeout -k 10 300 python3 tools/k2_16_sweep.py 60 > $OUT/sweep.json 2> $OUT/sweep.err
echo "sweep rc=$?"; cat $OUT/sweep.json


