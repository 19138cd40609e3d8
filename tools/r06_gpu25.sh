#!/bin/bash
# Round-6 check 25: the chain's first level fused into the seeds' launch
# (prologue1_kernel, knob CHAIN_FUSE_SEEDS: 2 = two levels, 1 = one, 0 = none):
# search fused / unfused alternating (in-process and kernel time, nodes).
set -u
cd "$(dirname "$0")/.."
OUT=gpurun_out/r06/fuse
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_search_gpu.py tests/test_tsplib.py tests/test_search_cli.py tests/test_rccl_gpu.py tests/test_search_dist.py -m gpu -x -q --timeout 240 --timeout-method thread > $OUT/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 $OUT/tests.log; [ $rc -eq 0 ] || exit $rc
SETS_JSON='[{}, {"CHAIN_FUSE_SEEDS": 1}, {"CHAIN_FUSE_SEEDS": 0}, {}, {"CHAIN_FUSE_SEEDS": 1}, {"CHAIN_FUSE_SEEDS": 0}]' timeout -k 10 300 python3 tools/k2_16_sweep.py 60 > $OUT/sweep.json 2> $OUT/sweep.err
echo "sweep rc=$?"; cat $OUT/sweep.json
