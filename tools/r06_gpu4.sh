#!/bin/bash
# Round-6 check 4: K2 device bound vs host multi-start (sharded + native), and
# the backtracking A/B (member values in two halves vs all at once).
set -u
cd "$(dirname "$0")/.."
OUT=gpurun_out/r06/gpu4
mkdir -p $OUT
timeout -k 10 400 python3 tools/k2_sharded_phases.py > $OUT/k2_phases.json 2> $OUT/k2_phases.err
echo "k2 phases rc=$?"; cat $OUT/k2_phases.json; tail -3 $OUT/k2_phases.err
OUT=gpurun_out/r06/ab_bt2 ROUNDS=2 timeout -k 10 600 bash tools/ab_time.sh
echo "ab rc=$?"
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_k1_variants_gpu.py tests/test_i32_gpu.py -x -q --timeout 240 --timeout-method thread > $OUT/k1_tests.log 2>&1
rc=$?; echo "k1 tests rc=$rc"; tail -2 $OUT/k1_tests.log
