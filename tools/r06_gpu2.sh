#!/bin/bash
# Round-6 check 2: the pair-form backtracking recompute (hk_tiled.h) against
# the K1 GPU suite, its timing at 65536 blocks, and the K2 host/device split.
set -u
cd "$(dirname "$0")/.."
OUT=gpurun_out/r06/gpu2
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_k1_variants_gpu.py tests/test_i32_gpu.py tests/test_tsplib.py -x -q --timeout 240 --timeout-method thread > $OUT/k1_tests.log 2>&1
rc=$?; echo "k1 tests rc=$rc"; tail -3 $OUT/k1_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 -u tools/k1_time.py 16 65536 8 6 > $OUT/k1_time_65536.log 2>&1
echo "k1 time rc=$?"; tail -1 $OUT/k1_time_65536.log
timeout -k 10 300 python3 -u tools/k1_time.py 16 65536 4 6 > $OUT/k1_time_65536_i32.log 2>&1
echo "k1 i32 time rc=$?"; tail -1 $OUT/k1_time_65536_i32.log
timeout -k 10 300 python3 tools/k2_sharded_phases.py > $OUT/k2_phases.json 2> $OUT/k2_phases.err
echo "k2 phases rc=$?"; cat $OUT/k2_phases.json
timeout -k 10 600 python3 tools/startup_split_probe.py > $OUT/startup_split_probe.json 2>&1
echo "startup probe rc=$?"; cat $OUT/startup_split_probe.json
