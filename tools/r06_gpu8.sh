#!/bin/bash
# Round-6 check 8: the certificate's prefix minima from the optimal records
# (tspgpu_tie_tour_records; native search_solve and the one-rank sharded
# solve) — the K2 GPU tests and the host/device split again.
set -u
cd "$(dirname "$0")/.."
OUT=gpurun_out/r06/gpu8
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_search_gpu.py tests/test_rccl_gpu.py tests/test_search_dist.py tests/test_search_cli.py tests/test_tsplib.py -x -q --timeout 240 --timeout-method thread > $OUT/k2_tests.log 2>&1
rc=$?; echo "k2 tests rc=$rc"; tail -3 $OUT/k2_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python3 tools/k2_sharded_phases.py > $OUT/k2_phases.json 2> $OUT/k2_phases.err
echo "k2 phases rc=$?"; cat $OUT/k2_phases.json; tail -3 $OUT/k2_phases.err
