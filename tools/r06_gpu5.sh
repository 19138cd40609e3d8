#!/bin/bash
# Round-6 check 5: per-kernel layer units (csrc/k1l) — the whole GPU suite,
# the start-up probe, and a bench line.
set -u
cd "$(dirname "$0")/.."
OUT=gpurun_out/r06/gpu5
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > $OUT/gpu_tests.log 2>&1
rc=$?; echo "gpu tests rc=$rc"; tail -3 $OUT/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python3 tools/startup_split_probe.py > $OUT/startup_split_probe.json 2>&1
echo "startup probe rc=$?"; cat $OUT/startup_split_probe.json
timeout -k 10 500 python3 bench.py > $OUT/bench.json 2> $OUT/bench.err
echo "bench rc=$?"; tail -c 300 $OUT/bench.json
