#!/bin/bash
# Round-5 GPU check: the whole GPU suite (one process), then the start-up probes.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/r05
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/r05/gpu_tests_full.log 2>&1
rc=$?; echo "gpu tests rc=$rc"; tail -5 gpurun_out/r05/gpu_tests_full.log
[ $rc -eq 0 ] || exit $rc
rm -f gpurun_out/r05/startup/probe4.txt gpurun_out/r05/startup/tsp16_clock.txt
bash tools/r05_startup2.sh
