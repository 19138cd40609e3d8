#!/bin/bash
# Round-6 last check: smoke and the whole GPU suite on the final library.
set -u
cd "$(dirname "$0")/.."
OUT=gpurun_out/r06/last
mkdir -p $OUT
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $OUT/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -2 $OUT/smoke.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > $OUT/gpu_tests.log 2>&1
rc=$?; echo "gpu tests rc=$rc"; tail -3 $OUT/gpu_tests.log; exit $rc
