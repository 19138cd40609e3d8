#!/bin/bash
# Round-6 check 28: bench.py line after counting prologue1_kernel in the K2
# counter pass (the fused first level).
set -u
cd "$(dirname "$0")/.."
OUT=gpurun_out/r06/final3
mkdir -p $OUT
timeout -k 10 500 python3 bench.py > $OUT/bench.json 2> $OUT/bench.err
rc=$?; echo "bench rc=$rc"; tail -c 300 $OUT/bench.json; exit $rc
