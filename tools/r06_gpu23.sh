#!/bin/bash
# Round-6 check 23: the 16-city search with the device heuristic's 2-opt
# bounded (SEARCH_HEUR_ITERS 0 = nearest neighbour only, 2, 4, 8, default
# 8 n): in-process time, kernel time, nodes; and a kernel trace of the init
# launch at the default and at 0.
set -u
cd "$(dirname "$0")/.."
ROOT=$PWD
OUT=$ROOT/gpurun_out/r06/heur
mkdir -p $OUT
SETS_JSON='[{}, {"SEARCH_HEUR_ITERS": 0}, {"SEARCH_HEUR_ITERS": 2}, {"SEARCH_HEUR_ITERS": 4}, {"SEARCH_HEUR_ITERS": 8}, {}]' timeout -k 10 300 python3 tools/k2_16_sweep.py 60 > $OUT/sweep.json 2> $OUT/sweep.err
echo "sweep rc=$?"; cat $OUT/sweep.json
cd /tmp && export TMPDIR=/tmp
SETS_JSON='[{"SEARCH_HEUR_ITERS": 0}]' timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o k2 -- python3 $ROOT/tools/k2_16_sweep.py 20 > $OUT/trace_run.log 2>&1
echo "trace rc=$?"
