#!/bin/bash
# K2 frontier-step size knobs on large random instances (development aid):
#   gpurun -- 'bash tools/k2_knob_sweep.sh'   -> gpurun_out/k2_knobs.log
set -u
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
OUT=gpurun_out/k2_knobs.log
mkdir -p gpurun_out
: > $OUT
for knobs in "23 21" "25 21" "25 23" "26 24"; do
    set -- $knobs
    echo "== TSPGPU_SEARCH_TAIL_CAP_LOG2=$1 TSPGPU_SEARCH_EXPAND_LOG2=$2" >> $OUT
    TSPGPU_SEARCH_TAIL_CAP_LOG2=$1 TSPGPU_SEARCH_EXPAND_LOG2=$2 timeout -k 10 150 \
        python -u tools/k2_size_probe.py 28 30 32 --seeds=2 >> $OUT 2>&1 || { echo "stop rc=$?" >> $OUT; break; }
done
cat $OUT
