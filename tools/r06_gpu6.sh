#!/bin/bash
# Round-6 check 6: the 16-city K2 chain — knob sweep and a rocprofv3 kernel trace.
set -u
cd "$(dirname "$0")/.."
ROOT=$PWD
OUT=$ROOT/gpurun_out/r06/k2_16
mkdir -p $OUT
timeout -k 10 300 python3 tools/k2_16_sweep.py 30 > $OUT/sweep.json 2> $OUT/sweep.err
echo "sweep rc=$?"; cat $OUT/sweep.json; tail -3 $OUT/sweep.err
cd /tmp && export TMPDIR=/tmp
timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o k2 -- python3 $ROOT/tools/k2_trace16.py 40 > $OUT/trace_run.log 2>&1
echo "trace rc=$?"; cd $ROOT; f=$(ls $OUT/trace/*/k2_kernel_trace.csv $OUT/trace/k2_kernel_trace.csv 2>/dev/null | head -1); echo "$f"; python3 tools/k2_trace_summary.py $f | head -20
