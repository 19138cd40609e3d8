#!/bin/bash
# Round-6 final check 5 (compacted fused level):
# rocprofv3 kernel trace, a plain bench.py line, and a kernel trace of the
# 16-city K2 chain.
set -u
cd "$(dirname "$0")/.."
ROOT=$PWD
OUT=$ROOT/gpurun_out/r06/final5
mkdir -p $OUT
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $OUT/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -2 $OUT/smoke.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > $OUT/gpu_tests.log 2>&1
rc=$?; echo "gpu tests rc=$rc"; tail -3 $OUT/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o bench -- python3 $ROOT/bench.py --steps 5 --warmup 1 > $OUT/bench_prof.json 2> $OUT/bench_prof.err
rc=$?; echo "prof rc=$rc"; [ $rc -eq 0 ] || exit $rc
cd $ROOT
timeout -k 10 500 python3 bench.py > $OUT/bench.json 2> $OUT/bench.err
rc=$?; echo "bench rc=$rc"; tail -c 400 $OUT/bench.json; [ $rc -eq 0 ] || exit $rc
cd /tmp
timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/k2trace -o k2 -- python3 $ROOT/tools/k2_trace16.py 40 > $OUT/k2trace_run.log 2>&1
echo "k2 trace rc=$?"; cd $ROOT; f=$(ls $OUT/k2trace/*/k2_kernel_trace.csv $OUT/k2trace/k2_kernel_trace.csv 2>/dev/null | head -1); python3 tools/k2_trace_summary.py $f > $OUT/k2_16city_chain.txt; cat $OUT/k2_16city_chain.txt | head -12
