#!/bin/bash
# Round-6 first GPU check after removing the losing experiments from the
# product kernels (hk_sub.h, hk_tiled.h, enum.hip) and the per-device slot
# pools (xfer.hip): smoke, the whole GPU suite once, bench.py under a
# rocprofv3 kernel trace, then a plain bench.py line.
set -u
cd "$(dirname "$0")/.."
ROOT=$PWD
OUT=$ROOT/gpurun_out/r06/gpu1
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
echo "bench rc=$?"; tail -c 600 $OUT/bench.json
# K1 A/B: next pass's push loads issued before this pass's push stores (TSPGPU_SUB_PF=1)
OUT=gpurun_out/r06/ab_pf ROUNDS=2 timeout -k 10 600 bash tools/ab_time.sh
echo "ab rc=$?"
# K2: host/device split of the sharded solve at N = 1 (32-city seed 35, 16-city golden)
timeout -k 10 300 python3 tools/k2_sharded_phases.py > gpurun_out/r06/gpu1/k2_phases.json 2> gpurun_out/r06/gpu1/k2_phases.err
echo "k2 phases rc=$?"; cat gpurun_out/r06/gpu1/k2_phases.json
