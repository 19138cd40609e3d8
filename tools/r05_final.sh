#!/bin/bash
# Round-5 closing measurement: bench.py under rocprofv3 kernel trace (the
# kernel stats the line's roofline is checked against), then a plain bench.py.
set -u
cd "$(dirname "$0")/.."
OUT=$PWD/gpurun_out/r05/final
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o bench -- python3 $GRAFT_REPO_ROOT/bench.py --steps 5 --warmup 1 > $OUT/bench_prof.json 2> $OUT/bench_prof.err
echo "prof rc=$?"
cd $GRAFT_REPO_ROOT
timeout -k 10 500 python3 bench.py > $OUT/bench.json 2> $OUT/bench.err
echo "bench rc=$?"; tail -c 400 $OUT/bench.json
