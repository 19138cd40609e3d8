#!/bin/bash
set -u
cd "$(dirname "$0")/.."
OUT=$PWD/gpurun_out/r05/k2trace
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT -o k2 -- python3 $GRAFT_REPO_ROOT/tools/k2_trace16.py 40 > $OUT/run.log 2>&1
echo "trace rc=$?"; tail -2 $OUT/run.log
