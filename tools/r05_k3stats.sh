#!/bin/bash
# rocprofv3 kernel stats (csv) of the merge-dominated ./tsp 8 1024 1000 1000 at P = 8
set -u
cd "$(dirname "$0")/.."
OUT=$PWD/gpurun_out/r05/k3stats
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
TSP_NPROCS=8 TSP_STATS=1 timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT -o k3 -- $GRAFT_REPO_ROOT/tsp-mpi-reduction_amd/bin/tsp 8 1024 1000 1000 > $OUT/run.log 2>&1
echo "trace rc=$?"; grep -E "tsp stats|TSP ran" $OUT/run.log
