#!/bin/bash
# HIP API trace of `./tsp 16 1 1000 1000` (round 5 start-up study): every
# runtime call's duration, to find what the first solve pays besides the
# runtime's own initialisation.
set -u
cd "$(dirname "$0")/.."
OUT=gpurun_out/r05/startup
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --hip-trace --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$OUT/trace -o tsp16 -- $GRAFT_REPO_ROOT/tsp-mpi-reduction_amd/bin/tsp 16 1 1000 1000 > $GRAFT_REPO_ROOT/$OUT/tsp16.log 2>&1
echo "trace rc=$?"
