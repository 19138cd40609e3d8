#!/bin/bash
# `./tsp 16 1 1000 1000` with the previous library (lib_old, runtime copy path)
# and the current one (small transfers through xfer.hip), interleaved, with the
# program's own clock and TSP_STATS phases.
set -u
cd "$(dirname "$0")/.."
OUT=gpurun_out/r05/startup
mkdir -p $OUT; rm -f $OUT/ab.txt
for r in 1 2 3 4 5 6; do
  for v in old new; do
    if [ $v = old ]; then lp=$PWD/tsp-mpi-reduction_amd/lib_old; else lp=; fi
    o=$(LD_LIBRARY_PATH=$lp TSP_STATS=1 timeout -k 10 60 tsp-mpi-reduction_amd/bin/tsp 16 1 1000 1000 2>&1) || { echo "$v failed"; echo "$o"; exit 1; }
    echo "$v $(echo "$o" | grep -E 'TSP ran|tsp stats' | tr '\n' ' ')" >> $OUT/ab.txt
  done
done
cat $OUT/ab.txt
