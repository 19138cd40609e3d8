#!/bin/bash
# Start-up probes (round 5): tools/init_probe4.cpp in both modes, three
# processes each, and the program clock of `./tsp 16 1` five times.
set -u
cd "$(dirname "$0")/.."
OUT=gpurun_out/r05/startup
mkdir -p $OUT
for r in 1 2 3; do
  for m in raw lib; do timeout -k 10 60 tsp-mpi-reduction_amd/bin/init_probe4 $m >> $OUT/probe4.txt 2>&1 || exit 1; done
done
for r in 1 2 3 4 5; do timeout -k 10 60 tsp-mpi-reduction_amd/bin/tsp 16 1 1000 1000 | tail -1 >> $OUT/tsp16_clock.txt || exit 1; done
cat $OUT/probe4.txt $OUT/tsp16_clock.txt
