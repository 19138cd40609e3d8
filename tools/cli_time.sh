#!/bin/bash
# End-to-end drop-in timings (bin/tsp): GPU merges (K3) vs the host replay.
set -u
cd "$(dirname "$0")/.."
T=tsp-mpi-reduction_amd/bin/tsp
for args in "16 64 1000 1000" "16 1024 1000 1000"; do
  for P in 1 8; do
    echo "== ./tsp $args P=$P GPU-merge"; TSP_NPROCS=$P timeout -k 5 300 $T $args | tail -1 || exit $?
    echo "== ./tsp $args P=$P host-merge"; TSP_NPROCS=$P TSP_HOST_MERGE=1 timeout -k 5 300 $T $args | tail -1 || exit $?
  done
done
for args in "16 4096 1000 1000" "16 16384 1000 1000"; do
  for P in 1 8; do
    echo "== ./tsp $args P=$P GPU-merge"; TSP_NPROCS=$P timeout -k 5 300 $T $args | tail -1 || exit $?
  done
done
