#!/bin/bash
set -u
cd "$(dirname "$0")/.."
for so in tsp-mpi-reduction_amd/lib_ab/tail_*.so; do
  echo "$(basename $so) $(TSPGPU_LIB=$PWD/$so timeout -k 10 60 python3 tools/k2_chain_ms.py)" || exit 1
done
