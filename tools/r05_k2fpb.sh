#!/bin/bash
# chained expand: paths per block (CHAIN_FPB) and blocks per CU (CHAIN_GRID)
set -u
cd "$(dirname "$0")/.."
for v in "256 2" "128 2" "128 4" "64 4" "64 8" "512 1"; do
  set -- $v
  echo "fpb $1 grid $2 $(TSPGPU_CHAIN_FPB=$1 TSPGPU_CHAIN_GRID=$2 timeout -k 10 60 python3 tools/k2_chain_ms.py)" || exit 1
done
