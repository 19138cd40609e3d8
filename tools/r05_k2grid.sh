#!/bin/bash
# chained tail grid sweep (workgroups per CU) on the 16- and 32-city K2 instances
set -u
cd "$(dirname "$0")/.."
for g in 8 2 1 4; do
  echo "tail_grid $g"; TSPGPU_CHAIN_TAIL_GRID=$g timeout -k 10 120 python3 tools/k2_solve_time.py 20 || exit 1
done
