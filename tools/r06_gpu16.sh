#!/bin/bash
# Round-6 check 16: the 16-city chain with expand_kernel's first-run paths
# read beside the set-up and kept for pass 2 (TSPGPU_EXPAND_PRE) against the
# product, three alternating rounds of 60 searches each.
set -u
cd "$(dirname "$0")/.."
OUT=gpurun_out/r06/pre
mkdir -p $OUT
for r in 1 2 3; do
  for so in tsp-mpi-reduction_amd/lib/libtspgpu.so tsp-mpi-reduction_amd/lib_ab/pre.so; do
    name=$(basename $so .so)
    DEFAULT_ONLY=1 TSPGPU_LIB=$PWD/$so timeout -k 10 120 python3 -u tools/k2_16_sweep.py 60 > $OUT/$name.r$r.log 2>&1
    echo "$name r$r rc=$? $(tail -1 $OUT/$name.r$r.log)"
  done
done
