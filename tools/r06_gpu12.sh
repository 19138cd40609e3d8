#!/bin/bash
# Round-6 check 12 (timing only): does the slot working set matter?  The
# forward kernel with each block's push/parent slot reused modulo 1536 (one
# slot per resident workgroup: 2.5 GB instead of 108 GB per 65536-block
# launch) or 6144, against the product; tours of the A/B builds are wrong
# (the backtracking reads overwritten slots), the forward times are valid.
set -u
cd "$(dirname "$0")/.."
OUT=gpurun_out/r06/slotmod
mkdir -p $OUT
for r in 1 2; do
  for so in tsp-mpi-reduction_amd/lib/libtspgpu.so tsp-mpi-reduction_amd/lib_ab/slotmod1536.so tsp-mpi-reduction_amd/lib_ab/slotmod6144.so; do
    name=$(basename $so .so)
    TSPGPU_LIB=$PWD/$so timeout -k 10 200 python3 -u tools/k1_time.py 16 65536 8 6 > $OUT/$name.r$r.log 2>&1
    echo "$name r$r rc=$? $(tail -1 $OUT/$name.r$r.log)"
  done
done
