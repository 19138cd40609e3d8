#!/bin/bash
# Round-6 check 14: K1 i32 at 16 cities computed in f32 (v_pk_add_f32 member
# pairs + v_min3_f32, exact below 2^24) against the i32 product kernel,
# 65536 blocks; bit-exact check against variant 5 (i32) in the tool.
set -u
cd "$(dirname "$0")/.."
OUT=gpurun_out/r06/f32
mkdir -p $OUT
for r in 1 2; do
  for so in tsp-mpi-reduction_amd/lib/libtspgpu.so tsp-mpi-reduction_amd/lib_ab/f32.so; do
    name=$(basename $so .so)
    TSPGPU_LIB=$PWD/$so timeout -k 10 200 python3 -u tools/k1_time.py 16 65536 4 6 > $OUT/$name.r$r.log 2>&1
    echo "$name r$r rc=$? $(tail -1 $OUT/$name.r$r.log)"
  done
done
