#!/bin/bash
# GPU side of tools/ab_build.sh: every lib_ab/*.so (and the tree's own lib)
# timed on K1 n = 16 f64, 16384 blocks, in ROUNDS interleaved rounds
# (one process per library per round; bit-exactness vs variant 5 reported).
set -u
cd "$(dirname "$0")/.."
OUT=${OUT:-gpurun_out/r05/ab}
mkdir -p $OUT
N=${N:-16}; VB=${VB:-8}
for r in $(seq 1 ${ROUNDS:-2}); do
    for so in tsp-mpi-reduction_amd/lib/libtspgpu.so tsp-mpi-reduction_amd/lib_ab/*.so; do
        name=$(basename $so .so)
        wg=$(echo $name | sed -n 's/.*_wg\([0-9]\).*/\1/p')  # NAME_wgK: a build for K workgroups per CU
        TSPGPU_WG_PER_CU=${wg:-0} TSPGPU_LIB=$PWD/$so timeout -k 10 120 python3 -u tools/k1_time.py $N 16384 $VB 6 > $OUT/$name.r$r.log 2>&1 || { echo "$name failed"; tail -5 $OUT/$name.r$r.log; exit 1; }
        echo "$name r$r $(tail -1 $OUT/$name.r$r.log)"
    done
done
