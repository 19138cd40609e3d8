#!/bin/bash
# Round-6 check 15: counters of the K1 i32 forward kernel, i32 product vs the
# f32 member-pair build (first two passes only: instruction mix and busy time).
set -u
cd "$(dirname "$0")/.."
bash tools/k1_pmc_r06.sh i32 "hk_sub_kernel<int" 6 16 4096 4 && \
bash tools/k1_pmc_r06.sh f32 "hk_sub_kernel<float" 6 16 4096 4 tsp-mpi-reduction_amd/lib_ab/f32.so
