#!/bin/bash
# Build ablation variants of libtspgpu (hkt_c2 = the n=16 default config compiled
# with -DTSPGPU_TILED_ABL=<mask>) as lib/libtspgpu_abl<mask>.so (timing only).
set -e
cd "$(dirname "$0")/../tsp-mpi-reduction_amd"
for m in "$@"; do
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -fPIC -Wall -I../include -Iinclude \
     -fno-honor-nans -mno-amdgpu-ieee -DTSPGPU_TILED_ABL=$m -c csrc/hkt_c2.hip -o lib/_abl_c2_$m.o &
done
wait
for m in "$@"; do
  objs=$(ls lib/*.o | grep -v "_abl_" | grep -v "hkt_c2.o")
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o lib/libtspgpu_abl$m.so $objs lib/_abl_c2_$m.o
done
