#!/bin/bash
# Build timing variants of libtspgpu: hkt_c$CFG (default 14 = the n=16 default
# configuration) and tspgpu.cpp (which sizes the slots) compiled with extra
# flags, as lib/libtspgpu_abl<name>.so.
#   abl_build.sh NAME:FLAGS ...   e.g. 8:-DTSPGPU_TILED_ABL=8 ta2:-DTSPGPU_TILED_TA_OFF=2
# (a bare number N means -DTSPGPU_TILED_ABL=N; ablated results are WRONG, timing only)
set -e
cd "$(dirname "$0")/../tsp-mpi-reduction_amd"
C=${CFG:-14}
F="--offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -fPIC -Wall -I../include -Iinclude"
for a in "$@"; do
  name=${a%%:*}; flags=${a#*:}; [ "$name" = "$a" ] && flags="-DTSPGPU_TILED_ABL=$a"
  /opt/rocm/bin/hipcc $F -fno-honor-nans -mno-amdgpu-ieee $flags -c csrc/hkt_c$C.hip -o lib/_abl_c_$name.o &
  /opt/rocm/bin/hipcc $F -fno-builtin-pow $flags -c csrc/tspgpu.cpp -o lib/_abl_t_$name.o &
done
wait
for a in "$@"; do
  name=${a%%:*}
  objs=$(ls lib/*.o | grep -v "_abl_" | grep -v "hkt_c$C.o" | grep -v "lib/tspgpu.o")
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o lib/libtspgpu_abl$name.so $objs lib/_abl_c_$name.o lib/_abl_t_$name.o
done
rm -f lib/_abl_*.o
