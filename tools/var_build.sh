#!/bin/bash
# A libtspgpu variant with the n=16 tiled configs (2, 12) compiled with extra
# -D flags (timing experiments):  tools/var_build.sh NAME "-DFOO=1 -DBAR=2"
#   -> lib/libtspgpu_NAME.so
set -e
cd "$(dirname "$0")/../tsp-mpi-reduction_amd"
NAME=$1; FLAGS=$2
for c in 2 12; do
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -fPIC -Wall -I../include -Iinclude \
     -fno-honor-nans -mno-amdgpu-ieee $FLAGS -c csrc/hkt_c$c.hip -o lib/_v_${NAME}_c$c.o &
done
wait
objs=$(ls lib/*.o | grep -v "^lib/_" | grep -v "hkt_c2.o\|hkt_c12.o")
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o lib/libtspgpu_$NAME.so $objs lib/_v_${NAME}_c2.o lib/_v_${NAME}_c12.o 2>&1 | grep -v hip-link || true
rm -f lib/_v_${NAME}_*.o
