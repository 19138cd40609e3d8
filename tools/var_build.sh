#!/bin/bash
# A libtspgpu variant with the n=16 tiled configs (2, 12) compiled with extra
# -D flags (timing experiments):  tools/var_build.sh NAME "-DFOO=1 -DBAR=2" [cfg ...]
#   -> lib/libtspgpu_NAME.so  (configs: default 2 12 14)
set -e
cd "$(dirname "$0")/../tsp-mpi-reduction_amd"
NAME=$1; FLAGS=$2; shift 2 || true
CFGS=${*:-2 12 14}
for c in $CFGS; do
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -fPIC -Wall -I../include -Iinclude \
     -fno-honor-nans -mno-amdgpu-ieee $FLAGS -c csrc/hkt_c$c.hip -o lib/_v_${NAME}_c$c.o &
done
wait
skip=$(for c in $CFGS; do printf '%s\\|' "hkt_c$c.o"; done)
objs=$(ls lib/*.o | grep -v "^lib/_" | grep -v "${skip%\\|}")
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o lib/libtspgpu_$NAME.so $objs lib/_v_${NAME}_c*.o 2>&1 | grep -v hip-link || true
rm -f lib/_v_${NAME}_*.o
