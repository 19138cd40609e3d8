#!/bin/bash
# A/B variant of libtspgpu (development aid, CPU side): the n = 16 f64 K1
# configuration (csrc/k1/hks_p60.hip) recompiled with extra -D flags, linked
# with the tree's other objects into tsp-mpi-reduction_amd/lib_ab/NAME.so
# (git-ignored; travels to the GPU box; tools/k1_time.py picks it via TSPGPU_LIB).
#   bash tools/ab_build.sh NAME "-DFOO=1 -DBAR=0" [CFG]   (CFG: the configuration file, default hks_p60;
#   hks_p61 = n = 16 i32)
set -eu
cd "$(dirname "$0")/../tsp-mpi-reduction_amd"
NAME=$1; FLAGS=${2:-}; CFG=${3:-hks_p60}
mkdir -p lib_ab/obj
make -s lib/libtspgpu.so
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -fPIC -Wall -I../include -Iinclude -Icsrc \
    -fno-honor-nans -mno-amdgpu-ieee $FLAGS -c csrc/k1/$CFG.hip -o lib_ab/obj/$NAME.o
objs=$(ls lib/*.o lib/k1/*.o lib/k1l/*.o | grep -v "k1/$CFG.o")
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o lib_ab/$NAME.so $objs lib_ab/obj/$NAME.o
echo "built lib_ab/$NAME.so ($FLAGS)"
