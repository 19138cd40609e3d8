#!/bin/bash
# A/B variant of libtspgpu for any one kernel translation unit (development
# aid, CPU side): csrc/SRC.hip recompiled with extra -D flags (kernel flags),
# linked with the tree's other objects into tsp-mpi-reduction_amd/lib_ab/NAME.so
#   bash tools/ab_build_obj.sh NAME SRC "-DFOO=1"      (e.g. SRC = enum)
set -eu
cd "$(dirname "$0")/../tsp-mpi-reduction_amd"
NAME=$1; SRC=$2; FLAGS=${3:-}
mkdir -p lib_ab/obj
make -s lib/libtspgpu.so
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -fPIC -Wall -I../include -Iinclude -Icsrc \
    -fno-honor-nans -mno-amdgpu-ieee $FLAGS -c csrc/$SRC.hip -o lib_ab/obj/$NAME.o
objs=$(ls lib/*.o lib/k1/*.o lib/k1l/*.o | grep -v "^lib/$SRC.o$")
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o lib_ab/$NAME.so $objs lib_ab/obj/$NAME.o
echo "built lib_ab/$NAME.so ($SRC.hip $FLAGS)"
