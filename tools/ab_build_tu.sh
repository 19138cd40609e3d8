#!/bin/bash
# A/B variant of libtspgpu with ONE translation unit recompiled with extra -D
# flags (development aid): lib_ab/NAME.so, picked by the Python tools via
# TSPGPU_LIB.   bash tools/ab_build_tu.sh NAME TU "-DFOO=1"   (TU e.g. enum)
set -eu
cd "$(dirname "$0")/../tsp-mpi-reduction_amd"
NAME=$1; TU=$2; FLAGS=${3:-}
mkdir -p lib_ab/obj
make -s lib/libtspgpu.so
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -fPIC -Wall -I../include -Iinclude -Icsrc \
    -fno-honor-nans -mno-amdgpu-ieee $FLAGS -c csrc/$TU.hip -o lib_ab/obj/$NAME.o
objs=$(ls lib/*.o lib/k1/*.o | grep -v "lib/$TU.o")
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o lib_ab/$NAME.so $objs lib_ab/obj/$NAME.o
echo "built lib_ab/$NAME.so ($TU: $FLAGS)"
