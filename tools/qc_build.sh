#!/bin/bash
# Variants of libtspgpu with the n=16 tiled configs compiled at another
# TSPGPU_TILED_QC / TSPGPU_TILED_AHEAD (timing experiments):
#   tools/qc_build.sh QC AHEAD  -> lib/libtspgpu_qc<QC>_ah<AHEAD>.so
set -e
cd "$(dirname "$0")/../tsp-mpi-reduction_amd"
QC=$1; AH=$2
for c in 2 12; do
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -fPIC -Wall -I../include -Iinclude \
     -fno-honor-nans -mno-amdgpu-ieee -DTSPGPU_TILED_QC=$QC -DTSPGPU_TILED_AHEAD=$AH -c csrc/hkt_c$c.hip -o lib/_qc_c${c}_$QC_$AH.o &
done
wait
objs=$(ls lib/*.o | grep -v "^lib/_" | grep -v "hkt_c2.o\|hkt_c12.o")
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o lib/libtspgpu_qc${QC}_ah${AH}.so $objs lib/_qc_c2_$QC_$AH.o lib/_qc_c12_$QC_$AH.o
rm -f lib/_qc_*.o
