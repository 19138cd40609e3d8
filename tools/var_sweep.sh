#!/bin/bash
# A/B timing of libtspgpu variants (tools/var_build.sh) on one tiled config:
# parity vs the oracle + time per 16384-block launch, each library in its own
# process, the default library first.  Every step has its own time limit and a
# failure ends the script.
#   gpurun -- 'bash tools/var_sweep.sh CFG NAME ...'   (NAME = lib/libtspgpu_NAME.so)
set -u
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
CFG=$1
shift
OUT=gpurun_out/var_sweep.log
mkdir -p gpurun_out
: > $OUT
for name in default "$@"; do
    lib=tsp-mpi-reduction_amd/lib/libtspgpu_$name.so
    [ "$name" = default ] && lib=tsp-mpi-reduction_amd/lib/libtspgpu.so
    echo "== $name" >> $OUT
    TSPGPU_LIB=$PWD/$lib timeout -k 10 120 python -u tools/k1_tiled_check.py 16384 $CFG >> $OUT 2>&1 || { echo "stop after $name rc=$?" >> $OUT; cat $OUT; exit 1; }
done
cat $OUT
