#!/bin/bash
# Round-6 check 24: the init launch reading the heuristic's distances in the
# same PCIe round trip as its table copies (hv) against the previous build:
# in-process and kernel time of the 16-city search, 3 alternating rounds,
# then the init kernel's duration in a kernel trace of each.
set -u
cd "$(dirname "$0")/.."
ROOT=$PWD
OUT=$ROOT/gpurun_out/r06/hv
mkdir -p $OUT
for r in 1 2 3; do
  for so in tsp-mpi-reduction_amd/lib_ab/base.so tsp-mpi-reduction_amd/lib_ab/hv.so; do
    name=$(basename $so .so)
    DEFAULT_ONLY=1 TSPGPU_LIB=$ROOT/$so timeout -k 10 120 python3 -u tools/k2_16_sweep.py 60 > $OUT/$name.r$r.log 2>&1
    echo "$name r$r rc=$? $(tail -1 $OUT/$name.r$r.log)"
  done
done
cd /tmp && export TMPDIR=/tmp
for name in base hv; do
  DEFAULT_ONLY=1 TSPGPU_LIB=$ROOT/tsp-mpi-reduction_amd/lib_ab/$name.so timeout -k 10 180 rocprofv3 --kernel-trace --output-format csv -d $OUT/trace_$name -o k2 -- python3 $ROOT/tools/k2_16_sweep.py 20 > $OUT/trace_$name.log 2>&1
  echo "trace $name rc=$?"; python3 $ROOT/tools/k2_trace_summary.py $OUT/trace_$name/k2_kernel_trace.csv | grep init
done
