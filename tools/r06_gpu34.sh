#!/bin/bash
# Round-6 check 34: the tail kernel's queue carrying the prefixes' words (one read
# (tq) against the product (base): K2 GPU tests on tq, then the 16-city
# search alternating, then a kernel trace of each.
set -u
cd "$(dirname "$0")/.."
ROOT=$PWD
OUT=$ROOT/gpurun_out/r06/tq
mkdir -p $OUT
TSPGPU_LIB=$ROOT/tsp-mpi-reduction_amd/lib_ab/tq.so timeout -k 10 600 python -u -m pytest tests/test_search_gpu.py tests/test_tsplib.py tests/test_search_cli.py -m gpu -x -q --timeout 240 --timeout-method thread > $OUT/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 $OUT/tests.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2 3; do
  for name in base tq; do
    DEFAULT_ONLY=1 TSPGPU_LIB=$ROOT/tsp-mpi-reduction_amd/lib_ab/$name.so timeout -k 10 120 python3 -u tools/k2_16_sweep.py 60 > $OUT/$name.r$r.log 2>&1
    echo "$name r$r rc=$? $(tail -1 $OUT/$name.r$r.log)"
  done
done
cd /tmp && export TMPDIR=/tmp
for name in base tq; do
  DEFAULT_ONLY=1 TSPGPU_LIB=$ROOT/tsp-mpi-reduction_amd/lib_ab/$name.so timeout -k 10 180 rocprofv3 --kernel-trace --output-format csv -d $OUT/trace_$name -o k2 -- python3 $ROOT/tools/k2_16_sweep.py 20 > $OUT/trace_$name.log 2>&1
  echo "trace $name rc=$?"; python3 $ROOT/tools/k2_trace_summary.py $OUT/trace_$name/k2_kernel_trace.csv
done
