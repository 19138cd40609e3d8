#!/bin/bash
# Round-6 check 20: suffix table by a left-fold DP (bit-identical) against the
# enumeration: 16-city chain time and K2 SQ counters, then the K2 GPU tests.

set -u
cd "$(dirname "$0")/.."
OUT=gpurun_out/r06/dp
mkdir -p $OUT
export TMPDIR=/tmp
for r in 1 2 3; do
  for so in tsp-mpi-reduction_amd/lib_ab/base.so tsp-mpi-reduction_amd/lib_ab/dp.so; do
    name=$(basename $so .so)
    DEFAULT_ONLY=1 TSPGPU_LIB=$PWD/$so timeout -k 10 120 python3 -u tools/k2_16_sweep.py 60 > $OUT/$name.r$r.log 2>&1
    echo "$name r$r rc=$? $(tail -1 $OUT/$name.r$r.log)"
  done
done
for so in tsp-mpi-reduction_amd/lib_ab/dp.so; do
  name=$(basename $so .so)
  TSPGPU_LIB=$PWD/$so timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE --output-format csv -d $OUT/pmc_$name -o pmc -- python3 bench.py --pmc-child-k2 > $OUT/pmc_$name.log 2>&1
  echo "pmc $name rc=$?"
  f=$(ls $OUT/pmc_$name/*counter_collection.csv $OUT/pmc_$name/*/*counter_collection.csv 2>/dev/null | head -1)
  [ -n "$f" ] && python3 tools/k2_pmc_split.py $f 2479117 4 > $OUT/split_$name.json && tail -2 $OUT/split_$name.json
done
timeout -k 10 600 python -u -m pytest tests/test_search_gpu.py tests/test_tsplib.py tests/test_search_cli.py -m gpu -x -q --timeout 240 --timeout-method thread > $OUT/tests.log 2>&1; rc=$?; tail -3 $OUT/tests.log; exit $rc
