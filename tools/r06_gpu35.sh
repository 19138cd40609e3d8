#!/bin/bash
# Round-6 check 35: smaller read groups in expand_eval (remaining-set sums 4,
# children 2: lite) against 8 / 4 (base): K2 GPU tests on lite, the 16-city
# search alternating, and the K2 counter split of each (VALU per node).
set -u
cd "$(dirname "$0")/.."
ROOT=$PWD
OUT=$ROOT/gpurun_out/r06/lite
mkdir -p $OUT
TSPGPU_LIB=$ROOT/tsp-mpi-reduction_amd/lib_ab/lite.so timeout -k 10 600 python -u -m pytest tests/test_search_gpu.py tests/test_tsplib.py tests/test_search_cli.py -m gpu -x -q --timeout 240 --timeout-method thread > $OUT/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 $OUT/tests.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2 3; do
  for name in base lite; do
    DEFAULT_ONLY=1 TSPGPU_LIB=$ROOT/tsp-mpi-reduction_amd/lib_ab/$name.so timeout -k 10 120 python3 -u tools/k2_16_sweep.py 60 > $OUT/$name.r$r.log 2>&1
    echo "$name r$r rc=$? $(tail -1 $OUT/$name.r$r.log)"
  done
done
cd /tmp && export TMPDIR=/tmp
for name in base lite; do
  TSPGPU_LIB=$ROOT/tsp-mpi-reduction_amd/lib_ab/$name.so timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE --output-format csv -d $OUT/pmc_$name -o pmc -- python3 $ROOT/bench.py --pmc-child-k2 > $OUT/pmc_$name.log 2>&1
  echo "pmc $name rc=$?"
  python3 $ROOT/tools/k2_pmc_split.py $OUT/pmc_$name/pmc_counter_collection.csv 2479117 4 > $OUT/split_$name.json && python3 -c "
import json;d=json.load(open('$OUT/split_$name.json'));print('$name', {k:round(v['valu_lane_instructions_per_node'],2) for k,v in d.items() if isinstance(v,dict)}, round(d['total_valu_lane_instructions_per_node'],2))"
done
