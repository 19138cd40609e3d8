#!/bin/bash
# Round-6 check 26: kernel traces of the 16-city chain with one and with two
# levels fused into the seeds' launch (CHAIN_FUSE_SEEDS 1 / 2).
set -u
cd "$(dirname "$0")/.."
ROOT=$PWD
OUT=$ROOT/gpurun_out/r06/fuse
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
for k in 1 2; do
  SETS_JSON="[{\"CHAIN_FUSE_SEEDS\": $k}]" timeout -k 10 180 rocprofv3 --kernel-trace --output-format csv -d $OUT/trace$k -o k2 -- python3 $ROOT/tools/k2_16_sweep.py 30 > $OUT/trace$k.log 2>&1
  echo "trace $k rc=$?"; python3 $ROOT/tools/k2_trace_summary.py $OUT/trace$k/k2_kernel_trace.csv
done
