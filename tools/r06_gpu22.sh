#!/bin/bash
# Round-6 check 22: K1-wide (one instance over the whole GPU) at n = 26 and 28:
# kernel time, then FETCH_SIZE and WRITE_SIZE of the push kernels (separate
# rocprofv3 passes) against the algorithmic table bytes.
set -u
cd "$(dirname "$0")/.."
OUT=$PWD/gpurun_out/r06/wide
mkdir -p $OUT
timeout -k 10 300 python3 tools/wide_time.py 24 26 28 > $OUT/time.txt 2>&1; echo "time rc=$?"; cat $OUT/time.txt
cd /tmp && export TMPDIR=/tmp
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 120 rocprofv3 --pmc $c --output-format csv -d $OUT/pmc_$c -o pmc -- python3 $OLDPWD/tools/wide_time.py 28 > $OUT/pmc_$c.log 2>&1
  echo "pmc $c rc=$?"
done
