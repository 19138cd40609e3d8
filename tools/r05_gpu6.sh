#!/bin/bash
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/r05
ROUNDS=${ROUNDS:-2} OUT=gpurun_out/r05/ab6 timeout -k 10 300 bash tools/ab_time.sh > gpurun_out/r05/ab6.txt 2>&1; echo ab rc=$?
python3 - <<'PY'
import json
for l in open("gpurun_out/r05/ab6.txt"):
    name, rd, js = l.split(" ", 2)
    try:
        d = json.loads(js)
        print(name, rd, "fwd %.3f" % d["forward_ms"], "bt %.3f" % d["backtrack_ms"], "same", d["same_as_v5"])
    except Exception:
        print(l[:200])
PY
for so in tsp-mpi-reduction_amd/lib_ab/stamp*.so; do
  TSPGPU_LIB=$PWD/$so timeout -k 10 120 python3 tools/k1_stamp.py 16 16384 >> gpurun_out/r05/stamp6.txt 2>&1 || { echo "stamp $so failed"; tail -3 gpurun_out/r05/stamp6.txt; exit 1; }
done
cat gpurun_out/r05/stamp6.txt
