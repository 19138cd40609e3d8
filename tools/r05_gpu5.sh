#!/bin/bash
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/r05
ROUNDS=2 OUT=gpurun_out/r05/ab5 timeout -k 10 300 bash tools/ab_time.sh > gpurun_out/r05/ab5.txt 2>&1; echo ab rc=$?
python3 - <<'PY'
import json
for l in open("gpurun_out/r05/ab5.txt"):
    name, rd, js = l.split(" ", 2)
    try:
        d = json.loads(js)
        print(name, rd, "fwd %.3f" % d["forward_ms"], "bt %.3f" % d["backtrack_ms"], "same", d["same_as_v5"])
    except Exception:
        print(l[:200])
PY
for so in tsp-mpi-reduction_amd/lib_ab/stamp*.so; do
  TSPGPU_LIB=$PWD/$so timeout -k 10 120 python3 tools/k1_stamp.py 16 16384 >> gpurun_out/r05/stamp3.txt 2>&1 || { echo "stamp $so failed"; tail -3 gpurun_out/r05/stamp3.txt; exit 1; }
done
cat gpurun_out/r05/stamp3.txt
timeout -k 10 400 python -u -m pytest tests/test_merge_gpu.py tests/test_cli_gpu.py -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/r05/k3_tests3.log 2>&1; echo k3 tests rc=$?; tail -2 gpurun_out/r05/k3_tests3.log
timeout -k 10 200 python3 -c "import sys; sys.path.insert(0,'tsp-mpi-reduction_amd'); import json, bench; print(json.dumps(bench.k3_merge()))" > gpurun_out/r05/k3_bench3.json 2>&1; echo k3 bench rc=$?; cat gpurun_out/r05/k3_bench3.json
for m in stream null pinned stream; do timeout -k 5 60 ./tsp-mpi-reduction_amd/bin/init_probe3 $m; done > gpurun_out/r05/init_probe3.txt 2>&1; cat gpurun_out/r05/init_probe3.txt
for dep in 0 5 6; do
  if [ $dep = 0 ]; then timeout -k 5 120 python3 tools/k2_solve_time.py 20 > gpurun_out/r05/k2_depth_$dep.txt 2>&1;
  else TSPGPU_SEARCH_DEPTH=$dep timeout -k 5 120 python3 tools/k2_solve_time.py 20 > gpurun_out/r05/k2_depth_$dep.txt 2>&1; fi
  echo "== depth $dep rc=$?"; cat gpurun_out/r05/k2_depth_$dep.txt
done
