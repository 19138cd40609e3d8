#!/bin/bash
# K3 timing and a kernel + HIP API trace of the merge-dominated ./tsp 8 1024 at P = 8
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/r05
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_merge_gpu.py tests/test_cli_gpu.py -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/r05/k3_tests2.log 2>&1; echo k3 tests rc=$?; tail -2 gpurun_out/r05/k3_tests2.log
timeout -k 10 200 python3 -c "import sys; sys.path.insert(0,'tsp-mpi-reduction_amd'); import json, bench; print(json.dumps(bench.k3_merge()))" > gpurun_out/r05/k3_bench2.json 2>&1; echo k3 bench rc=$?; cat gpurun_out/r05/k3_bench2.json
TSP_NPROCS=8 TSP_STATS=1 timeout -k 10 120 rocprofv3 --kernel-trace --hip-trace --stats -d gpurun_out/r05/k3trace -o k3 -- ./tsp-mpi-reduction_amd/bin/tsp 8 1024 1000 1000 > gpurun_out/r05/k3trace.log 2>&1; echo trace rc=$?
