mkdir -p gpurun_out/r05
for so in tsp-mpi-reduction_amd/lib_ab/stamp*.so; do
  TSPGPU_LIB=$PWD/$so timeout -k 10 120 python3 tools/k1_stamp.py 16 16384 >> gpurun_out/r05/stamp1.txt 2>&1 || { echo "stamp $so failed"; tail -3 gpurun_out/r05/stamp1.txt; exit 1; }
done
cat gpurun_out/r05/stamp1.txt
timeout -k 10 400 python -u -m pytest tests/test_merge_gpu.py tests/test_cli_gpu.py -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/r05/k3_tests.log 2>&1; echo k3 tests rc=$?; tail -3 gpurun_out/r05/k3_tests.log
timeout -k 10 200 python3 -c "import sys; sys.path.insert(0,'tsp-mpi-reduction_amd'); import json, bench; print(json.dumps(bench.k3_merge()))" > gpurun_out/r05/k3_bench.json 2>&1; echo k3 bench rc=$?; cat gpurun_out/r05/k3_bench.json
