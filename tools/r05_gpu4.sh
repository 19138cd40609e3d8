#!/bin/bash
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/r05
ROUNDS=2 OUT=gpurun_out/r05/ab4 timeout -k 10 300 bash tools/ab_time.sh > gpurun_out/r05/ab4.txt 2>&1; echo ab rc=$?; cut -c1-300 gpurun_out/r05/ab4.txt
for so in tsp-mpi-reduction_amd/lib_ab/stamp*.so; do
  TSPGPU_LIB=$PWD/$so timeout -k 10 120 python3 tools/k1_stamp.py 16 16384 >> gpurun_out/r05/stamp2.txt 2>&1 || { echo "stamp $so failed"; tail -3 gpurun_out/r05/stamp2.txt; exit 1; }
done
cat gpurun_out/r05/stamp2.txt
bash tools/r05_k3trace.sh
for dl in default 0 1; do
  if [ $dl = default ]; then ./tsp-mpi-reduction_amd/bin/init_probe2 > gpurun_out/r05/init_probe_$dl.txt 2>&1;
  else HIP_ENABLE_DEFERRED_LOADING=$dl ./tsp-mpi-reduction_amd/bin/init_probe2 > gpurun_out/r05/init_probe_$dl.txt 2>&1; fi
  echo "== deferred=$dl rc=$?"; cat gpurun_out/r05/init_probe_$dl.txt
done
