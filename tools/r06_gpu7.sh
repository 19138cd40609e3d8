#!/bin/bash
# Round-6 check 7 (verdict r05 item 1): L = 11 against L = 10 in the
# sub-cube kernel that has both (variant 5: cfg 14 = L 10, 256 threads, six
# workgroups per CU; cfg 2 = L 11, 256 threads, three per CU), timed with the
# product's variant 6 beside them, plus counters of both variant-5 forms.
set -u
cd "$(dirname "$0")/.."
OUT=gpurun_out/r06/l11
mkdir -p $OUT
for r in 1 2; do
  TSPGPU_LIB=$PWD/tsp-mpi-reduction_amd/lib_ab/sweep.so timeout -k 10 300 python3 -u tools/k1_time.py 16 16384 8 5:14 5:2 6 > $OUT/time_r$r.log 2>&1
  echo "time r$r rc=$?"; cat $OUT/time_r$r.log | tail -3
done
timeout -k 10 400 bash tools/k1_pmc_r06.sh l10_v5 hk_tiled_kernel 5:14 16 4096 8 tsp-mpi-reduction_amd/lib_ab/sweep.so > /dev/null 2>&1; echo "pmc l10 rc=$?"; cat gpurun_out/r06/pmc_l10_v5/summary.txt | tail -8
timeout -k 10 400 bash tools/k1_pmc_r06.sh l11_v5 hk_tiled_kernel 5:2 16 4096 8 tsp-mpi-reduction_amd/lib_ab/sweep.so > /dev/null 2>&1; echo "pmc l11 rc=$?"; cat gpurun_out/r06/pmc_l11_v5/summary.txt | tail -8
timeout -k 10 400 bash tools/k1_pmc_r06.sh v6 hk_sub_kernel 6 16 4096 8 > /dev/null 2>&1; echo "pmc v6 rc=$?"; cat gpurun_out/r06/pmc_v6/summary.txt | tail -8
