#!/bin/bash
# Kernel-trace each timing variant of tools/abl_build.sh (GPU box):
#   bash tools/abl_prof.sh NAME ...  -> gpurun_out/abl_prof/<name>/*kernel_stats.csv
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
mkdir -p $R/gpurun_out/abl_prof; cd /tmp && export TMPDIR=/tmp
for m in "$@"; do
  lib=$R/tsp-mpi-reduction_amd/lib/libtspgpu_abl$m.so
  [ "$m" = "cur" ] && lib=$R/tsp-mpi-reduction_amd/lib/libtspgpu.so
  TSPGPU_LIB=$lib timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/abl_prof/$m -o run -- \
      python3 $R/tools/abl_time.py --one $m > $R/gpurun_out/abl_prof/$m.log 2>&1 || { echo "$m failed"; exit 1; }
  grep "abl=" $R/gpurun_out/abl_prof/$m.log
  cut -d, -f1-4 $R/gpurun_out/abl_prof/$m/run_kernel_stats.csv | grep -v rocclr | sed 's/(.*)//' 
done
