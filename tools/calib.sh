#!/bin/bash
# Roofline calibration on one MI355X (gpurun):
#   1. VALU issue rates of the relaxation's instructions (ubench valu)
#   2. FETCH_SIZE / WRITE_SIZE / TCC hit-miss / EA request counters over a
#      known byte count with 8-byte-per-lane loads and stores, from a 2 GiB
#      buffer (HBM) and a 64 MiB one (Infinity-Cache resident after rep 0)
#   3. the available counter list (to find Infinity-Cache / DRAM counters)
# Each GPU step has its own time limit; the script stops at the first failure.
set -u
cd "$(dirname "$0")/.."
OUT=gpurun_out/${1:-calib}
mkdir -p $OUT
export TMPDIR=/tmp
UB=tsp-mpi-reduction_amd/bin/ubench
step() {  # name secs cmd...
  local name=$1 secs=$2; shift 2
  timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc" >&2
  if [ $rc -ne 0 ]; then tail -5 "$OUT/$name.log" >&2; exit $rc; fi
}
step valu 120 $UB valu
step mem_plain 60 $UB mem 2048 3
step list 60 rocprofv3 -L
i=0
for sz in 2048 64; do
  for p in "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum" "TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum"; do
    i=$((i+1))
    step pmc_${sz}_$i 60 rocprofv3 --pmc $p --output-format csv -d $OUT/pmc_${sz}_$i -o pmc -- $UB mem $sz 4
  done
done
python3 - "$OUT" <<'PY'
import csv, glob, os, sys, collections
out = sys.argv[1]
rows = collections.defaultdict(list)
for f in sorted(glob.glob(os.path.join(out, "pmc_*", "**", "*counter_collection.csv"), recursive=True)):
    sz = f.split("pmc_")[1].split("_")[0]
    for row in csv.DictReader(open(f)):
        if "stream_kernel" in row["Kernel_Name"]:
            rows[(sz, row["Counter_Name"])].append(float(row["Counter_Value"]))
with open(os.path.join(out, "summary.txt"), "w") as fh:
    for (sz, c), v in sorted(rows.items()):
        line = f"{sz}MiB {c} per-rep {v}"
        print(line); fh.write(line + "\n")
PY
