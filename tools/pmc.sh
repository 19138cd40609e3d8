#!/bin/bash
# PMC passes over the K1 kernel, one counter group per rocprofv3 run
# (MI355X_MICROARCH.md: <= 8 SQ, 4 TCC (FETCH_SIZE=3, WRITE_SIZE=2), 2 GRBM per pass).
#   gpurun -- 'bash tools/pmc.sh TAG [n] [blocks]'
set -u
cd "$(dirname "$0")/.."
TAG=${1:-pmc}; N=${2:-16}; B=${3:-4096}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
PASSES=(
  "FETCH_SIZE"
  "WRITE_SIZE"
  "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU"
  "SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE GRBM_COUNT"
  "TCC_HIT_sum TCC_MISS_sum"
  "TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum"
)
i=0
for p in "${PASSES[@]}"; do
  i=$((i+1))
  echo "== pass $i: $p" >&2
  timeout -s KILL 90 rocprofv3 --pmc $p --output-format csv -d $OUT/p$i -o pmc -- python3 tools/kernel_run.py $N $B 2 > $OUT/p$i.log 2>&1
  rc=$?
  echo "   rc=$rc" >&2
  if [ $rc -ne 0 ]; then tail -5 $OUT/p$i.log >&2; fi
  if [ $rc -ge 124 ]; then echo "stopping" >&2; exit $rc; fi
done
python3 - "$OUT" <<'PY'
import csv, glob, os, sys, collections
out = sys.argv[1]
vals = collections.defaultdict(list)
for f in glob.glob(os.path.join(out, "p*", "**", "*counter_collection.csv"), recursive=True):
    for row in csv.DictReader(open(f)):
        if "heldkarp_kernel" in row["Kernel_Name"]:
            vals[row["Counter_Name"]].append(float(row["Counter_Value"]))
with open(os.path.join(out, "summary.txt"), "w") as fh:
    for k in sorted(vals):
        line = f"{k} {sum(vals[k]) / len(vals[k]):.6g} (n={len(vals[k])})"
        print(line); fh.write(line + "\n")
PY
