#!/bin/bash
# PMC passes over the K2 round kernel (one counter group per rocprofv3 run).
#   gpurun -- 'bash tools/k2_pmc.sh TAG [n]'
set -u
cd "$(dirname "$0")/.."
TAG=${1:-k2pmc}; N=${2:-16}; MODE=${3:-bnb}   # bnb: tools/k2_time.py, exh: tools/k2_exhaustive.py
PROG=tools/k2_time.py
[ "$MODE" = exh ] && PROG=tools/k2_exhaustive.py
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
PASSES=(
  "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU"
  "SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE GRBM_COUNT"
  "SQ_WAIT_INST_LDS SQ_INSTS_BRANCH SQ_ACTIVE_INST_SCA SQ_INSTS_SMEM SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_FLAT SQ_INST_CYCLES_SALU SQ_INSTS_FLAT"
)
i=0
for p in "${PASSES[@]}"; do
  i=$((i+1))
  echo "== pass $i: $p" >&2
  timeout -s KILL 90 rocprofv3 --pmc $p --output-format csv -d $OUT/p$i -o pmc -- python3 $PROG $N > $OUT/p$i.log 2>&1
  rc=$?
  echo "   rc=$rc" >&2
  if [ $rc -ne 0 ]; then tail -5 $OUT/p$i.log >&2; fi
  if [ $rc -ge 124 ]; then echo "stopping" >&2; exit $rc; fi
done
python3 - "$OUT" <<'PY'
import csv, glob, os, sys, collections
out = sys.argv[1]
vals = collections.defaultdict(float)
for f in glob.glob(os.path.join(out, "p*", "**", "*counter_collection.csv"), recursive=True):
    for row in csv.DictReader(open(f)):
        if "round_kernel" in row["Kernel_Name"]:
            vals[row["Counter_Name"]] += float(row["Counter_Value"])
with open(os.path.join(out, "summary.txt"), "w") as fh:
    for k in sorted(vals):
        line = f"{k} {vals[k]:.6g}"
        print(line); fh.write(line + "\n")
PY
