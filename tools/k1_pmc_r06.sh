#!/bin/bash
# PMC passes over one K1 kernel (one counter group per rocprofv3 run), medians
# per counter over the dispatches of tools/k1_once.py whose name contains KERN:
#   bash tools/k1_pmc_r06.sh TAG KERN spec [n] [blocks] [vb] [lib]
set -u
cd "$(dirname "$0")/.."
TAG=$1; KERN=$2; SPEC=$3; N=${4:-16}; B=${5:-4096}; VB=${6:-8}; LIB=${7:-}
OUT=gpurun_out/r06/pmc_$TAG
rm -rf $OUT; mkdir -p $OUT
export TMPDIR=/tmp
[ -n "$LIB" ] && export TSPGPU_LIB=$PWD/$LIB
PASSES=(
  "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU"
  "SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE GRBM_COUNT"
  "TCC_HIT_sum TCC_MISS_sum"
  "FETCH_SIZE"
  "WRITE_SIZE"
)
i=0
for p in "${PASSES[@]}"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $p --output-format csv -d $OUT/p$i -o pmc -- python3 tools/k1_once.py $N $B $VB $SPEC > $OUT/p$i.log 2>&1
  rc=$?
  if [ $rc -ne 0 ]; then echo "pass $i rc=$rc"; tail -5 $OUT/p$i.log; exit $rc; fi
done
python3 - "$OUT" "$B" "$KERN" <<'PY' | tee $OUT/summary.txt
import csv, glob, sys, collections, statistics
out, B, kern = sys.argv[1], int(sys.argv[2]), sys.argv[3]
vals = collections.defaultdict(list)
for f in glob.glob(out + "/p*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if kern in r["Kernel_Name"]:
            vals[r["Counter_Name"]].append(float(r["Counter_Value"]))
m = {k: statistics.median(v) for k, v in vals.items()}
for k in sorted(m):
    print(f"{k} {m[k]:.6g}  per_block {m[k] / B:.6g}")
w = m.get("SQ_WAVE_CYCLES")
if w:
    for k in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY"):
        if k in m: print(f"{k}/SQ_WAVE_CYCLES {m[k] / w:.3f}")
h, mi = m.get("TCC_HIT_sum"), m.get("TCC_MISS_sum")
if h is not None and mi: print(f"TCC hit rate {h / (h + mi):.3f}")
if "FETCH_SIZE" in m: print(f"FETCH_SIZE KB per block {m['FETCH_SIZE'] / B:.1f}")
if "WRITE_SIZE" in m: print(f"WRITE_SIZE KB per block {m['WRITE_SIZE'] / B:.1f}")
PY
