#!/bin/bash
# PMC passes over the K1 forward kernel (one counter group per rocprofv3 run,
# MI355X_MICROARCH.md: <= 8 SQ, 4 TCC, 2 GRBM per pass), medians per counter
# over the hk_sub_kernel dispatches of tools/k1_once.py:
#   bash tools/k1_pmc_r05.sh TAG [n] [blocks] [vb] [lib]
set -u
cd "$(dirname "$0")/.."
TAG=$1; N=${2:-16}; B=${3:-4096}; VB=${4:-8}; LIB=${5:-}
OUT=gpurun_out/r05/pmc_$TAG
rm -rf $OUT; mkdir -p $OUT
export TMPDIR=/tmp
[ -n "$LIB" ] && export TSPGPU_LIB=$PWD/$LIB
PASSES=(
  "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU"
  "SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE GRBM_COUNT"
  "SQ_WAIT_INST_LDS SQ_INSTS_SMEM SQ_INST_CYCLES_VMEM SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_SCA SQ_LDS_IDX_ACTIVE SQ_INSTS_BRANCH SQ_ACTIVE_INST_FLAT"
  "TCC_HIT_sum TCC_MISS_sum"
  "TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_DRAM_sum TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_DRAM_sum"
  "FETCH_SIZE"
  "WRITE_SIZE"
)
i=0
for p in "${PASSES[@]}"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $p --output-format csv -d $OUT/p$i -o pmc -- python3 tools/k1_once.py $N $B $VB 6 > $OUT/p$i.log 2>&1
  rc=$?
  if [ $rc -ne 0 ]; then echo "pass $i rc=$rc"; tail -5 $OUT/p$i.log; exit $rc; fi
done
python3 - "$OUT" "$B" <<'PY' | tee $OUT/summary.txt
import csv, glob, sys, collections, statistics
out, B = sys.argv[1], int(sys.argv[2])
vals = collections.defaultdict(list)
for f in glob.glob(out + "/p*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "hk_sub_kernel" in r["Kernel_Name"]:
            vals[r["Counter_Name"]].append(float(r["Counter_Value"]))
m = {k: statistics.median(v) for k, v in vals.items()}
for k in sorted(m):
    print(f"{k} {m[k]:.6g}  per_block {m[k] / B:.6g}")
w = m.get("SQ_WAVE_CYCLES")
if w:
    for k in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_BUSY_CYCLES"):
        if k in m:
            print(f"frac {k}/SQ_WAVE_CYCLES {m[k] / w:.4f}")
if "TCC_HIT_sum" in m:
    print(f"TCC hit rate {m['TCC_HIT_sum'] / (m['TCC_HIT_sum'] + m['TCC_MISS_sum']):.4f}")
PY
