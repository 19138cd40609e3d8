#!/bin/bash
# PMC passes over one K1 configuration (one counter group per rocprofv3 run;
# MI355X_MICROARCH.md: <= 8 SQ, 4 TCC, 2 GRBM per pass), summarised per kernel.
#   gpurun -- 'bash tools/pmc_k1.sh TAG KERNEL_SUBSTR [n] [blocks]'   (env: TSPGPU_K1, TSPGPU_TILED_CFG)
set -u
cd "$(dirname "$0")/.."
TAG=${1:-pmc}; KERN=${2:-heldkarp_kernel}; N=${3:-16}; B=${4:-4096}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
PASSES=(
  "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU"
  "SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE GRBM_COUNT"
  "SQ_WAIT_INST_LDS SQ_INSTS_SMEM SQ_INST_CYCLES_VMEM SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_SCA SQ_LDS_IDX_ACTIVE SQ_INSTS_BRANCH SQ_ACTIVE_INST_FLAT"
  "FETCH_SIZE"
  "WRITE_SIZE"
  "TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_DRAM_sum TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_DRAM_sum"
  "TCC_HIT_sum TCC_MISS_sum"
)
i=0
for p in "${PASSES[@]}"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $p --output-format csv -d $OUT/p$i -o pmc -- python3 tools/kernel_run.py $N $B 2 > $OUT/p$i.log 2>&1
  rc=$?
  echo "== $TAG pass $i rc=$rc" >&2
  if [ $rc -ne 0 ]; then tail -5 $OUT/p$i.log >&2; exit $rc; fi
done
python3 - "$OUT" "$KERN" "$B" <<'PY'
import csv, glob, os, sys, collections
out, kern, B = sys.argv[1], sys.argv[2], int(sys.argv[3])
vals = collections.defaultdict(list)
for f in glob.glob(os.path.join(out, "p*", "**", "*counter_collection.csv"), recursive=True):
    for row in csv.DictReader(open(f)):
        if kern in row["Kernel_Name"]:
            vals[row["Counter_Name"]].append(float(row["Counter_Value"]))
c = {k: sum(v) / len(v) for k, v in vals.items()}
with open(os.path.join(out, "summary.txt"), "w") as fh:
    for k in sorted(c):
        fh.write(f"{k} {c[k]:.6g} (n={len(vals[k])})\n")
    cyc = c.get("GRBM_GUI_ACTIVE", 0) / 8.0
    if cyc:
        d = {
            "blocks": B,
            "valu_insts_per_block": c["SQ_INSTS_VALU"] / B,
            "lds_insts_per_block": c.get("SQ_INSTS_LDS", 0) / B,
            "salu_insts_per_block": c.get("SQ_INSTS_SALU", 0) / B,
            "valu_active_per_simd_cycle": 4 * c["SQ_ACTIVE_INST_VALU"] / (1024 * cyc),
            "resident_waves_per_cu": 4 * c["SQ_WAVE_CYCLES"] / (256 * cyc),
            "wait_any_frac": c["SQ_WAIT_ANY"] / c["SQ_WAVE_CYCLES"],
            "wait_inst_any_frac": c["SQ_WAIT_INST_ANY"] / c["SQ_WAVE_CYCLES"],
            "active_inst_any_frac": c["SQ_ACTIVE_INST_ANY"] / c["SQ_WAVE_CYCLES"],
            "lds_bank_conflict_over_lds_active": c.get("SQ_LDS_BANK_CONFLICT", 0) / max(c.get("SQ_ACTIVE_INST_LDS", 1), 1),
            "kernel_cycles": cyc,
            "fetch_x2_bytes_per_block": 2 * 1024 * c.get("FETCH_SIZE", 0) / B,
            "write_bytes_per_block": 1024 * c.get("WRITE_SIZE", 0) / B,
            "ea_rd_bytes_per_block": 128 * c.get("TCC_EA0_RDREQ_sum", 0) / B,
            "dram_rd_frac": c.get("TCC_EA0_RDREQ_DRAM_sum", 0) / max(c.get("TCC_EA0_RDREQ_sum", 1), 1),
            "dram_wr_frac": c.get("TCC_EA0_WRREQ_DRAM_sum", 0) / max(c.get("TCC_EA0_WRREQ_sum", 1), 1),
            "l2_hit": c.get("TCC_HIT_sum", 0) / max(c.get("TCC_HIT_sum", 0) + c.get("TCC_MISS_sum", 0), 1),
        }
        for k, v in d.items():
            fh.write(f"derived {k} {v:.6g}\n")
print(open(os.path.join(out, "summary.txt")).read())
PY
