#!/bin/bash
# Instruction-fetch and latency counters of one K1 configuration.
#   gpurun -- 'bash tools/pmc_ifetch.sh TAG KERNEL_SUBSTR'   (env: TSPGPU_K1, TSPGPU_TILED_CFG)
set -u
cd "$(dirname "$0")/.."
TAG=${1:-ifetch}; KERN=${2:-hk_tiled_kernel}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
PASSES=(
  "SQC_ICACHE_HITS SQC_ICACHE_MISSES"
  "SQC_ICACHE_MISSES_DUPLICATE SQC_TC_INST_REQ"
  "SQ_IFETCH SQ_IFETCH_LEVEL SQ_INSTS_LDS SQ_INST_LEVEL_LDS SQ_INSTS_VMEM_RD SQ_INST_LEVEL_VMEM SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE"
  "SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_BUSY_CYCLES"
)
i=0
for p in "${PASSES[@]}"; do
  i=$((i+1))
  timeout -s KILL 60 rocprofv3 --pmc $p --output-format csv -d $OUT/p$i -o pmc -- python3 tools/kernel_run.py 16 4096 2 > $OUT/p$i.log 2>&1
  rc=$?
  echo "== $TAG pass $i rc=$rc" >&2
  if [ $rc -ne 0 ]; then tail -3 $OUT/p$i.log >&2; [ $rc -ge 124 ] && exit $rc; fi
done
python3 - "$OUT" "$KERN" <<'PY'
import csv, glob, os, sys, collections
out, kern = sys.argv[1], sys.argv[2]
vals = collections.defaultdict(list)
for f in glob.glob(os.path.join(out, "p*", "**", "*counter_collection.csv"), recursive=True):
    for row in csv.DictReader(open(f)):
        if kern in row["Kernel_Name"]:
            vals[row["Counter_Name"]].append(float(row["Counter_Value"]))
c = {k: sum(v) / len(v) for k, v in vals.items()}
with open(os.path.join(out, "summary.txt"), "w") as fh:
    for k in sorted(c):
        fh.write(f"{k} {c[k]:.6g}\n")
    g = lambda k: c.get(k, float("nan"))
    fh.write(f"derived icache_hit_rate {g('SQC_ICACHE_HITS') / (g('SQC_ICACHE_HITS') + g('SQC_ICACHE_MISSES')):.4f}\n")
    fh.write(f"derived ifetch_latency_cycles {g('SQ_IFETCH_LEVEL') / g('SQ_IFETCH'):.1f}\n")
    fh.write(f"derived lds_latency {g('SQ_INST_LEVEL_LDS') / g('SQ_INSTS_LDS'):.1f}\n")
    fh.write(f"derived vmem_rd_latency {g('SQ_INST_LEVEL_VMEM') / g('SQ_INSTS_VMEM_RD'):.1f}\n")
    fh.write(f"derived wait_any_frac {g('SQ_WAIT_ANY') / g('SQ_WAVE_CYCLES'):.3f}\n")
    fh.write(f"derived wait_inst_any_frac {g('SQ_WAIT_INST_ANY') / g('SQ_WAVE_CYCLES'):.3f}\n")
    fh.write(f"derived ifetch_per_valu {g('SQ_IFETCH') / g('SQ_INSTS_VALU'):.3f}\n")
print(open(os.path.join(out, "summary.txt")).read())
PY
