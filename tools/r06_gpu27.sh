#!/bin/bash
# Round-6 check 27: instruction-cache counters of the 16-city K2 chain
# kernels (bench.py's K2 PMC child: 4 searches), two passes.
set -u
cd "$(dirname "$0")/.."
ROOT=$PWD
OUT=$ROOT/gpurun_out/r06/k2if
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
i=0
for p in "SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE" "SQ_IFETCH SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_WAVES SQ_WAIT_ANY SQ_BUSY_CYCLES"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $p --output-format csv -d $OUT/p$i -o pmc -- python3 $ROOT/bench.py --pmc-child-k2 > $OUT/p$i.log 2>&1
  echo "pass $i rc=$?"
done
cd $ROOT
python3 - $OUT <<'PY'
import csv, glob, sys, collections
out = sys.argv[1]
agg = collections.defaultdict(lambda: collections.defaultdict(float)); disp = collections.defaultdict(set)
for f in glob.glob(out + "/p*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        fam = r["Kernel_Name"].replace("(anonymous namespace)::", "").replace("void ", "").split("(")[0].split("<")[0].split("::")[-1]
        agg[fam][r["Counter_Name"]] += float(r["Counter_Value"]); disp[fam].add(r["Dispatch_Id"])
for fam, c in agg.items():
    d = max(1, len(disp[fam]) // 2)
    print(fam, "dispatches", d, {k: round(v / d, 1) for k, v in sorted(c.items())})
PY
