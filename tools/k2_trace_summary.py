"""Per-kernel summary of a rocprofv3 kernel trace of tools/k2_trace16.py: for
each kernel name, launches and mean duration, and the chain's mean span
(first kernel start to last kernel end of one search) — development aid for
the 16-city latency chain.   python tools/k2_trace_summary.py TRACE.csv"""
import csv
import sys
from collections import defaultdict

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
dur = defaultdict(list)
for r in rows:
    name = r["Kernel_Name"].replace("(anonymous namespace)::", "").split("(")[0].replace("void ", "")
    dur[name].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
for name, v in sorted(dur.items(), key=lambda kv: -sum(kv[1])):
    v2 = sorted(v)
    print(f"{len(v):6d} x {sum(v) / len(v):8.2f} us (median {v2[len(v2) // 2]:8.2f})  {name[:110]}")
