"""Per-kernel split of bench.py's K2 counter pass (development aid, round 5).

bench.py's `k2_single_instance.pmc` sums SQ counters over every kernel of the
16-city search; this reads the same rocprofv3 collection
(`pmc_k2_sq/pmc_counter_collection.csv`, one row per dispatch and counter)
and splits it per kernel family: dispatches, waves, VALU wave-instructions,
VALU lane-instructions per B&B node of the whole search, busy cycles.

    python tools/k2_pmc_split.py CSV NODES_PER_SEARCH SEARCHES
"""
import collections
import csv
import json
import sys


def main():
    path, nodes, searches = sys.argv[1], float(sys.argv[2]), int(sys.argv[3])
    agg = collections.defaultdict(lambda: collections.defaultdict(float))
    disp = collections.defaultdict(set)
    for r in csv.DictReader(open(path)):
        name = r["Kernel_Name"]
        fam = name.replace("(anonymous namespace)::", "").replace("void ", "").split("(")[0].split("<")[0].split("::")[-1]
        agg[fam][r["Counter_Name"]] += float(r["Counter_Value"])
        disp[fam].add(r["Dispatch_Id"])
    out = {}
    tot = 0.0
    for fam, c in agg.items():
        valu = c["SQ_INSTS_VALU"] / searches
        tot += valu
        out[fam] = {
            "dispatches_per_search": len(disp[fam]) / searches,
            "waves_per_search": c["SQ_WAVES"] / searches,
            "valu_wave_instructions_per_search": valu,
            "valu_lane_instructions_per_node": valu * 64 / nodes,
            "busy_cycles_per_search": c["SQ_BUSY_CYCLES"] / searches,
            "wave_cycles_per_search": c["SQ_WAVE_CYCLES"] / searches,
        }
    out["total_valu_lane_instructions_per_node"] = tot * 64 / nodes
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
