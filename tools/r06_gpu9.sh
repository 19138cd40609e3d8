#!/bin/bash
# Round-6 check 9: bench.py --gpus 2 on ONE GPU (two ranks sharing it; the
# K2 exchange over gloo), the per-rank host/device split of the scaling leg.
set -u
cd "$(dirname "$0")/.."
OUT=gpurun_out/r06/g2
mkdir -p $OUT
timeout -k 10 600 python3 -u bench.py --gpus 2 --steps 5 --warmup 1 > $OUT/bench_g2.json 2> $OUT/bench_g2.err
rc=$?; echo "bench g2 rc=$rc"; tail -c 400 $OUT/bench_g2.json; tail -5 $OUT/bench_g2.err
python3 - <<'PY'
import json
d = json.loads(open("gpurun_out/r06/g2/bench_g2.json").read().strip().splitlines()[-1])
k = d.get("k2_strong_scaling", {})
print(json.dumps({"n_gpus": d.get("n_gpus"), "value": d.get("value"), "scaling": d.get("scaling"),
                  "k2_time_to_optimal_ms": k.get("time_to_optimal_ms"), "exchanges": k.get("exchanges"),
                  "in_chain_exchanges": k.get("in_chain_exchanges"), "cost": k.get("cost"),
                  "rank_split": k.get("rank_split")}, indent=1))
PY
