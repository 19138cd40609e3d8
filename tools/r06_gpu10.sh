#!/bin/bash
# Round-6 check 10: K1 one launch pair vs 2/4 concurrent lanes (contexts) per step.
set -u
cd "$(dirname "$0")/.."
OUT=gpurun_out/r06/lanes
mkdir -p $OUT
timeout -k 10 600 python3 -u tools/k1_two_lane.py 6 > $OUT/lanes.json 2> $OUT/lanes.err
echo "lanes rc=$?"; cat $OUT/lanes.json; tail -3 $OUT/lanes.err
