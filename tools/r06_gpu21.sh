#!/bin/bash
# Round-6 check 21: the multi-rank bench path after the K2 changes — the
# driver's own launcher form (torch.distributed.run, 2 ranks sharing the one
# GPU: device = LOCAL_RANK mod device count), then bench.py --gpus 2.
set -u
cd "$(dirname "$0")/.."
OUT=gpurun_out/r06/g2b
mkdir -p $OUT
timeout -k 10 600 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 3 --warmup 1 > $OUT/bench_torchrun_g2.json 2> $OUT/bench_torchrun_g2.err
rc=$?; echo "torchrun rc=$rc"; tail -c 600 $OUT/bench_torchrun_g2.json; [ $rc -eq 0 ] || { tail -20 $OUT/bench_torchrun_g2.err; exit $rc; }
timeout -k 10 600 python3 -u bench.py --gpus 2 --steps 5 --warmup 1 > $OUT/bench_g2.json 2> $OUT/bench_g2.err
rc=$?; echo "bench g2 rc=$rc"; tail -c 300 $OUT/bench_g2.json; exit $rc
