"""bench.py's multi-rank path on a real GPU: `bench.py --gpus 2` starts two
ranks itself (torch.distributed.run child); on a one-GPU box both ranks share
device 0 and the K2 incumbent exchange runs over gloo (RCCL wants one rank
per device), on an 8-GPU node the same code takes the RCCL group.  Checks
the line the driver reads: n_gpus, the fixed global block count (strong
scaling) and the weak probe beside it, both ranks' K2
shards and the strong-scaling instance's optimum (= K1-wide on one GPU)."""
import json
import os
import subprocess
import sys

import numpy as np
import pytest

import tspgpu

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_bench_two_ranks_end_to_end(gpu_ctx):
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "2", "--warmup", "1",
           "--global-blocks", "1000", "--blocks-per-gpu", "512", "--no-pmc", "--no-cpu-baseline", "--no-tto",
           "--no-ref-multiblock", "--k2-n", "18", "--k2-seed", "1"]
    env = dict(os.environ, BENCH_I32="0")
    p = subprocess.run(cmd, capture_output=True, text=True, timeout=300, env=env, cwd=ROOT)
    assert p.returncode == 0, p.stderr[-2000:]
    line = json.loads([ln for ln in p.stdout.splitlines() if ln.startswith("{")][-1])
    ndev = tspgpu.device_count()
    assert line["ranks"] == 2 and line["n_gpus"] == min(2, ndev) and line["config"]["global_blocks"] == 1000
    assert line["ranks_per_gpu"] == (1 if ndev >= 2 else 2)
    assert line["config"]["blocks_rank0"] == 500  # the reference's deal of 1000 blocks over 2 ranks
    assert line["value"] > 0 and line["scaling"] == "strong"
    other = line["other_scaling"]
    assert other["scaling"] == "weak" and other["global_blocks"] == 1024 and other["value"] > 0
    split = line["k1_kernel_split"]  # forward + backtracking kernels of the timed launches fit in the step
    assert split is None or split["forward_kernel_ms"] + split["backtrack_kernel_ms"] <= line["ms_per_step"] * 1.001
    k2s = line["k2_strong_scaling"]
    assert "error" not in k2s, k2s
    assert k2s["ranks"] == 2 and len(k2s["rank_walls_ms"]) == 2
    sys.path.insert(0, ROOT)
    from bench import k2_instance

    d = k2_instance(18, 1)
    wide_cost, wide_tour, _ = gpu_ctx.solve_instance(np.asarray(d, dtype=np.float64))
    assert k2s["cost"] == wide_cost and k2s["tour"] == [int(x) for x in wide_tour]
    k2 = line["k2_single_instance"]
    assert "error" not in k2 and k2["ranks"] == 2 and k2["cost"] == 3871.1947567096445
    # every rank one device chain, the winner from the all-reduced device tie key
    rule = k2["device_tie_rule"]
    assert rule["used"] == 1 and rule["phases"] == 1 and rule["record_gather"] == 0 and rule["chained"] == 1, rule
