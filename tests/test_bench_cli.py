"""bench.py's launcher path on CPU: `python bench.py --gpus N` with no
torchrun starts the N ranks itself (a torch.distributed.run child over
127.0.0.1, gloo here), every rank takes its contiguous shard of the global
instance and rank 0 reports n_gpus = N.  --plumbing skips every device call,
so this runs without a GPU; the device path is the same code under -m gpu."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(*args, timeout=240):
    env = dict(os.environ)
    env.pop("WORLD_SIZE", None)
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), *args], capture_output=True, text=True,
                       timeout=timeout, env=env, cwd=ROOT)
    assert p.returncode == 0, p.stderr[-2000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, p.stdout
    return json.loads(lines[0])


@pytest.mark.parametrize("gpus", [2, 3])
def test_bench_spawns_ranks_and_shards_disjointly(gpus):
    out = _run("--gpus", str(gpus), "--plumbing", "--steps", "2", "--warmup", "1", "--blocks-per-gpu", "8")
    assert out["plumbing"] is True
    assert out["n_gpus"] == gpus
    assert out["steps"] == 2 and out["warmup"] == 1
    assert out["shards"] == [[8 * r, 8 * (r + 1)] for r in range(gpus)]
    assert out["global_blocks"] == 8 * gpus
    assert out["wall_max_s"] >= 0


def test_bench_single_rank_plumbing():
    out = _run("--plumbing", "--steps", "1", "--warmup", "0", "--blocks-per-gpu", "4")
    assert out["n_gpus"] == 1 and out["shards"] == [[0, 4]]
