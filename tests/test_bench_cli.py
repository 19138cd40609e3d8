"""bench.py's launcher path on CPU: `python bench.py --gpus N` with no
torchrun starts the N ranks itself (a torch.distributed.run child over
127.0.0.1, gloo here), every rank takes its contiguous shard — of one fixed
global instance (strong scaling, the default) or a fixed per-rank count
(weak) — and rank 0 reports n_gpus = N.  --plumbing skips every device call,
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
def test_bench_weak_shards_disjointly(gpus):
    out = _run("--gpus", str(gpus), "--plumbing", "--scaling", "weak", "--steps", "2", "--warmup", "1",
               "--blocks-per-gpu", "8")
    assert out["plumbing"] is True
    assert out["n_gpus"] == gpus and out["scaling"] == "weak"
    assert out["steps"] == 2 and out["warmup"] == 1
    assert out["shards"] == [[8 * r, 8 * (r + 1)] for r in range(gpus)]
    assert out["global_blocks"] == 8 * gpus
    assert out["wall_max_s"] >= 0


@pytest.mark.parametrize("gpus,blocks", [(2, 16), (3, 16), (3, 65536), (2, 3)])
def test_bench_strong_splits_one_fixed_instance(gpus, blocks):
    """The default line: one fixed `./tsp n G` instance, disjoint contiguous
    shards covering [0, G) with the reference's per-rank counts (tsp.cpp:167-171)."""
    out = _run("--gpus", str(gpus), "--plumbing", "--steps", "1", "--warmup", "0", "--global-blocks", str(blocks))
    assert out["scaling"] == "strong" and out["global_blocks"] == blocks and out["n_gpus"] == gpus
    sh = out["shards"]
    assert sh[0][0] == 0 and sh[-1][1] == blocks
    assert all(sh[r][1] == sh[r + 1][0] for r in range(gpus - 1))
    cnt = [0] * gpus
    for b in range(blocks, 0, -1):  # the reference's deal
        cnt[b % gpus] += 1
    assert [hi - lo for lo, hi in sh] == cnt


def test_bench_single_rank_plumbing():
    out = _run("--plumbing", "--steps", "1", "--warmup", "0", "--global-blocks", "4")
    assert out["n_gpus"] == 1 and out["shards"] == [[0, 4]] and out["scaling"] == "strong"
