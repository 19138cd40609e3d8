"""The drop-in C++ interface (include/assignment2_gpu.h + host/tsp_shim.cpp):
the reference's own single-rank call sequence (distributeCities, tsp() per
block or tspBatch(), the mergeBlocks fold — K3 on the GPU for large merges)
reproduces `mpirun -np 1 ./tsp n B X Y` (tests/golden/cli.json)."""
import os
import re
import subprocess

import pytest

import oracle_py as O
import tspgpu

pytestmark = pytest.mark.gpu
BIN = os.path.join(os.path.dirname(tspgpu.TSP_BIN), "shim_example")
CASES = [c for c in O.load_golden("cli.json") if not c.get("error_case") and c["P"] == 1]


@pytest.mark.parametrize("case", CASES, ids=lambda c: "-".join(map(str, c["args"])))
@pytest.mark.parametrize("batch", [0, 1])
def test_shim_program_matches_reference(case, batch):
    p = subprocess.run([BIN, *map(str, case["args"]), str(batch)], capture_output=True, text=True, timeout=300)
    assert p.returncode == 0, p.stderr
    want = re.search(r"for (\d+) cities and the trip cost (\S+)$", case["lines"][-1])
    got = re.search(r"^(\d+) cities and the trip cost (\S+)$", p.stdout.splitlines()[-1])
    assert got.group(2) == want.group(2)
