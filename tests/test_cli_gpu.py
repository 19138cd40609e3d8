"""End-to-end drop-in check: bin/tsp (GPU block search + host reduction
replay) against the reference CLI's stdout captured under mpirun
(tests/golden/cli.json).  The measured milliseconds are the only field that
may differ; the "process ..." lines of different MPI ranks interleave
nondeterministically under mpirun, so they are compared as a multiset."""
import os
import re
import subprocess

import pytest

import oracle_py as O
import tspgpu

MS = re.compile(r"^TSP ran in \d+ ms ")
CASES = O.load_golden("cli.json")
# SURVEY Appendix B's merge-dominated runs, where K3 (the GPU mergeBlocks)
# carries the program: ./tsp 4 1024 at P=1/8, ./tsp 8 1024 at P=8 (the
# reference: 7.1 / 30.9 / 237 s on 8 cores)
LARGE = O.load_golden("cli_large.json")


def run_tsp(args, P):
    env = dict(os.environ, TSP_NPROCS=str(P))
    for k in ("PMI_SIZE", "PMI_RANK", "OMPI_COMM_WORLD_SIZE", "OMPI_COMM_WORLD_RANK"):
        env.pop(k, None)
    p = subprocess.run([tspgpu.TSP_BIN, *map(str, args)], capture_output=True, text=True, env=env, timeout=300)
    lines = [MS.sub("TSP ran in <ms> ms ", ln) for ln in p.stdout.splitlines()]
    return p.returncode, lines, p.stderr


def split(lines):
    proc = sorted(ln for ln in lines if ln.startswith("process "))
    rest = [ln for ln in lines if not ln.startswith("process ")]
    return rest, proc


@pytest.mark.parametrize("case", [c for c in CASES if c.get("error_case")], ids=lambda c: "err-" + "-".join(c["args"]))
def test_cli_argument_errors(case):
    # no GPU involved: argument checks come first, as in the reference
    rc, lines, _ = run_tsp(case["args"], 1)
    assert rc == case["rc"] and lines == case["lines"]


@pytest.mark.gpu
@pytest.mark.parametrize("case", [c for c in CASES if not c.get("error_case")],
                         ids=lambda c: "-".join(map(str, c["args"])) + f"-P{c['P']}")
def test_cli_matches_reference(case):
    rc, lines, err = run_tsp(case["args"], case["P"])
    assert rc == case["rc"], err
    assert split(lines) == split(case["lines"])


@pytest.mark.gpu
@pytest.mark.parametrize("case", LARGE, ids=lambda c: "-".join(map(str, c["args"])) + f"-P{c['P']}")
def test_cli_merge_dominated_matches_reference(case):
    rc, lines, err = run_tsp(case["args"], case["P"])
    assert rc == case["rc"], err
    assert split(lines) == split(case["lines"])


@pytest.mark.gpu
def test_cli_stats_line_is_opt_in_and_on_stderr():
    """TSP_STATS=1 adds one statistics line on stderr; stdout stays the
    reference's (SURVEY.md §5 "Metrics")."""
    case = next(c for c in CASES if not c.get("error_case") and list(c["args"][:2]) == [16, 8] and c["P"] == 1)
    env = dict(os.environ, TSP_NPROCS=str(case["P"]), TSP_STATS="1")
    for k in ("PMI_SIZE", "PMI_RANK", "OMPI_COMM_WORLD_SIZE", "OMPI_COMM_WORLD_RANK"):
        env.pop(k, None)
    p = subprocess.run([tspgpu.TSP_BIN, *map(str, case["args"])], capture_output=True, text=True, env=env, timeout=300)
    assert p.returncode == case["rc"], p.stderr
    lines = [MS.sub("TSP ran in <ms> ms ", ln) for ln in p.stdout.splitlines()]
    assert split(lines) == split(case["lines"])
    stats = [ln for ln in p.stderr.splitlines() if ln.startswith("tsp stats: ")]
    assert len(stats) == 1 and "DP relaxations/s" in stats[0] and "block search" in stats[0]
    _, _, plain_err = run_tsp(case["args"], case["P"])
    assert "tsp stats" not in plain_err
