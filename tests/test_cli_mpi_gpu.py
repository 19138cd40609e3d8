"""The drop-in CLI in its multi-process forms, against the reference's own
stdout captured under mpirun (tests/golden/cli.json):

  * bin/tsp as P processes with the PMI rank variables an mpirun sets
    (PMI_SIZE/PMI_RANK): every rank solves its cnt[r] blocks (tsp.cpp:167-192)
    on GPU r mod (visible devices) and rank 0 gathers them for the reduction;
  * bin/tsp with TSP_GPUS=2 (device g mod visible devices: testable on one GPU);
  * the same under a real `mpirun -np P` when the box has MPICH (/opt/conda);
  * the reference's own, unmodified tsp.cpp linked against the GPU shim
    (oracle/_ref/tsp_dropin, built by oracle/Makefile where /root/reference
    exists) under mpirun: the drop-in boundary with the reference's program.

Only the measured milliseconds may differ; the "process ..." lines of
different ranks interleave, so they are compared as a multiset."""
import os
import re
import shutil
import subprocess
import tempfile

import pytest

import oracle_py as O
import tspgpu

pytestmark = pytest.mark.gpu

MS = re.compile(r"^TSP ran in \d+ ms ")
CASES = [c for c in O.load_golden("cli.json") if not c.get("error_case")]
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
DROPIN = os.path.join(ROOT, "oracle", "_ref", "tsp_dropin")
MPIRUN = shutil.which("mpirun") or ("/opt/conda/bin/mpirun" if os.path.exists("/opt/conda/bin/mpirun") else None)


def _clean_env():
    env = dict(os.environ)
    for k in ("PMI_SIZE", "PMI_RANK", "OMPI_COMM_WORLD_SIZE", "OMPI_COMM_WORLD_RANK", "TSP_NPROCS", "TSP_GPUS",
              "TSP_GATHER_DIR"):
        env.pop(k, None)
    return env


def _norm(text):
    lines = [MS.sub("TSP ran in <ms> ms ", ln) for ln in text.splitlines()]
    return sorted(ln for ln in lines if ln.startswith("process ")), [ln for ln in lines if not ln.startswith("process ")]


def _expect(case):
    return _norm("\n".join(case["lines"]))


def _pick(ps):
    return [c for c in CASES if c["P"] in ps and c["args"][0] <= 12]


@pytest.mark.parametrize("case", _pick({2, 3, 4}), ids=lambda c: "-".join(map(str, c["args"])) + f"-P{c['P']}")
def test_rank_processes_gather_to_rank0(case):
    P = case["P"]
    with tempfile.TemporaryDirectory() as gd:
        procs = []
        for r in range(P):
            env = dict(_clean_env(), PMI_SIZE=str(P), PMI_RANK=str(r), TSP_GATHER_DIR=gd)
            procs.append(subprocess.Popen([tspgpu.TSP_BIN, *map(str, case["args"])], stdout=subprocess.PIPE,
                                          stderr=subprocess.PIPE, text=True, env=env))
        outs = [p.communicate(timeout=300) for p in procs]
        assert all(p.returncode == case["rc"] or (r > 0 and p.returncode == 0) for r, p in enumerate(procs)), \
            [o[1] for o in outs]
        assert all(o[0] == "" for o in outs[1:]), "worker ranks print nothing"
        assert _norm(outs[0][0]) == _expect(case)
        assert os.listdir(gd) == [], "rank 0 consumed every rank file"


@pytest.mark.parametrize("case", _pick({1, 3, 8})[:6], ids=lambda c: "-".join(map(str, c["args"])) + f"-P{c['P']}")
def test_two_gpus_split_in_one_process(case):
    env = dict(_clean_env(), TSP_NPROCS=str(case["P"]), TSP_GPUS="2")
    p = subprocess.run([tspgpu.TSP_BIN, *map(str, case["args"])], capture_output=True, text=True, env=env, timeout=300)
    assert p.returncode == case["rc"], p.stderr
    assert _norm(p.stdout) == _expect(case)


MPI_CASES = [c for c in CASES if (c["args"], c["P"]) in (([6, 8, 1000, 1000], 3), ([12, 4, 1000, 1000], 4),
                                                         ([8, 12, 1000, 1000], 5), ([10, 16, 1000, 1000], 8),
                                                         # SURVEY Appendix B's 16-city multi-block runs
                                                         ([16, 8, 1000, 1000], 1), ([16, 8, 1000, 1000], 2),
                                                         ([16, 8, 1000, 1000], 4), ([16, 8, 1000, 1000], 8),
                                                         ([16, 16, 1000, 1000], 8), ([14, 64, 1000, 1000], 8))]


@pytest.mark.skipif(MPIRUN is None, reason="no mpirun on this machine")
@pytest.mark.parametrize("case", MPI_CASES, ids=lambda c: "-".join(map(str, c["args"])) + f"-P{c['P']}")
def test_bin_tsp_under_mpirun(case):
    p = subprocess.run([MPIRUN, "-np", str(case["P"]), tspgpu.TSP_BIN, *map(str, case["args"])], capture_output=True,
                       text=True, env=_clean_env(), timeout=300, cwd="/tmp")
    assert p.returncode == case["rc"], p.stderr[-2000:]
    assert _norm(p.stdout) == _expect(case)


@pytest.mark.skipif(MPIRUN is None or not os.path.exists(DROPIN),
                    reason="needs mpirun and oracle/_ref/tsp_dropin (built where /root/reference exists)")
@pytest.mark.parametrize("case", MPI_CASES, ids=lambda c: "-".join(map(str, c["args"])) + f"-P{c['P']}")
def test_reference_tsp_cpp_linked_against_gpu_shim(case):
    """The reference's own program (tsp.cpp unmodified, its tsp() and
    mergeBlocks() resolved to the GPU shim) prints the reference's answer."""
    p = subprocess.run([MPIRUN, "-np", str(case["P"]), DROPIN, *map(str, case["args"])], capture_output=True,
                       text=True, env=_clean_env(), timeout=300, cwd="/tmp")
    assert p.returncode == case["rc"], p.stderr[-2000:]
    assert _norm(p.stdout) == _expect(case)


def _two_rank_case():
    return next(c for c in CASES if c["args"] == [6, 8, 1000, 1000] and c["P"] == 2)


def test_stale_rank_file_of_an_earlier_run_is_ignored():
    """a rank file left in the gather directory by an earlier run
    (another job key) must not be taken for this run's: rank 0 drops it and
    waits for this job's own file."""
    import struct

    case = _two_rank_case()
    with tempfile.TemporaryDirectory() as gd:
        # header of the current format (magic "TSP2"), same rank/n/B/X/Y, foreign job key, no payload
        n, B, X, Y = case["args"]
        with open(os.path.join(gd, "rank1.bin"), "wb") as f:
            f.write(struct.pack("<4I4iQ", 0x32505354, 1, 4, n, B, X, Y, 0, 0x1234))
        procs = []
        for r in range(2):
            env = dict(_clean_env(), PMI_SIZE="2", PMI_RANK=str(r), TSP_GATHER_DIR=gd)
            procs.append(subprocess.Popen([tspgpu.TSP_BIN, *map(str, case["args"])], stdout=subprocess.PIPE,
                                          stderr=subprocess.PIPE, text=True, env=env))
        outs = [p.communicate(timeout=300) for p in procs]
        assert procs[0].returncode == 0, outs[0][1]
        assert _norm(outs[0][0]) == _expect(case)
        assert os.listdir(gd) == []


def test_failed_worker_rank_ends_the_wait_at_once():
    """A worker rank that fails publishes a failure record: rank 0 exits with
    that rank's error within seconds instead of polling for 600 s."""
    import time

    case = _two_rank_case()
    with tempfile.TemporaryDirectory() as gd:
        t0 = time.monotonic()
        procs = []
        for r in range(2):
            env = dict(_clean_env(), PMI_SIZE="2", PMI_RANK=str(r), TSP_GATHER_DIR=gd, TSP_INJECT_FAIL_RANK="1")
            procs.append(subprocess.Popen([tspgpu.TSP_BIN, *map(str, case["args"])], stdout=subprocess.PIPE,
                                          stderr=subprocess.PIPE, text=True, env=env))
        outs = [p.communicate(timeout=120) for p in procs]
        assert procs[1].returncode == 3 and procs[0].returncode == 3, [o[1] for o in outs]
        assert "rank 1 failed" in outs[0][1]
        assert time.monotonic() - t0 < 60
