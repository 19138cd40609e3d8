import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "tsp-mpi-reduction_amd")
for p in (os.path.join(ROOT, "tests"), PKG, ROOT):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (HIP device); run with -m gpu")
    config.addinivalue_line("markers", "slow: longer CPU test")


@pytest.fixture(scope="session")
def gpu_ctx():
    import tspgpu

    ctx = tspgpu.Context(device=0)
    yield ctx
    ctx.close()


class Knobs:
    """Tuning / test knobs of libtspgpu (tspgpu_tuning_set), reset after the test."""

    def set(self, name, value):
        import tspgpu

        tspgpu.tune(name, float(value))

    def clear(self, name=None):
        import tspgpu

        tspgpu.untune(name)


@pytest.fixture
def knobs():
    k = Knobs()
    yield k
    k.clear()
