import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (runs the HIP kernels)")


def _have_gpu() -> bool:
    try:
        import torch
        return torch.cuda.is_available()
    except Exception:
        return False


@pytest.fixture(scope="session")
def have_gpu():
    return _have_gpu()


@pytest.fixture(params=["auto", "robust"])
def engine(request):
    """A fresh engine on cuda:0 with small segments (exercise segment boundaries), once
    with the fast three-pass decode (robust pipeline on abort) and once robust-only."""
    from clonos_amd import Engine
    e = Engine(segment_bytes=256, pool_segments=1 << 16, timing=True, decode=request.param)
    yield e
    e.close()
