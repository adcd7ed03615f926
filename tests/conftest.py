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


@pytest.fixture
def engine():
    """A fresh engine on cuda:0 with small segments (exercise segment boundaries)."""
    from clonos_amd import Engine
    e = Engine(segment_bytes=256, pool_segments=1 << 16, timing=True)
    yield e
    e.close()
