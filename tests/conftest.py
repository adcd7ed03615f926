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


@pytest.fixture(params=["auto", "robust", "one_pass"])
def engine(request, monkeypatch):
    """A fresh engine on cuda:0 with small segments (exercise segment boundaries): with the
    fast decode (single-launch small path, one-pass or three-pass decode, robust pipeline on
    abort), robust-only, and with the one-pass decode forced onto every batch it may take
    (CLONOS_ONE_PASS=2, no small path; its aborts go to the three passes)."""
    from clonos_amd import Engine
    if request.param == "one_pass":
        monkeypatch.setenv("CLONOS_ONE_PASS", "2")
        e = Engine(segment_bytes=256, pool_segments=1 << 16, timing=True, decode="three_pass")
        monkeypatch.delenv("CLONOS_ONE_PASS")
    else:
        e = Engine(segment_bytes=256, pool_segments=1 << 16, timing=True, decode=request.param)
    yield e
    e.close()
