"""CPU: the polled hand-off word encoding of the fused decode (clonos_amd/csrc/handoff.h).

Compiled for the host from the header the kernels include.  A published word round-trips its
state and 60-bit value; the zeroed word, and any word made of one write's high half and
another's low half (a torn read, or a state-to-state mix such as the scan's aggregate then
inclusive prefix), reads as not published -- so a poll never takes a mixed value.
"""
import ctypes as C
import os
import random
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
MASK60 = (1 << 60) - 1


@pytest.fixture(scope="module")
def ho(tmp_path_factory):
    so = str(tmp_path_factory.mktemp("handoff") / "libhandoff.so")
    hipcc = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
    subprocess.run([hipcc, "-x", "hip", "--offload-host-only", "-O2", "-std=c++17", "-fPIC", "-shared", "-o", so,
                    os.path.join(ROOT, "tests", "handoff_host.cpp")], check=True)
    lib = C.CDLL(so)
    lib.ho_word.restype = C.c_uint64
    lib.ho_word.argtypes = [C.c_uint32, C.c_uint64]
    lib.ho_state.restype = C.c_uint32
    lib.ho_state.argtypes = [C.c_uint64]
    lib.ho_val.restype = C.c_uint64
    lib.ho_val.argtypes = [C.c_uint64]
    return lib


def _values(rng):
    edge = [0, 1, (1 << 30) - 1, 1 << 30, (1 << 30) + 1, (1 << 32) - 1, 1 << 32, 0x464003, MASK60]
    return edge + [rng.getrandbits(60) for _ in range(200)] + [rng.getrandbits(34) for _ in range(200)]


def test_round_trip(ho):
    rng = random.Random(5)
    for s in (1, 2, 3):
        for v in _values(rng):
            w = ho.ho_word(s, v)
            assert ho.ho_state(w) == s and ho.ho_val(w) == v


def test_unpublished_words(ho):
    assert ho.ho_state(0) == 0
    assert ho.ho_state(1 << 62) == 0  # the tiny pass's st_x marker is not a published exit
    assert ho.ho_state(1 << 63) == 0  # the old encoding's "published, offset 0"


def test_mixed_halves_read_unpublished(ho):
    rng = random.Random(7)
    lo32 = (1 << 32) - 1
    for _ in range(3000):
        s1, s2 = rng.choice([(0, 1), (0, 2), (0, 3), (1, 2), (2, 1), (1, 3), (2, 3), (3, 2), (3, 0), (2, 0)])
        a = ho.ho_word(s1, rng.getrandbits(60)) if s1 else 0
        b = ho.ho_word(s2, rng.getrandbits(60)) if s2 else 0
        for torn in ((a & ~lo32) | (b & lo32), (b & ~lo32) | (a & lo32)):
            assert ho.ho_state(torn) == 0
