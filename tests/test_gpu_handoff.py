"""GPU: the decode's cross-block hand-offs are checked after the fact, so a wrong read of a
published word cannot change a result.

The fast decode passes three kinds of word from one workgroup to another while both run:
a chunk's entry (the count pass: the previous chunk's published exit), the small path's
tile entries and running bases, and the one-launch scan's look-back prefixes.  Each is now
verified once its producer is done ("Hand-off checks"):

* k_decode_repair compares the entry every chunk took with the true exit of the tile before
  it and walks the chunk again when they differ;
* the host compares every small-path tile's entry and base with its predecessor's exit and
  base, and decodes the batch the three-pass way when one differs;
* emit compares every scan block's offset with its predecessor's final prefix, and the host
  decodes the batch again when one differs.

CLONOS_FUSED_PERTURB (a test switch, read when an engine opens) plants the faults: bits 15:0
are added to every hand-off entry, bit 16 raises scan block 1's look-back result by one
record.  A +2 entry in a run of channel-0 Order records ("00 00") is a valid chain that
drops one record per chunk: without the check it would decode silently wrong.  Every case is
compared record for record with the CPU oracle.
"""
import numpy as np
import pytest

from clonos_amd import CausalLogID, Engine
from clonos_amd import synth
from test_gpu_decode import assert_span_equal

pytestmark = pytest.mark.gpu


def _count(eng, name):
    return eng.kernel_stats().get(name, {}).get("launches", 0)


def _log(kind, n_bytes, seed):
    rng = np.random.default_rng(seed)
    if kind == "zeros":  # Order(channel 0) records: valid at every even offset
        return bytes(n_bytes & ~1)
    if kind == "config2":
        b, _ = synth.config2_log(n_bytes // 6, rng)
        return b.tobytes()
    return synth.random_log(n_bytes // 7, rng, allow_serializable=False)


@pytest.fixture
def perturbed(monkeypatch):
    engines = []

    def make(perturb, **kw):
        monkeypatch.setenv("CLONOS_FUSED_PERTURB", str(perturb))
        e = Engine(timing=True, **kw)
        monkeypatch.delenv("CLONOS_FUSED_PERTURB")
        engines.append(e)
        return e

    yield make
    for e in engines:
        e.close()


@pytest.mark.parametrize("kind", ["zeros", "config2", "mixed"])
@pytest.mark.parametrize("perturb", [2, 1, 9])
def test_wrong_chunk_entries_are_repaired(perturbed, kind, perturb):
    eng = perturbed(perturb, decode="three_pass")
    buf = _log(kind, 3 << 20, 7 + perturb)
    dec = eng.decode_host(buf)
    assert_span_equal(dec, 0, buf)
    assert _count(eng, "decode_entry_repair") + _count(eng, "decode_chunk_repair") >= 1
    assert _count(eng, "decode_fallback") == 0


def test_zero_run_plus_two_is_caught_by_the_entry_check(perturbed):
    """The silent case: every perturbed chain is valid, so only the entry check sees it."""
    eng = perturbed(2, decode="three_pass")
    buf = _log("zeros", 2 << 20, 0)
    dec = eng.decode_host(buf)
    assert_span_equal(dec, 0, buf)
    assert _count(eng, "decode_entry_repair") >= 1
    assert _count(eng, "decode_fallback") == 0


def test_wrong_entries_in_logs_in_hbm(perturbed):
    """The bench's shape: several logs in HBM segments, decoded as one batch."""
    eng = perturbed(2, decode="three_pass")
    rng = np.random.default_rng(5)
    logs, blobs = [], []
    for v in range(6):
        log = eng.open_log(CausalLogID.main(v))
        b, _ = synth.config2_log(int(rng.integers(150_000, 400_000)), rng)
        log.processUpstreamDelta(b.tobytes(), 0, 0)
        logs.append(log)
        blobs.append(b.tobytes())
    dec = eng.decode_logs(logs, [0] * len(logs))
    for s, b in enumerate(blobs):
        assert_span_equal(dec, s, b)
    assert _count(eng, "decode_entry_repair") >= 1
    assert _count(eng, "decode_fallback") == 0


@pytest.mark.parametrize("kind,perturb", [("zeros", 2), ("config2", 3), ("mixed", 1)])
def test_small_path_entries_checked_by_the_host(perturbed, kind, perturb):
    """decode="auto": the single-launch path for batches up to 1 MiB.  A wrong entry whose
    chain fails flags the batch in the kernel; one whose chain is valid (zeros, +2) is caught
    only by the host's check of the tiles' hand-off words."""
    eng = perturbed(perturb)
    buf = _log(kind, 300_000, 11)
    dec = eng.decode_host(buf)
    assert_span_equal(dec, 0, buf)
    assert _count(eng, "decode_small_fallback") >= 1
    if kind == "zeros":
        assert _count(eng, "decode_small_handoff") >= 1


def test_wrong_lookback_prefix_is_caught(perturbed):
    eng = perturbed(1 << 16, decode="three_pass")
    buf = _log("config2", 12 << 20, 3)  # > 1024 tiles: two scan blocks at least
    dec = eng.decode_host(buf)
    assert_span_equal(dec, 0, buf)
    assert _count(eng, "decode_lookback_check") >= 1


@pytest.mark.parametrize("kind", ["config2", "mixed"])
def test_no_check_fires_without_faults(kind):
    e = Engine(timing=True, decode="three_pass")
    try:
        buf = _log(kind, 12 << 20, 21)
        for _ in range(3):
            dec = e.decode_host(buf)
        assert_span_equal(dec, 0, buf)
        st = e.kernel_stats()
        for name in ("decode_entry_repair", "decode_lookback_check", "decode_canon_before_end", "decode_fallback"):
            assert name not in st, name
    finally:
        e.close()
