"""GPU: Serializable records built from the reference's own JDK-written streams.

Every stream of tests/golden/jser_reference.json (199 distinct ObjectOutputStream outputs
the reference's test resources hold behind a TypeSerializerSerializationUtil length
prefix; tests/test_jser_reference.py pins the oracle and the walker source to those
lengths on the CPU) becomes a `03`-tagged record (SimpleDeterminantEncoder.java:316-323)
inside logs of every other tag: inline between other records, crossing the fast decode's
8 KiB tiles, the robust pipeline's 16 KiB tiles and 256-byte HBM segments.  Each log is
decoded through the fast three-pass path and the robust pipeline and compared with the
CPU oracle word for word; with a tiny initial spill arena the engine must grow it
(`jser_arena_grow`) and still match.  Replay-prep's subpartition classification walks
the same streams (a Serializable record in a recovery buffer).
"""
import json
import os
import struct

import numpy as np
import pytest

import _oracle as O
from clonos_amd import CausalLogID, Engine, synth
from clonos_amd import _lib
from clonos_amd.replay import DeterminantResponseEvent, prepare_replay
from test_gpu_decode import assert_span_equal

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
FIX = json.load(open(os.path.join(ROOT, "tests", "golden", "jser_reference.json")))
RECS = [b"\x03" + bytes.fromhex(x["hex"]) for x in FIX]


def _log_with_streams(rng, recs, filler_per_gap=(0, 400)):
    """Records of every other tag with the given Serializable records spliced in between."""
    parts = []
    for r in recs:
        n = int(rng.integers(*filler_per_gap))
        if n:
            parts.append(synth.random_log(n, rng, allow_serializable=False))
        parts.append(r)
    parts.append(synth.random_log(int(rng.integers(1, 300)), rng, allow_serializable=False))
    return b"".join(parts)


def _fill(n: int, rng) -> bytes:
    """Exactly n bytes of Timestamp (9 B) and Order (2 B) records; n not in {1, 3, 5, 7}."""
    k9 = n // 9
    while k9 > 0 and (n - 9 * k9) % 2:
        k9 -= 1
    assert (n - 9 * k9) % 2 == 0 and n - 9 * k9 >= 0, n
    ts = b"".join(b"\x01" + struct.pack(">q", int(x)) for x in rng.integers(0, 1 << 40, k9))
    return ts + b"\x00\x02" * ((n - 9 * k9) // 2)


def _edge_log(rng, recs, edge):
    """Each record placed so that it starts 1..40 bytes before a multiple of `edge`."""
    out = bytearray()
    for r in recs:
        want = (edge - len(out) % edge) % edge - int(rng.integers(1, 40))
        while want < 0:
            want += edge
        if want in (1, 3, 5, 7):
            want -= 1
        out += _fill(want, rng) + r
    return bytes(out)


@pytest.fixture(params=[(256, "auto"), (16384, "auto"), (256, "robust"), (16384, "robust")],
                ids=["seg256-auto", "seg16k-auto", "seg256-robust", "seg16k-robust"])
def jeng(request):
    seg, mode = request.param
    e = Engine(segment_bytes=seg, pool_segments=(1 << 26) // seg, timing=True, decode=mode)
    yield e
    e.close()


def test_every_reference_stream_inline(jeng):
    """All 199 streams in one batch of 8 logs (span by span, shuffled order)."""
    rng = np.random.default_rng(0xA5)
    order = rng.permutation(len(RECS))
    logs = [_log_with_streams(rng, [RECS[i] for i in order[k::8]]) for k in range(8)]
    blob, spans = b"", []
    for lg in logs:
        blob += bytes(int(rng.integers(0, 16)))
        spans.append((len(blob), len(lg)))
        blob += lg
    dec = jeng.decode_host(blob, spans)
    n_ser = 0
    for s, lg in enumerate(logs):
        assert_span_equal(dec, s, lg)
        sl = dec.span_slice(s)
        n_ser += int((dec.tag[sl] == 3).sum())
    assert n_ser == len(RECS)
    ser = dec.tag == 3
    assert sorted((dec.v0[ser]).tolist()) == sorted(x["len"] for x in FIX)


@pytest.mark.parametrize("edge", [8192, 16384, 256])
def test_reference_streams_across_edges(jeng, edge):
    rng = np.random.default_rng(edge)
    lg = _edge_log(rng, RECS, edge)
    dec = jeng.decode_host(lg)
    assert_span_equal(dec, 0, lg)
    assert int((dec.tag == 3).sum()) == len(RECS)


def test_reference_streams_in_hbm_logs(jeng):
    """The streams appended to engine logs (HBM segments) and decoded in place."""
    rng = np.random.default_rng(7)
    logs, want = [], []
    for v in range(16):
        lg = jeng.open_log(CausalLogID.main(v))
        b = _log_with_streams(rng, RECS[v::16], (0, 200))
        lg.processUpstreamDelta(b, 0, 0)
        logs.append(lg)
        want.append(b)
    dec = jeng.decode_logs(logs, [0] * len(logs))
    for s, b in enumerate(want):
        assert_span_equal(dec, s, b)


def test_spill_arena_grows(monkeypatch):
    """A 4 KiB initial spill arena: the 23 streams past the private tier exhaust it, the
    engine grows it and decodes again -- bit-exact, never CLG_E_BAD_SERIAL."""
    monkeypatch.setenv("CLONOS_JSER_ARENA", "4096")
    rng = np.random.default_rng(11)
    lg = _log_with_streams(rng, RECS * 3, (0, 50))
    for mode in ("auto", "robust"):
        e = Engine(segment_bytes=16384, pool_segments=4096, timing=True, decode=mode)
        try:
            dec = e.decode_host(lg)
            assert_span_equal(dec, 0, lg)
            assert "jser_arena_grow" in e.kernel_stats(), mode
        finally:
            e.close()


def test_replay_classifies_reference_streams():
    """A subpartition recovery buffer holding BufferBuilt records then a Serializable one:
    SubpartitionRecoveryThread decodes the record (walking the stream) and then fails
    the instanceof check (ReplayingState.java:172-177) -> CLG_E_NOT_BUFFER_BUILT at its
    offset; a truncated stream is CLG_E_BAD_SERIAL."""
    e = Engine(segment_bytes=16384, pool_segments=4096)
    try:
        acc = DeterminantResponseEvent(True, 3)
        subs, want = [], []
        for i, r in enumerate(RECS):
            lid = CausalLogID.sub(3, 11, 22, i % 100)
            if i >= 100:
                lid = CausalLogID.sub(3, 11, 23, i % 100)
            bb = b"".join(b"\x07" + struct.pack(">i", 1000 + k) for k in range(i % 7))
            tail = r if i % 5 else r[:-1]
            acc.put(lid, bb + tail)
            subs.append(lid)
            want.append((i % 7, _lib.CLG_E_NOT_BUFFER_BUILT if i % 5 else _lib.CLG_E_BAD_SERIAL, len(bb)))
        _, res = prepare_replay(e, [(3, acc, subs)])
        for sp, (n, st, off) in zip(res[0].subpartitions, want):
            assert len(sp.buffer_sizes) == n
            assert sp.status == st and sp.err_off == off and sp.err_tag == 3
    finally:
        e.close()
