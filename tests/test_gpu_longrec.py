"""GPU: records longer than a fast-decode tile (8 KiB), and spans the fast path cannot
settle, cost only their own span.

A TimerTrigger name of 40 KB or a Serializable stream of 9 KB anywhere in a batch used to
send the whole batch to the robust pipeline, and in round 3 still its span (the per-span
fallback).  Now such records stay on the fast path: a record that crosses a chunk boundary of
the count pass is repaired there (k_decode_repair), and only a span the fast rules cannot
settle goes robust.  Each case is bit-exact against the oracle (16 KiB segments; a record
may cross segments, tiles and the count pass's chunk boundaries).  SimpleDeterminantEncoder.java:228-242 (TimerTrigger
name), :273-287 (SourceCheckpoint reference), :333-341 (Serializable stream)."""
import numpy as np
import pytest

import _oracle as O
from clonos_amd import ClonosError, Engine
from clonos_amd import determinants as D
from clonos_amd import synth
from test_gpu_decode import assert_span_equal

pytestmark = pytest.mark.gpu


def fell_back(eng) -> bool:
    return "decode_fallback" in eng.kernel_stats()


def went_robust(eng) -> bool:
    """Any robust decode: the whole batch or a span of it."""
    ks = eng.kernel_stats()
    return "decode_fallback" in ks or "decode_span_fallback" in ks


def _join(spans):
    blob, sp = b"", []
    for b in spans:
        sp.append((len(blob), len(b)))
        blob += b
    return blob, sp


@pytest.fixture
def leng():
    e = Engine(segment_bytes=16384, pool_segments=1 << 14, timing=True, decode="three_pass")
    yield e
    e.close()


def _long(kind: str, n: int, i: int = 0) -> bytes:
    if kind == "timer":
        return D.encode(D.TimerTriggerDeterminant(i, 7 * i, D.INTERNAL, bytes([65 + i % 26]) * n))
    if kind == "checkpoint":
        return D.encode(D.SourceCheckpointDeterminant(i, i, 3 * i, D.CHECKPOINT, b"r" * n))
    if kind == "string":
        return D.encode(D.SerializableDeterminant(D.jser_string("s" * n)))
    if kind == "intarray":
        return D.encode(D.SerializableDeterminant(D.jser_int_array(list(range(n // 4)))))
    raise ValueError(kind)


@pytest.mark.parametrize("kind,n", [("timer", 40000), ("checkpoint", 20000), ("string", 9000),
                                    ("intarray", 9000), ("timer", 9000), ("string", 30000)])
def test_long_record_span_alone(leng, kind, n):
    """One long record in one span of a batch of twelve: the batch stays on the fast path
    (neither decode_span_fallback nor decode_fallback); bit-exact.  The batch is small, so
    every count-pass chunk is one tile and the record crosses several chunk boundaries."""
    rng = np.random.default_rng(n)
    for pos in range(3):  # the long record at different offsets (tile / chunk phases)
        spans = [synth.config3_epoch(8000, rng)[0].tobytes() for _ in range(12)]
        head = synth.config3_epoch(3000 + 1777 * pos, rng)[0].tobytes()
        spans[5] = head + _long(kind, n, pos) + spans[5]
        blob, sp = b"", []
        for b in spans:
            sp.append((len(blob), len(b)))
            blob += b
        for _ in range(2):  # the first batch may learn the Serializable table hint
            leng.kernel_stats_reset()
            dec = leng.decode_host(blob, sp)
            for s_, b in enumerate(spans):
                assert_span_equal(dec, s_, b)
        assert not went_robust(leng), (kind, n, pos, leng.kernel_stats())


def test_config3_batch_with_long_records(leng):
    """The verdict's case: a config-3 batch (many spans) with one 40 KB TimerTrigger name
    and one 9 KB Serializable stream, bit-exact and on the fast path."""
    rng = np.random.default_rng(0xC1050003)
    spans = []
    for i in range(12):
        b, offs = synth.config3_epoch(20000, rng)
        b = b.tobytes()
        if i == 3:
            k = int(offs[len(offs) // 2])
            b = b[:k] + _long("timer", 40000, 3) + b[k:]
        if i == 7:
            k = int(offs[len(offs) // 3])
            b = b[:k] + _long("intarray", 9000) + b[k:]
        spans.append(b)
    blob, sp = b"", []
    for b in spans:
        sp.append((len(blob), len(b)))
        blob += b
    for _ in range(2):
        leng.kernel_stats_reset()
        dec = leng.decode_host(blob, sp)
        for s, b in enumerate(spans):
            assert_span_equal(dec, s, b)
    assert not went_robust(leng), leng.kernel_stats()


@pytest.mark.parametrize("n_spans,per_span", [(6, 4000), (16, 150000)])
def test_many_long_records_repaired(leng, n_spans, per_span):
    """Several long records per span (TimerTrigger names, SourceCheckpoint references and
    Serializable streams of 9-40 KB), in a small batch (one tile per chunk) and in a 20 MB
    one (a few tiles per chunk): the count pass repairs the chunks they cross
    (decode_chunk_repair), nothing goes robust, bit-exact."""
    rng = np.random.default_rng(per_span)
    kinds = [("timer", 40000), ("intarray", 9000), ("checkpoint", 20000), ("string", 30000), ("timer", 12000)]
    spans = []
    for i in range(n_spans):
        parts = [synth.config3_epoch(per_span // 4, rng)[0].tobytes()]
        for j in range(2):
            kind, n = kinds[(i + 2 * j) % len(kinds)]
            parts.append(_long(kind, n, i + j))
            parts.append(synth.config3_epoch(per_span // 4, rng)[0].tobytes())
        spans.append(b"".join(parts))
    blob, sp = _join(spans)
    for _ in range(2):
        leng.kernel_stats_reset()
        dec = leng.decode_host(blob, sp)
        for s, b in enumerate(spans):
            assert_span_equal(dec, s, b)
        ks = leng.kernel_stats()
        assert not went_robust(leng), ks
    assert "decode_chunk_repair" in ks, ks


@pytest.mark.parametrize("bad", [b"\x08", b"\x01\x00\x00"])
def test_error_after_long_record(leng, bad):
    """A decode error a few records after a long record, where the count pass's chunk after
    the record entered at a wrong place: the repair finds the error is real, and the error
    (status, offset, tag) is the oracle's."""
    rng = np.random.default_rng(len(bad))
    buf = (synth.config3_epoch(3000, rng)[0].tobytes() + _long("timer", 40000, 1)
           + synth.config3_epoch(500, rng)[0].tobytes() + bad + synth.config3_epoch(100, rng)[0].tobytes())
    st, _, eo, et = O.decode(buf)
    assert st != 0
    with pytest.raises(ClonosError) as ex:
        leng.decode_host(buf)
    assert ex.value.status == st
    assert ex.value.err_off == eo and ex.value.err_tag == et


def test_sixty_long_records_in_two_spans(leng):
    """60 long records in two spans, each crossing several one-tile chunks: every chunk they
    cross is repaired, nothing goes robust, bit-exact."""
    rng = np.random.default_rng(77)
    parts = []
    for i in range(60):
        parts.append(synth.config3_epoch(200, rng)[0].tobytes())
        parts.append(_long("timer", 20000, i))
    spans = [b"".join(parts[:60]), b"".join(parts[60:])]
    blob, sp = _join(spans)
    leng.kernel_stats_reset()
    dec = leng.decode_host(blob, sp)
    for s, b in enumerate(spans):
        assert_span_equal(dec, s, b)
    assert not went_robust(leng), leng.kernel_stats()
    assert leng.kernel_stats()["decode_chunk_repair"]["launches"] >= 60


def _odd_chain(n):
    """A Timestamp then Order(0) runs: valid, but the true chain sits on odd offsets of the span
    and, for a span that starts 16-byte aligned, every speculative chain on even ones, so the
    fast count pass cannot settle it across tiles."""
    return D.encode(D.TimestampDeterminant(5)) + D.encode(D.OrderDeterminant(0)) * n


def test_zero_runs_settled_without_fallback(leng):
    """Two spans whose true chains sit on odd offsets of long channel-0 Order runs ("00 00"),
    among 20 ordinary ones: every chunk entered on the even chain, and the chunk-repair walk
    crosses the all-zero tiles without walking them (zero_tile_walk) -- nothing goes robust,
    every span bit-exact."""
    rng = np.random.default_rng(41)  # no Serializable records: the count pass runs without tables
    spans = [synth.config2_log(int(rng.integers(2000, 9000)), rng)[0].tobytes() for _ in range(20)]
    spans[7] = _odd_chain(30000)
    spans[13] = _odd_chain(9000)
    blob, sp = b"", []
    for i, b in enumerate(spans):
        blob += bytes(int(rng.integers(0, 16)) if i else 0)  # (decode_host stages from span 0's first byte)
        if i in (7, 13):  # 16-byte aligned: the true chain on odd tile coordinates
            blob += bytes(-len(blob) % 16)
        sp.append((len(blob), len(b)))
        blob += b
    for _ in range(2):
        leng.kernel_stats_reset()
        dec = leng.decode_host(blob, sp)
        for s, b in enumerate(spans):
            assert_span_equal(dec, s, b)
        assert dec.span_rec_base[-1] == dec.n_rec
        assert not went_robust(leng), leng.kernel_stats()


def test_long_odd_chains_past_walk_cap(leng):
    """Spans of 200 000 channel-0 Order records at odd offsets, beside ordinary spans: every
    chunk of such a span entered on the even chain, so a repair walk does not meet the old
    chain before the span's end.  Its all-zero tiles are settled without a walk and do not
    count towards kZWalkDisagree, so nothing goes robust; bit-exact."""
    rng = np.random.default_rng(45)
    spans = [synth.config2_log(20000, rng)[0].tobytes() for _ in range(12)]
    for i in (2, 5, 9):
        spans[i] = _odd_chain(200000)
    blob, sp = b"", []
    for i, b in enumerate(spans):
        if i in (2, 5, 9):
            blob += bytes(-len(blob) % 16)
        sp.append((len(blob), len(b)))
        blob += b
    leng.kernel_stats_reset()
    dec = leng.decode_host(blob, sp)
    for s, b in enumerate(spans):
        assert_span_equal(dec, s, b)
    assert not went_robust(leng), leng.kernel_stats()


def test_span_fallback_error_equals_robust():
    """A decode error in one span and an unsettled span elsewhere: the error (status, span,
    offset, tag) and the record count equal the robust pipeline's on the whole batch."""
    from clonos_amd import ClonosError
    rng = np.random.default_rng(43)
    spans = [synth.config3_epoch(3000, rng)[0].tobytes() for _ in range(12)]
    spans[4] = _odd_chain(20000)
    b9, o9 = synth.config3_epoch(3000, rng)
    k = int(o9[1500])  # a record boundary: the corrupt tag is where a record starts
    spans[9] = b9.tobytes()[:k] + b"\x7f" + b9.tobytes()[k:]
    blob, sp = b"", []
    for i, b in enumerate(spans):
        if i == 4:  # a gap: span 4 16-byte aligned (_odd_chain)
            blob += bytes(-len(blob) % 16)
        sp.append((len(blob), len(b)))
        blob += b
    errs = []
    for mode in ("auto", "robust"):
        e = Engine(segment_bytes=16384, pool_segments=1 << 13, timing=True, decode=mode if mode == "robust" else "three_pass")
        try:
            with pytest.raises(ClonosError) as ei:
                e.decode_host(blob, sp)
            x = ei.value
            errs.append((x.status, x.err_span, x.err_off, x.err_tag, x.n_rec))
            if mode == "auto":
                ks = e.kernel_stats()
                # the error span keeps its records before the error (decode_kept_errors); only a
                # span the fast rules cannot settle would go robust (decode_span_fallback)
                assert ("decode_span_fallback" in ks or "decode_kept_errors" in ks) and "decode_fallback" not in ks, ks
        finally:
            e.close()
    assert errs[0] == errs[1] and errs[0][1] == 9


@pytest.mark.parametrize("parity", ["odd", "even"])
@pytest.mark.parametrize("frac", [0.3, 0.7])
def test_config3_batch_with_zero_run(leng, parity, frac):
    """The verdict's other case: a config-3 batch (Serializable tables on) with a 64 KB run of
    channel-0 Order records ("00 00": a valid record at every offset) inserted at a record
    boundary of one span, crossing many chunk ends of the count pass; odd (after a 9-byte
    Timestamp) and even.  Bit-exact against the oracle, every span."""
    rng = np.random.default_rng(0xC1050003)
    run = (D.encode(D.TimestampDeterminant(5)) if parity == "odd" else b"") + D.encode(D.OrderDeterminant(0)) * 32768
    spans = []
    for i in range(12):
        b, offs = synth.config3_epoch(20000, rng)
        b = b.tobytes()
        if i == 5:
            k = int(offs[int(len(offs) * frac)])
            b = b[:k] + run + b[k:]
        spans.append(b)
    blob, sp = _join(spans)
    for _ in range(2):
        leng.kernel_stats_reset()
        dec = leng.decode_host(blob, sp)
        for s, b in enumerate(spans):
            assert_span_equal(dec, s, b)
        assert dec.n_rec == 12 * 20000 + 32768 + (parity == "odd")


def test_robust_config3_far_exits_bit_exact():
    """The robust pipeline alone on config-3 logs (10 epochs each): Serializable Integers (82 B)
    across 16 KiB tile ends leave all three next-tile points of a tile off the chain, so the
    last segment ends at a record start in the next tile (kEndFar) and the resolve enters the
    next tile there.  Every record equals the oracle's and no span needs the DP tables."""
    rng = np.random.default_rng(0xC1050003)
    gen = [synth.config3_epoch(40000, rng, e) for e in range(10)]
    spans = [b"".join(gen[(e + v) % 10][0].tobytes() for e in range(10)) for v in range(4)]
    blob, sp = _join(spans)
    e = Engine(segment_bytes=16384, pool_segments=1 << 13, timing=True, decode="robust")
    try:
        dec = e.decode_host(blob, sp)
        for s, b in enumerate(spans):
            assert_span_equal(dec, s, b)
        ks = e.kernel_stats()
        assert ks.get("robust_dp_spans", {}).get("launches", 0) == 0, ks
    finally:
        e.close()
