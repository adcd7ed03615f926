"""GPU: the fast decode path (decode_fused.hip: count / offsets / emit) on its own.

Every case checks bit-exactness against the CPU oracle's sequential decodeNext loop AND
which path produced the output: logs without Serializable records must be decoded by the
fast path itself (no `decode_fallback`), logs it cannot handle (Serializable streams,
decode errors, chains that never re-synchronise across a tile) must fall back to the
robust pipeline and still match.
"""
import numpy as np
import pytest

import _oracle as O
from clonos_amd import CausalLogID, ClonosError, Engine
from clonos_amd import determinants as D
from clonos_amd import synth
from test_gpu_decode import assert_span_equal

pytestmark = pytest.mark.gpu


def fell_back(eng) -> bool:
    return "decode_fallback" in eng.kernel_stats()


@pytest.fixture(params=[256, 16384])
def feng(request):
    e = Engine(segment_bytes=request.param, pool_segments=(1 << 26) // request.param, timing=True, decode="three_pass")
    yield e
    e.close()


@pytest.mark.parametrize("seed", range(6))
def test_fused_random_no_serializable(feng, seed):
    rng = np.random.default_rng(100 + seed)
    buf = synth.random_log(20000, rng, allow_serializable=False)
    dec = feng.decode_host(buf)
    assert_span_equal(dec, 0, buf)
    st = feng.kernel_stats()
    assert ("decode_one" in st or "decode_count" in st) and not fell_back(feng)


def test_fused_config2_multi_span(feng):
    rng = np.random.default_rng(synth.SEED_CONFIG2)
    parts, spans, blob = [], [], b""
    for i in range(9):
        b, _ = synth.config2_log(int(rng.integers(0, 60000)) if i != 4 else 0, rng)
        pad = int(rng.integers(0, 17))
        blob += bytes(pad)
        spans.append((len(blob), b.size))
        blob += b.tobytes()
        parts.append(b.tobytes())
    dec = feng.decode_host(blob, spans)
    for s, p in enumerate(parts):
        assert_span_equal(dec, s, p)
    assert dec.span_rec_base[-1] == dec.n_rec
    assert not fell_back(feng)


def test_fused_far_garbage_lengths(feng):
    """Timestamps whose bytes look like a TimerTrigger with a huge name length: a
    speculative chain that starts inside them must not jump past the tile."""
    ts = []
    for i in range(40000):
        # 04 .. at byte 1, type byte 06 at +13 and a name length of ~0x0002_0000
        ts.append(D.TimestampDeterminant(0x0400000000000000 | (i & 0xFFFF)))
        ts.append(D.OrderDeterminant(6))
        ts.append(D.RNGDeterminant(0x00020000 + i))
    buf = b"".join(D.encode(r) for r in ts)
    dec = feng.decode_host(buf)
    assert_span_equal(dec, 0, buf)
    assert not fell_back(feng)


def test_fused_logs_in_hbm_after_truncation(feng):
    rng = np.random.default_rng(31)
    logs = []
    for v in range(10):
        log = feng.open_log(CausalLogID.main(v))
        b, _ = synth.config2_log(int(rng.integers(1000, 40000)), rng)
        log.processUpstreamDelta(b.tobytes(), 0, 0)
        for ep in range(1, 4):
            for _ in range(int(rng.integers(10, 500))):
                log.appendDeterminant(synth.random_determinant(rng, allow_serializable=False), ep)
        if v % 3 == 0:
            log.notifyCheckpointComplete(2)
        logs.append(log)
    start = [int(rng.integers(0, 4)) for _ in logs]
    expect = [log.getDeterminants(e) for log, e in zip(logs, start)]
    dec = feng.decode_logs(logs, start)
    for s, b in enumerate(expect):
        assert_span_equal(dec, s, b)
    assert not fell_back(feng)


def test_fused_wide_records_side_table(feng):
    rng = np.random.default_rng(9)
    recs = []
    for i in range(6000):
        k = i % 5
        if k == 0:
            recs.append(D.TimerTriggerDeterminant(i, i * 3, D.INTERNAL, b"PTS"))
        elif k == 1:
            recs.append(D.SourceCheckpointDeterminant(i, i, i + 1, D.CHECKPOINT, b"ref" * (i % 7)))
        elif k == 2:
            recs.append(D.IgnoreCheckpointDeterminant(i, i * 7))
        else:
            recs.append(synth.random_determinant(rng, allow_serializable=False))
    buf = b"".join(D.encode(r) for r in recs)
    dec = feng.decode_host(buf)
    assert_span_equal(dec, 0, buf)
    assert not fell_back(feng)


def test_fused_serializable_tables(feng):
    """Serializable streams: the first batch aborts once (no tables), re-runs with the
    phase-3 length tables and stays on the fast path; the next batch builds the tables
    up front (no retry)."""
    rng = np.random.default_rng(3)
    buf, _ = synth.config3_epoch(20000, rng)
    dec = feng.decode_host(buf.tobytes())
    assert_span_equal(dec, 0, buf.tobytes())
    st = feng.kernel_stats()
    if feng.segment_bytes == 16384:
        assert not fell_back(feng)
        assert st["decode_jser_retry"]["launches"] == 1
    feng.kernel_stats_reset()
    buf2, _ = synth.config3_epoch(30000, rng)
    dec = feng.decode_host(buf2.tobytes())
    assert_span_equal(dec, 0, buf2.tobytes())
    st = feng.kernel_stats()
    if feng.segment_bytes == 16384:  # 256-byte tiles re-synchronise too rarely: robust path
        assert "decode_jser_retry" not in st and st["decode_jser"]["launches"] == 1
        assert not fell_back(feng)


def test_fused_serializable_long_streams(feng):
    """Streams far longer than a tile (int[] of 6000 elements = 24 KiB) and strings placed
    across tile boundaries: the table kernel reads past its LDS image from HBM."""
    rng = np.random.default_rng(11)
    parts = []
    for i in range(40):
        k = int(rng.integers(0, 4))
        if k == 0:
            parts.append(D.encode(D.SerializableDeterminant(D.jser_int_array(
                rng.integers(-2**31, 2**31, int(rng.integers(1000, 6000))).tolist()))))
        elif k == 1:
            parts.append(D.encode(D.SerializableDeterminant(D.jser_string("x" * int(rng.integers(0, 9000))))))
        else:
            parts.append(synth.random_log(int(rng.integers(1, 900)), rng, allow_serializable=(k == 2)))
    buf = b"".join(parts)
    dec = feng.decode_host(buf)
    assert_span_equal(dec, 0, buf)


def test_fused_tables_long_wide_records(feng):
    """With Serializable tables the count pass walks a step-code map whose codes hold
    lengths up to 126 bytes: longer TimerTrigger names, SourceCheckpoint references and
    Serializable streams get code 0x80, and the true walk measures them from HBM (TimerTrigger /
    SourceCheckpoint by the decodeNext rules, Serializable from the table), as does the
    canonical walk, so such a record across a chunk's last tile end leaves the published exit
    where the true chain exits.  Bit-exact against the oracle, on the batch that builds the
    tables and on the next one, and (16 KiB segments) without falling back."""
    rng = np.random.default_rng(21)
    for _ in range(2):
        parts = []
        for i in range(400):
            parts.append(synth.config3_epoch(int(rng.integers(5, 60)), rng)[0].tobytes())
            k = i % 4
            n = int(rng.integers(100, 320))
            if k == 0:
                parts.append(D.encode(D.TimerTriggerDeterminant(i, 7 * i, D.INTERNAL, b"A" * n)))
            elif k == 1:
                parts.append(D.encode(D.SourceCheckpointDeterminant(i, i, 3 * i, D.CHECKPOINT, b"r" * n)))
            elif k == 2:
                parts.append(D.encode(D.SerializableDeterminant(D.jser_string("s" * n))))
        buf = b"".join(parts)
        feng.kernel_stats_reset()
        dec = feng.decode_host(buf)
        assert_span_equal(dec, 0, buf)
        assert "decode_jser" in feng.kernel_stats()
        if feng.segment_bytes == 16384:
            assert not fell_back(feng)


def test_fused_long_names_no_tables(feng):
    """No Serializable records (no tables): TimerTrigger names and SourceCheckpoint
    references of 200-1500 bytes, past the 256 bytes the speculative rule follows.  The
    canonical walk measures them by the full rules, so the batch stays on the fast path
    (16 KiB segments) and matches the oracle bit for bit."""
    rng = np.random.default_rng(23)
    parts = []
    for i in range(300):
        parts.append(synth.random_log(int(rng.integers(5, 80)), rng, allow_serializable=False))
        n = int(rng.integers(200, 1500))
        if i % 2:
            parts.append(D.encode(D.TimerTriggerDeterminant(i, 5 * i, D.INTERNAL, b"N" * n)))
        else:
            parts.append(D.encode(D.SourceCheckpointDeterminant(i, i, 2 * i, D.CHECKPOINT, b"R" * n)))
    buf = b"".join(parts)
    dec = feng.decode_host(buf)
    assert_span_equal(dec, 0, buf)
    if feng.segment_bytes == 16384:
        assert not fell_back(feng)


@pytest.mark.parametrize("bad", ["magic_no_object", "truncated_stream", "bad_magic"])
def test_fused_serializable_errors(feng, bad):
    """Invalid Serializable records after valid ones: same status / offset / tag as the
    oracle (the fast path falls back and the robust pipeline classifies)."""
    rng = np.random.default_rng(12)
    good, _ = synth.config3_epoch(3000, rng)
    tail = {"magic_no_object": b"\x03\xac\xed\x00\x05\x70" [:-1] + b"\x99",
            "truncated_stream": D.encode(D.SerializableDeterminant(D.jser_string("abcdef")))[:-2],
            "bad_magic": b"\x03\xac\xed\x00\x06\x74\x00\x00"}[bad]
    buf = good.tobytes() + tail
    st, r, eo, et = O.decode(buf)
    assert st != 0
    with pytest.raises(ClonosError) as ei:
        feng.decode_host(buf)
    assert ei.value.status == st and ei.value.err_off == eo and ei.value.err_tag == et


@pytest.mark.parametrize("n", [100, 5000, 30000])
def test_fused_odd_chain_never_merges(feng, n):
    """Timestamp (9 bytes) then Order(0) runs: the true chain sits on odd offsets, every
    speculative chain on even ones.  Single tiles still settle; multi-tile spans abort."""
    buf = D.encode(D.TimestampDeterminant(5)) + D.encode(D.OrderDeterminant(0)) * n
    dec = feng.decode_host(buf)
    st, r, _, _ = O.decode(buf)
    assert st == 0 and dec.n_rec == n + 1
    np.testing.assert_array_equal(dec.off, r["off"])


def test_fused_device_output_large(feng):
    """Many tiles (the decoupled look-back chain); with 256-byte segments every tile is
    one segment, too short for the speculative chains to re-synchronise reliably, so
    only the 16 KiB configuration must stay on the fused path."""
    rng = np.random.default_rng(77)
    logs = []
    for v in range(16):
        log = feng.open_log(CausalLogID.main(v))
        b, _ = synth.config2_log(200_000, rng)
        log.processUpstreamDelta(b.tobytes(), 0, 1)
        logs.append(log)
    expect = [log.getDeterminants(1) for log in logs]
    dec = feng.decode_logs(logs, [1] * len(logs))
    for s, b in enumerate(expect):
        assert_span_equal(dec, s, b)
    if feng.segment_bytes >= 8192:
        assert not fell_back(feng)


@pytest.mark.parametrize("kind", ["strings", "nulls"])
def test_fused_dense_serializable_overflow(feng, kind):
    """Tiles holding more Serializable streams than the 256 table entries kept in LDS: short
    strings (9-21 byte records, ~500 per 8 KiB tile) and TC_NULL streams (6 bytes, ~1300 per
    tile, every one through the general walker's work list).  The entries past 256 go to the
    overflow arena in HBM (the arena or the work list grows and the batch runs again when
    they are full), so the batch stays on the fast path (16 KiB segments) -- it used to abort
    to the robust pipeline -- and matches the oracle bit for bit, over several spans."""
    rng = np.random.default_rng(41 if kind == "strings" else 43)
    parts = []
    for s in range(3):
        recs = []
        for i in range(int(rng.integers(30000, 60000))):
            if i % 97 == 0:
                recs.append(synth.random_determinant(rng, allow_serializable=False))
            elif kind == "strings":
                recs.append(D.SerializableDeterminant(D.jser_string("s" * int(rng.integers(0, 13)))))
            else:
                recs.append(D.SerializableDeterminant(D.jser_null()))
        parts.append(b"".join(D.encode(r) for r in recs))
    blob, spans = b"", []
    for p in parts:
        spans.append((len(blob), len(p)))
        blob += p
    for _ in range(2):  # the batch that grows the arenas, then one that fits
        feng.kernel_stats_reset()
        dec = feng.decode_host(blob, spans)
        for s, p in enumerate(parts):
            assert_span_equal(dec, s, p)
        ks = feng.kernel_stats()
        if feng.segment_bytes == 16384:
            assert not fell_back(feng) and "decode_span_fallback" not in ks, ks


@pytest.mark.parametrize("where", [0.2, 0.9])
def test_fused_dense_serializable_error_past_lds_entries(feng, where):
    """A dense tile of short strings whose invalid stream (a truncated string: its length
    runs past the span end, or a bad type code) sits past the 256 entries LDS holds: the
    error is the oracle's (status, offset, tag), from the table's overflow entries."""
    rng = np.random.default_rng(47)
    recs = [D.encode(D.SerializableDeterminant(D.jser_string("s" * int(rng.integers(0, 13)))))
            for _ in range(20000)]
    k = int(len(recs) * where)
    recs[k] = b"\x03\xac\xed\x00\x05\x99"  # magic, then no valid type code
    buf = b"".join(recs)
    st, r, eo, et = O.decode(buf)
    assert st != 0
    with pytest.raises(ClonosError) as ei:
        feng.decode_host(buf)
    assert ei.value.status == st and ei.value.err_off == eo and ei.value.err_tag == et
