"""GPU: batched decode (HIP) == the CPU oracle's sequential decodeNext loop, bit-exact.

Covers: every tag with random values, Serializable streams, spans crossing 16 KiB tiles
and HBM segment boundaries, unaligned span starts, empty spans, many spans per batch,
pathological non-self-synchronising streams (runs of Order(0)), records longer than the
transfer-table domain, and every error class with its offset and tag.
"""
import numpy as np
import pytest

import _oracle as O
from clonos_amd import ClonosError, CausalLogID
from clonos_amd import determinants as D
from clonos_amd import synth

pytestmark = pytest.mark.gpu


def assert_span_equal(dec, s, buf):
    st, r, _, _ = O.decode(buf)
    assert st == 0
    sl = dec.span_slice(s)
    assert sl.stop - sl.start == len(r["tag"])
    np.testing.assert_array_equal(dec.off[sl], r["off"])
    np.testing.assert_array_equal(dec.tag[sl], r["tag"])
    np.testing.assert_array_equal(dec.v0[sl], r["v0"])
    # wide rows of this span
    wsel = (dec.w_idx >= sl.start) & (dec.w_idx < sl.stop)
    np.testing.assert_array_equal(dec.w_idx[wsel] - sl.start, r["w_idx"])
    np.testing.assert_array_equal(dec.w_rc[wsel], r["w_rc"])
    np.testing.assert_array_equal(dec.w_v1[wsel], r["w_v1"])
    np.testing.assert_array_equal(dec.w_var_off[wsel], r["w_var_off"])
    np.testing.assert_array_equal(dec.w_var_len[wsel], r["w_var_len"])
    np.testing.assert_array_equal(dec.w_sub[wsel], r["w_sub"])


@pytest.mark.parametrize("seed", range(4))
def test_decode_random_all_tags(engine, seed):
    rng = np.random.default_rng(seed)
    buf = synth.random_log(3000, rng)
    dec = engine.decode_host(buf)
    assert_span_equal(dec, 0, buf)


def test_decode_many_spans_unaligned(engine):
    rng = np.random.default_rng(7)
    parts = [synth.random_log(int(rng.integers(0, 400)), rng) for _ in range(40)]
    blob = b""
    spans = []
    for p in parts:
        pad = int(rng.integers(0, 17))
        blob += bytes(pad)
        spans.append((len(blob), len(p)))
        blob += p
    dec = engine.decode_host(blob, spans)
    for s, p in enumerate(parts):
        assert_span_equal(dec, s, p)
    assert dec.span_rec_base[-1] == dec.n_rec


def test_decode_config2_large(engine):
    rng = np.random.default_rng(synth.SEED_CONFIG2)
    buf, offs = synth.config2_log(400_000, rng)
    dec = engine.decode_host(buf.tobytes())
    assert dec.n_rec == 400_000
    np.testing.assert_array_equal(dec.off, offs.astype(np.uint32))
    assert_span_equal(dec, 0, buf.tobytes())


def test_decode_config3_mixed(engine):
    rng = np.random.default_rng(synth.SEED_CONFIG3)
    buf, offs = synth.config3_epoch(60_000, rng)
    dec = engine.decode_host(buf.tobytes())
    assert dec.n_rec == 60_000
    assert_span_equal(dec, 0, buf.tobytes())


@pytest.mark.parametrize("n", [0, 1, 2, 3, 15, 16, 17, 255, 256, 257, 16383, 16384, 16385, 40000])
def test_decode_order_zero_runs(engine, n):
    # Order(0) = 00 00: every byte offset parses, speculative paths never converge
    buf = D.encode(D.OrderDeterminant(0)) * n
    dec = engine.decode_host(buf)
    assert dec.n_rec == n
    assert (dec.tag == 0).all() and (dec.v0 == 0).all()
    np.testing.assert_array_equal(dec.off, np.arange(n, dtype=np.uint32) * 2)


def test_decode_long_records(engine):
    rng = np.random.default_rng(11)
    recs = []
    for i in range(300):
        k = i % 4
        if k == 0:
            recs.append(D.encode(D.TimerTriggerDeterminant(i, i, D.INTERNAL, b"n" * int(rng.integers(60, 5000)))))
        elif k == 1:
            recs.append(D.encode(D.SourceCheckpointDeterminant(i, i, i, D.SAVEPOINT, bytes(int(rng.integers(100, 20000))))))
        elif k == 2:
            recs.append(D.encode(D.SerializableDeterminant(D.jser_int_array(list(range(int(rng.integers(20, 3000))))))))
        else:
            recs.append(D.encode(D.OrderDeterminant(1)) * int(rng.integers(1, 50)))
    buf = b"".join(recs)
    dec = engine.decode_host(buf)
    assert_span_equal(dec, 0, buf)


@pytest.mark.parametrize("prefix_n,bad", [
    (1000, b"\x08"),
    (5000, b"\xff"),
    (2000, b"\x04" + b"\x00" * 12 + b"\x07" + b"\x00"),
    (3000, b"\x04" + b"\x00" * 12 + b"\x06" + b"\xff\xff\xff\xff"),
    (100, b"\x05" + b"\x00" * 20 + b"\x05\x00"),
    (4000, b"\x01\x00\x00"),
    (10, b"\x03\xac\xed\x00\x05\x99"),
])
def test_decode_errors(engine, prefix_n, bad):
    rng = np.random.default_rng(prefix_n)
    prefix = synth.random_log(prefix_n, rng, allow_serializable=False)
    buf = prefix + bad + synth.random_log(50, rng, allow_serializable=False)
    st, r, eo, et = O.decode(buf)
    assert st != 0
    with pytest.raises(ClonosError) as ex:
        engine.decode_host(buf)
    assert ex.value.status == st
    assert ex.value.err_off == eo and ex.value.err_tag == et


def test_decode_logs_in_hbm(engine):
    """decode_logs reads the segments in place: spans start mid-segment after truncation."""
    rng = np.random.default_rng(5)
    logs, expect = [], []
    for v in range(12):
        log = engine.open_log(CausalLogID.main(v))
        for ep in range(4):
            for _ in range(int(rng.integers(50, 900))):
                log.appendDeterminant(synth.random_determinant(rng), ep)
        if v % 2:
            log.notifyCheckpointComplete(2)
        logs.append(log)
    start = [int(rng.integers(0, 4)) for _ in logs]
    for log, e in zip(logs, start):
        expect.append(log.getDeterminants(e))
    dec = engine.decode_logs(logs, start)
    for s, b in enumerate(expect):
        assert_span_equal(dec, s, b)


@pytest.mark.parametrize("seg", [48, 4096, 65536])
def test_decode_logs_segment_sizes(seg):
    """Tiles are planned on the device when the segment size and the 16 KiB tile divide
    one another (4096, 65536) and on the host otherwise (48); both decode bit-exactly."""
    from clonos_amd import Engine
    rng = np.random.default_rng(seg)
    with Engine(segment_bytes=seg, pool_segments=(1 << 22) // seg + 64) as eng:
        logs, expect = [], []
        for v in range(5):
            log = eng.open_log(CausalLogID.main(v))
            b, _ = synth.config2_log(int(rng.integers(1000, 60000)), rng)
            log.processUpstreamDelta(b.tobytes(), 0, 0)
            for _ in range(int(rng.integers(0, 400))):
                log.appendDeterminant(synth.random_determinant(rng), 1)
            logs.append(log)
        start = [int(rng.integers(0, 2)) for _ in logs]
        expect = [log.getDeterminants(e) for log, e in zip(logs, start)]
        dec = eng.decode_logs(logs, start)
        for s, b in enumerate(expect):
            assert_span_equal(dec, s, b)
