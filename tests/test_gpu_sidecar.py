"""GPU: the write path's Serializable candidates (the per-segment sidecar, kernels.h SideCar).

k_scatter lists every "03 AC ED 00 05" it writes, with the record length where the stream's
shape is one the decode measures inline and it ends inside the written chunk; the decode's
phase 3 then builds each tile's Serializable table from that list instead of reading the
tile.  These tests cut logs at arbitrary places (inside magics, inside streams, at segment
ends), write them through the host staging path and the device batch path (several chunks
of one segment in one launch), reuse segments after truncation, overflow a segment's list,
and compare every decode with the CPU oracle -- with the sidecar on and off
(CLONOS_SIDECAR=0: every tile scanned, the previous behaviour).
"""
import numpy as np
import pytest

import _oracle as O
from clonos_amd import CausalLogID, Engine, synth, _lib
from clonos_amd import determinants as D
from test_gpu_decode import assert_span_equal

pytestmark = pytest.mark.gpu


def _ser(rng) -> bytes:
    k = int(rng.integers(0, 7))
    if k == 0:
        s = D.jser_string("x" * int(rng.integers(0, 60)))
    elif k == 1:
        s = D.jser_boolean(bool(rng.integers(0, 2)))
    elif k == 2:
        s = D.jser_integer(int(rng.integers(-2 ** 31, 2 ** 31)))
    elif k == 3:
        s = D.jser_long(int(rng.integers(-2 ** 62, 2 ** 62)))
    elif k == 4:
        s = D.jser_int_array([int(x) for x in rng.integers(0, 1000, int(rng.integers(0, 40)))])
    elif k == 5:
        s = D.jser_null()
    else:  # a long string: runs past a 256-byte segment and past a written piece
        s = D.jser_string("y" * int(rng.integers(200, 2000)))
    return D.encode(D.SerializableDeterminant(s))


def _mixed(rng, n: int, p_ser: float = 0.3) -> bytes:
    out = []
    for _ in range(n):
        if rng.random() < p_ser:
            out.append(_ser(rng))
        elif rng.random() < 0.05:  # the magic inside another record's payload (not a record start)
            out.append(D.encode(D.TimerTriggerDeterminant(1, 2, D.INTERNAL, b"\x03\xac\xed\x00\x05\x74\x00\x02hi")))
        else:
            out.append(D.encode(synth.random_determinant(rng, allow_serializable=False)))
    return b"".join(out)


def _cuts(rng, n: int, hi: int = 300):
    """Random piece boundaries of [0, n)."""
    cuts, p = [0], 0
    while p < n:
        p = min(n, p + int(rng.integers(1, hi)))
        cuts.append(p)
    return cuts


def _engine(monkeypatch, side: bool, seg: int, pool: int = 8192, decode: str = "auto") -> Engine:
    monkeypatch.setenv("CLONOS_SIDECAR", "1" if side else "0")
    return Engine(segment_bytes=seg, pool_segments=pool, decode=decode)


def _write_host(eng, logs, blobs, rng):
    """Host staging path: each piece appended and flushed on its own (a chunk per piece)."""
    for lg, b in zip(logs, blobs):
        cuts = _cuts(rng, len(b))
        for a, z in zip(cuts, cuts[1:]):
            lg.appendDeterminant(b[a:z], 0)
            eng.sync()


def _write_device(eng, logs, blobs, rng):
    """Device batch path: every piece of every log one request of ONE batch (a log's pieces in
    order; several chunks of one segment in one k_scatter launch)."""
    import torch
    from clonos_amd import dist as X
    host, reqs = bytearray(), []
    cuts = [_cuts(rng, len(b)) for b in blobs]
    for lg, b, c in zip(logs, blobs, cuts):
        for a, z in zip(c, c[1:]):
            reqs.append((lg.handle, a, 0, len(host), z - a, 0))
            host += b[a:z]
    r = np.array(reqs, X.DELTA_REQ)
    d = torch.frombuffer(bytearray(host or b"\0"), dtype=torch.uint8).to("cuda")
    _lib.check(_lib.lib.clg_upstream_delta_batch(eng.handle, r.ctypes.data, len(r), d.data_ptr(), _lib.CLG_MEM_DEVICE))
    torch.cuda.synchronize()
    assert (r["status"] == 0).all()


@pytest.mark.parametrize("side", [True, False], ids=["sidecar", "scan"])
@pytest.mark.parametrize("seg", [256, 4096, 16384])
@pytest.mark.parametrize("path", ["host", "device"])
def test_pieces_cut_anywhere(monkeypatch, side, seg, path):
    rng = np.random.default_rng(seg * 7 + (path == "device"))
    with _engine(monkeypatch, side, seg) as eng:
        n_logs = 6
        logs = [eng.open_log(CausalLogID.main(v)) for v in range(n_logs)]
        blobs = [_mixed(rng, int(rng.integers(200, 1500))) for _ in range(n_logs)]
        (_write_host if path == "host" else _write_device)(eng, logs, blobs, rng)
        for _ in range(2):  # the first batch learns that the logs hold Serializable records
            dec = eng.decode_logs(logs, [0] * n_logs)
            for s, b in enumerate(blobs):
                assert_span_equal(dec, s, b)


@pytest.mark.parametrize("cut", range(0, 14))
def test_magic_split_at_every_byte(monkeypatch, cut):
    """A Serializable record and a payload magic, the write split at each byte around them."""
    rng = np.random.default_rng(cut)
    rec = D.encode(D.SerializableDeterminant(D.jser_integer(12345)))
    tt = D.encode(D.TimerTriggerDeterminant(1, 2, D.INTERNAL, b"\x03\xac\xed\x00\x05\x74\x00\x02hi"))
    pre = synth.random_log(50, rng, allow_serializable=False)
    blob = pre + rec + tt + rec + synth.random_log(20, rng, allow_serializable=False)
    with _engine(monkeypatch, True, 16384) as eng:
        logs = []
        for k, at in enumerate((len(pre) + cut, len(pre) + len(rec) + 1 + cut)):
            lg = eng.open_log(CausalLogID.main(k))
            lg.appendDeterminant(blob[:at], 0)
            eng.sync()
            lg.appendDeterminant(blob[at:], 0)
            eng.sync()
            logs.append(lg)
        for _ in range(2):
            dec = eng.decode_logs(logs, [0, 0])
            assert_span_equal(dec, 0, blob)
            assert_span_equal(dec, 1, blob)


def test_truncated_stream_at_the_log_end(monkeypatch):
    """A log ending inside a Serializable stream (and inside a magic): the record is an error
    at its offset, as the oracle says, with the sidecar as with the scan."""
    rng = np.random.default_rng(3)
    rec = D.encode(D.SerializableDeterminant(D.jser_string("hello world")))
    base = synth.random_log(100, rng, allow_serializable=False)
    for cut in (3, 5, 9, len(rec) - 1):
        blob = base + rec[:cut]
        st, _, eo, et = O.decode(blob)
        assert st != 0
        for side in (True, False):
            with _engine(monkeypatch, side, 16384) as eng:
                lg = eng.open_log(CausalLogID.main(0))
                lg.appendDeterminant(blob, 0)
                eng.sync()
                with pytest.raises(_lib.ClonosError) as ex:
                    eng.decode_logs([lg], [0])
                assert (ex.value.status, ex.value.err_off, ex.value.err_tag) == (st, eo, et), (cut, side)


def test_segments_reused_after_truncation(monkeypatch):
    """Segments freed by a checkpoint and taken by another log start a new sidecar life: the
    old entries (other positions and lengths) are not used."""
    rng = np.random.default_rng(11)
    with _engine(monkeypatch, True, 256, pool=512) as eng:
        a = eng.open_log(CausalLogID.main(0))
        dense = b"".join(_ser(rng) for _ in range(60))
        a.appendDeterminant(dense, 0)
        eng.sync()
        tail = _mixed(rng, 30)
        a.appendDeterminant(tail, 1)
        eng.sync()
        dec = eng.decode_logs([a], [0])
        assert_span_equal(dec, 0, dense + tail)
        free0 = eng.pool_stats()[1]
        a.notifyCheckpointComplete(1)
        eng.sync()
        assert eng.pool_stats()[1] > free0
        # new logs over the freed segments: candidates at other positions, other lengths
        bs = [_mixed(rng, int(rng.integers(100, 400)), p_ser=0.4) for _ in range(4)]
        logs = [eng.open_log(CausalLogID.main(1 + k)) for k in range(4)]
        _write_host(eng, logs, bs, rng)
        for _ in range(2):
            dec = eng.decode_logs(logs + [a], [0] * 4 + [1])
            for s, b in enumerate(bs):
                assert_span_equal(dec, s, b)
            assert_span_equal(dec, 4, a.getDeterminants(1))


def test_overflowing_segment_lists_fall_back_to_the_scan(monkeypatch):
    """A 16 KiB segment of 8-byte Serializable strings holds ~2 000 candidates, past the list's
    256: its tiles are scanned, the batch's other tiles use their lists."""
    rng = np.random.default_rng(5)
    empty = D.encode(D.SerializableDeterminant(D.jser_string("")))
    assert len(empty) == 8
    with _engine(monkeypatch, True, 16384) as eng:
        dense = empty * 5000
        mixed = _mixed(rng, 3000)
        blobs = [dense, mixed, empty * 100 + _mixed(rng, 400) + empty * 2500]
        logs = [eng.open_log(CausalLogID.main(k)) for k in range(3)]
        for lg, b in zip(logs, blobs):
            lg.appendDeterminant(b, 0)
        eng.sync()
        for _ in range(2):
            dec = eng.decode_logs(logs, [0, 0, 0])
            for s, b in enumerate(blobs):
                assert_span_equal(dec, s, b)


def test_config3_epochs_equal_with_and_without_the_sidecar(monkeypatch):
    """Config 3's generator (5 % Serializable among every tag), written as the bench writes it:
    the sidecar decode equals the scan decode and the oracle, word for word."""
    rng = np.random.default_rng(synth.SEED_CONFIG3)
    epochs = [synth.config3_epoch(8000, rng, e)[0].tobytes() for e in range(4)]
    outs = []
    for side in (True, False):
        with _engine(monkeypatch, side, 16384) as eng:
            logs = []
            for v in range(8):
                lg = eng.open_log(CausalLogID.main(v))
                for e in range(4):
                    lg.processUpstreamDelta(epochs[(e + v) % 4], 0, e)
                logs.append(lg)
            eng.sync()
            for _ in range(2):
                dec = eng.decode_logs(logs, [0] * 8)
            outs.append({k: np.array(getattr(dec, k)).copy() for k in ("off", "tag", "v0", "w_idx", "w_rc", "w_v1",
                                                                         "w_var_off", "w_var_len", "w_sub")})
            for s, v in enumerate(range(8)):
                assert_span_equal(dec, s, b"".join(epochs[(e + v) % 4] for e in range(4)))
    for k in outs[0]:
        np.testing.assert_array_equal(outs[0][k], outs[1][k], err_msg=k)


@pytest.mark.parametrize("seg", [256, 16384])
@pytest.mark.parametrize("side", [True, False], ids=["sidecar", "scan"])
def test_robust_pipeline_tables_from_the_sidecar(monkeypatch, seg, side):
    """The robust pipeline's table fill (k_jser_fill) takes a deferred tile's table from the
    sidecar when every candidate's length is known, else scans the tile: both bit-exact."""
    rng = np.random.default_rng(seg + side)
    with _engine(monkeypatch, side, seg, decode="robust") as eng:
        logs = [eng.open_log(CausalLogID.main(v)) for v in range(5)]
        blobs = [_mixed(rng, int(rng.integers(300, 1200))) for _ in range(5)]
        _write_host(eng, logs[:3], blobs[:3], rng)
        _write_device(eng, logs[3:], blobs[3:], rng)
        for _ in range(2):
            dec = eng.decode_logs(logs, [0] * 5)
            for s_, b in enumerate(blobs):
                assert_span_equal(dec, s_, b)


_BAD_STREAMS = {
    # a TC_OBJECT whose class descriptor is TC_NULL (the inline flat parser once took it for a
    # 7-byte record)
    "null_class": b"\x03\xac\xed\x00\x05\x73\x70",
    # malformed modified UTF-8 (JDK 8 readUTF: UTFDataFormatException) in a string, in a class
    # name and in a field name of a flat object
    "utf_string": b"\x03\xac\xed\x00\x05\x74\x00\x03a\xc3z",
    "utf_class": D.encode(D.SerializableDeterminant(D.jser_integer(5)))[:9] + b"\xff" +
    D.encode(D.SerializableDeterminant(D.jser_integer(5)))[10:],  # (byte 9: the name's first)
    "utf_field": b"\x03\xac\xed\x00\x05\x73\x72\x00\x01K" + bytes(8) + b"\x02\x00\x01I\x00\x02f\x80\x78\x70" + bytes(4),
}


@pytest.mark.parametrize("kind", sorted(_BAD_STREAMS))
@pytest.mark.parametrize("mode", ["sidecar", "scan", "robust", "host"])
def test_streams_the_jdk_rejects_are_errors(monkeypatch, mode, kind):
    """Serializable records JDK 8's ObjectInputStream fails on (the reference's decodeNext
    throws): every path reports the oracle's error at its offset."""
    rng = np.random.default_rng(17)
    bad = _BAD_STREAMS[kind]
    blob = synth.random_log(200, rng, allow_serializable=False) + _ser(rng) + bad + \
        synth.random_log(30, rng, allow_serializable=False)
    st, _, eo, et = O.decode(blob)
    assert st != 0
    with _engine(monkeypatch, mode != "scan", 16384, decode="robust" if mode == "robust" else "auto") as eng:
        for _ in range(2):  # (the second batch with the table hint set)
            with pytest.raises(_lib.ClonosError) as ex:
                if mode == "host":
                    eng.decode_host(blob)
                else:
                    lg = eng.open_log(CausalLogID.main(int(rng.integers(0, 1 << 30))))
                    lg.appendDeterminant(blob, 0)
                    eng.sync()
                    eng.decode_logs([lg], [0])
            assert (ex.value.status, ex.value.err_off, ex.value.err_tag) == (st, eo, et)


def test_segments_past_64k_carry_no_sidecar(monkeypatch):
    """Segments over 64 KiB hold positions a 16-bit entry cannot name: such an engine keeps no
    lists and scans every tile, bit-exact as with them."""
    rng = np.random.default_rng(131)
    with _engine(monkeypatch, True, 131072, pool=256) as eng:
        logs = [eng.open_log(CausalLogID.main(v)) for v in range(3)]
        blobs = [_mixed(rng, int(rng.integers(2000, 6000))) for _ in range(3)]
        _write_host(eng, logs, blobs, rng)
        for _ in range(2):
            dec = eng.decode_logs(logs, [0, 0, 0])
            for s_, b in enumerate(blobs):
                assert_span_equal(dec, s_, b)
