"""GPU: the one-pass decode (k_decode_one, decode_fused.hip).

A block per tile counts its tile, takes its record base by a decoupled look-back and emits
from the image it holds.  It is off by default (slower than the three passes on MI355X, DESIGN.md
section 4); CLONOS_ONE_PASS=1 (read when an engine opens) turns it on for batches of more than
4 096 tiles without Serializable tables or small whole spans, =2 forces it onto every batch the
three passes would take, so that small cases reach it.  What its rules
do not settle (a record longer than the canonical walk's reach across a tile end, decode
errors, Serializable records) aborts it, and the three passes decode the batch: the result is
the same either way, and every case here is compared record for record with the CPU oracle
(SimpleDeterminantEncoder.decodeNext, :78-342).
"""
import numpy as np
import pytest
import torch

import _oracle as O
from clonos_amd import CausalLogID, ClonosError, Engine, _lib
from clonos_amd import determinants as D
from clonos_amd import synth
from test_gpu_decode import assert_span_equal
from test_gpu_decode_async import DevOut

pytestmark = pytest.mark.gpu


def _count(eng, name):
    return eng.kernel_stats().get(name, {}).get("launches", 0)


@pytest.fixture
def forced(monkeypatch):
    engines = []

    def make(perturb=None, **kw):
        monkeypatch.setenv("CLONOS_ONE_PASS", "2")
        if perturb is not None:
            monkeypatch.setenv("CLONOS_FUSED_PERTURB", str(perturb))
        kw.setdefault("decode", "three_pass")
        e = Engine(timing=True, **kw)
        monkeypatch.delenv("CLONOS_ONE_PASS")
        monkeypatch.delenv("CLONOS_FUSED_PERTURB", raising=False)
        engines.append(e)
        return e

    yield make
    for e in engines:
        e.close()


def _config2_spans(rng, n, lo, hi):
    parts = [synth.config2_log(int(rng.integers(lo, hi)), rng)[0].tobytes() for _ in range(n)]
    blob, spans = b"", []
    for p in parts:
        pad = int(rng.integers(0, 17))
        blob += bytes(pad)
        spans.append((len(blob), len(p)))
        blob += p
    return parts, blob, spans


@pytest.mark.parametrize("seed", range(4))
def test_one_pass_config2_host_input(forced, seed):
    eng = forced()
    rng = np.random.default_rng(200 + seed)
    parts, blob, spans = _config2_spans(rng, 7, 0 if seed == 0 else 1000, 120_000)
    dec = eng.decode_host(blob, spans)
    for s, p in enumerate(parts):
        assert_span_equal(dec, s, p)
    assert _count(eng, "decode_one") >= 1 and _count(eng, "decode_one_abort") == 0


@pytest.mark.parametrize("seg", [256, 16384])
def test_one_pass_logs_in_hbm(forced, seg):
    eng = forced(segment_bytes=seg, pool_segments=(1 << 26) // seg)
    rng = np.random.default_rng(seg)
    logs, blobs = [], []
    for v in range(9):
        b, _ = synth.config2_log(int(rng.integers(2000, 90_000)), rng)
        log = eng.open_log(CausalLogID.main(v))
        log.processUpstreamDelta(b.tobytes(), 0, 0)
        logs.append(log)
        blobs.append(b.tobytes())
    dec = eng.decode_logs(logs, [0] * len(logs))
    for s, b in enumerate(blobs):
        assert_span_equal(dec, s, b)
    if seg >= 16384:
        assert _count(eng, "decode_one") >= 1 and _count(eng, "decode_one_abort") == 0
    else:  # 256-byte tiles: a canonical exit from a few hundred bytes often misses (the three passes)
        assert _count(eng, "decode_one") + _count(eng, "decode_one_abort") >= 1


@pytest.mark.parametrize("seed", range(3))
def test_one_pass_mixed_fixed_and_wide_records(forced, seed):
    """Every tag but Serializable, with long TimerTrigger names now and then: a record longer
    than the canonical walk's reach across a tile end aborts the one pass (the three passes
    repair it), everything else stays on it."""
    eng = forced()
    rng = np.random.default_rng(300 + seed)
    buf = synth.random_log(150_000, rng, allow_serializable=False)
    dec = eng.decode_host(buf)
    assert_span_equal(dec, 0, buf)
    assert _count(eng, "decode_fallback") == 0


def test_one_pass_long_records_abort_to_three_pass(forced):
    eng = forced()
    rng = np.random.default_rng(11)
    recs = []
    for i in range(400):
        if i % 3 == 0:
            recs.append(D.encode(D.TimerTriggerDeterminant(i, i, D.INTERNAL, b"n" * int(rng.integers(3000, 20000)))))
        else:
            recs.append(D.encode(D.OrderDeterminant(1)) * int(rng.integers(1, 400)))
    buf = b"".join(recs)
    dec = eng.decode_host(buf)
    assert_span_equal(dec, 0, buf)
    assert _count(eng, "decode_one_abort") >= 1


def test_one_pass_zero_runs(forced):
    eng = forced()
    for n in (5, 4096, 40_000, 300_001):
        buf = D.encode(D.OrderDeterminant(0)) * n
        dec = eng.decode_host(buf)
        assert dec.n_rec == n
        np.testing.assert_array_equal(dec.off, np.arange(n, dtype=np.uint32) * 2)
    assert _count(eng, "decode_one_abort") == 0


@pytest.mark.parametrize("prefix_n,bad", [(50_000, b"\x08"), (20_000, b"\x01\x00\x00"),
                                          (30_000, b"\x04" + b"\x00" * 12 + b"\x07" + b"\x00")])
def test_one_pass_errors_match_the_oracle(forced, prefix_n, bad):
    eng = forced()
    rng = np.random.default_rng(prefix_n)
    buf = synth.random_log(prefix_n, rng, allow_serializable=False) + bad + synth.random_log(50, rng, False)
    st, _, eo, et = O.decode(buf)
    assert st != 0
    with pytest.raises(ClonosError) as ex:
        eng.decode_host(buf)
    assert ex.value.status == st and ex.value.err_off == eo and ex.value.err_tag == et


def test_one_pass_serializable_goes_to_tables(forced):
    eng = forced()
    rng = np.random.default_rng(7)
    buf = synth.config3_epoch(30_000, rng)[0].tobytes()
    dec = eng.decode_host(buf)
    assert_span_equal(dec, 0, buf)


@pytest.mark.parametrize("perturb,stat", [(2, "decode_one_abort"), (1 << 16, "decode_lookback_check")])
def test_one_pass_handoffs_checked(forced, perturb, stat):
    """A wrong entry (+2 in a run of channel-0 Order records: a valid chain that drops one
    record per tile) or a wrong look-back result is found when the tile reads the words it took
    again, and the batch is decoded by the three passes (where the same fault is repaired)."""
    eng = forced(perturb=perturb)
    buf = bytes(3 << 20) if perturb == 2 else synth.config2_log(500_000, np.random.default_rng(1))[0].tobytes()
    dec = eng.decode_host(buf)
    assert_span_equal(dec, 0, buf)
    assert _count(eng, stat) >= 1


def test_one_pass_on_large_batches(monkeypatch):
    """CLONOS_ONE_PASS=1: a batch of more than 4 096 tiles (33.5 MB) takes the one pass."""
    rng = np.random.default_rng(9)
    monkeypatch.setenv("CLONOS_ONE_PASS", "1")
    with Engine(timing=True) as eng:
        parts, blob, spans = _config2_spans(rng, 5, 1_200_000, 1_500_000)
        assert len(blob) > 4096 * 8192
        dec = eng.decode_host(blob, spans)
        for s, p in enumerate(parts):
            assert_span_equal(dec, s, p)
        assert _count(eng, "decode_one") >= 1 and _count(eng, "decode_count") == 0


def test_one_pass_two_in_flight_device_outputs(forced):
    """The bench's pipelined step on the one pass: two decodes queued into device outputs,
    slices gathered on the second stream between them, each compared with the oracle."""
    eng = forced(segment_bytes=16384, pool_segments=1 << 13, async_slice=True)
    rng = np.random.default_rng(41)
    blobs = [synth.config2_log(int(rng.integers(20_000, 80_000)), rng)[0] for _ in range(8)]
    logs = []
    for v, b in enumerate(blobs):
        lg = eng.open_log(CausalLogID.main(v))
        lg.processUpstreamDelta(b.tobytes(), 0, 1)
        logs.append(lg)
    n, total = len(logs), sum(int(b.size) for b in blobs)
    ref = eng.decode_logs(logs, [1] * n)
    for s, b in enumerate(blobs):
        assert_span_equal(ref, s, b.tobytes())
    sets = [DevOut(total // 2 + n + 1, total // 6 + n + 1) for _ in range(2)]
    h = np.array([lg.handle for lg in logs], np.uint32)
    creq = (_lib.SliceReq * n)()
    cres = (_lib.SliceRes * n)()
    for i, lg in enumerate(logs):
        creq[i].log, creq[i].consumer, creq[i].epoch = lg.handle, _lib.ChannelId(7, i), 1
    sl = torch.empty(total + 64, dtype=torch.uint8, device="cuda")
    queued = []
    for k in range(6):
        so = sets[k % 2]
        if len(queued) == 2:
            eng.decode_wait()
            queued.pop(0).check(ref)
        so.base = np.zeros(n + 1, np.uint64)
        eng.decode_logs_device_async(h, np.ones(n, np.int64), so.dec, so.base)
        queued.append(so)
        eng.seek_consumers_raw(creq, np.zeros(n, np.int32), n)
        assert eng.slice_batch_raw(creq, cres, n, sl.data_ptr(), sl.numel(), device=True) == total
    while queued:
        eng.decode_wait()
        queued.pop(0).check(ref)
    assert _count(eng, "decode_one") >= 1 and _count(eng, "decode_one_abort") == 0
