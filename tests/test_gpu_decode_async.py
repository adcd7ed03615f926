"""GPU: the asynchronous batched decode (clg_decode_logs_async + clg_decode_wait) gives the
synchronous decode's results bit for bit -- and so the oracle's -- whether it is waited for
directly, left pending across device slices on the gather stream and consumer seeks, or
completed implicitly by a call that needs the engine exclusively; errors and the fallback
paths (Serializable tables, robust pipeline) surface at the wait."""
import numpy as np
import pytest
import torch

import _oracle as O
from clonos_amd import ClonosError, CausalLogID, Engine, _lib
from clonos_amd import synth

pytestmark = pytest.mark.gpu


def logs_of(eng, blobs):
    logs = []
    for v, b in enumerate(blobs):
        lg = eng.open_log(CausalLogID.main(v))
        lg.processUpstreamDelta(bytes(b), 0, 1)
        logs.append(lg)
    return logs


def same(a, b):
    for f in ("off", "tag", "v0", "w_idx", "w_rc", "w_v1", "w_var_off", "w_var_len", "w_sub", "span_rec_base"):
        np.testing.assert_array_equal(getattr(a, f), getattr(b, f), err_msg=f)


def check_oracle(dec, blobs):
    for s, b in enumerate(blobs):
        st, r, _, _ = O.decode(bytes(b))
        assert st == 0
        sl = dec.span_slice(s)
        np.testing.assert_array_equal(dec.tag[sl], r["tag"])
        np.testing.assert_array_equal(dec.v0[sl], r["v0"])
        np.testing.assert_array_equal(dec.off[sl], r["off"])


@pytest.mark.parametrize("decode", ["auto", "robust"])
@pytest.mark.parametrize("seed", [0, 1])
def test_async_equals_sync(decode, seed):
    rng = np.random.default_rng(seed)
    blobs = [synth.random_log(int(rng.integers(0, 3000)), rng) for _ in range(12)]
    with Engine(segment_bytes=1024, pool_segments=1 << 14, decode=decode) as eng:
        logs = logs_of(eng, blobs)
        ref = eng.decode_logs(logs, [1] * len(logs))
        got = eng.decode_logs_async(logs, [1] * len(logs)).wait()
        same(got, ref)
        check_oracle(got, blobs)


def test_async_pending_across_device_slices_and_seeks():
    """The bench's step: decode queued, consumers rewound, slices gathered into device
    memory on the second stream while the decode runs, then the wait."""
    rng = np.random.default_rng(5)
    blobs = [synth.config2_log(20000, rng)[0] for _ in range(6)]
    with Engine(segment_bytes=16384, pool_segments=1 << 12, async_slice=True) as eng:
        logs = logs_of(eng, blobs)
        n_req = len(logs)
        creq = (_lib.SliceReq * n_req)()
        cres = (_lib.SliceRes * n_req)()
        for i, lg in enumerate(logs):
            creq[i].log, creq[i].consumer, creq[i].epoch = lg.handle, _lib.ChannelId(3, i), 1
        total = sum(int(b.size) for b in blobs)
        out = torch.empty(total + 64, dtype=torch.uint8, device="cuda")
        ref = eng.decode_logs(logs, [1] * n_req)
        for _ in range(3):
            pd = eng.decode_logs_async(logs, [1] * n_req)
            eng.seek_consumers_raw(creq, np.zeros(n_req, np.int32), n_req)
            got_bytes = eng.slice_batch_raw(creq, cres, n_req, out.data_ptr(), out.numel(), device=True)
            got = pd.wait()
            assert got_bytes == total
            same(got, ref)
            eng.sync()
            assert out[:total].cpu().numpy().tobytes() == b"".join(bytes(b) for b in blobs)


def test_async_settled_by_exclusive_call():
    """An append flush / log open in between completes the pending decode first; the wait
    then returns its result, and the decode saw the logs as they were when it was queued."""
    rng = np.random.default_rng(9)
    blobs = [synth.random_log(2000, rng) for _ in range(4)]
    with Engine(segment_bytes=512, pool_segments=1 << 13) as eng:
        logs = logs_of(eng, blobs)
        ref = eng.decode_logs(logs, [1] * len(logs))
        pd = eng.decode_logs_async(logs, [1] * len(logs))
        eng.open_log(CausalLogID.main(99))           # exclusive: settles the decode
        logs[0].appendDeterminant(bytes([0, 1]), 2)  # staged; flushed by the next exclusive call
        eng.sync()
        same(pd.wait(), ref)
        assert logs[0].getDeterminants(1)[-2:] == bytes([0, 1])


def test_async_error_at_wait():
    rng = np.random.default_rng(3)
    good = synth.random_log(500, rng, allow_serializable=False)
    bad = bytes(good) + bytes([0x7F, 1, 2, 3])  # corrupt tag after the good records
    with Engine(segment_bytes=256, pool_segments=1 << 12) as eng:
        logs = logs_of(eng, [good, bad])
        with pytest.raises(ClonosError) as sync_err:
            eng.decode_logs(logs, [1, 1])
        pd = eng.decode_logs_async(logs, [1, 1])
        eng.sync()  # settles: the error is kept for the wait
        with pytest.raises(ClonosError) as async_err:
            pd.wait()
        a, b = sync_err.value, async_err.value
        assert (a.status, a.err_span, a.err_off, a.err_tag) == (b.status, b.err_span, b.err_off, b.err_tag)
        assert b.status == _lib.CLG_E_CORRUPT_TAG and b.err_span == 1 and b.err_off == len(good)
        # the next wait has nothing pending
        eng.decode_wait()


def test_async_serializable_retry_and_hint():
    """A batch with Serializable records on a fresh engine (no table hint yet): the async
    decode aborts, and the wait re-runs it with the tables."""
    rng = np.random.default_rng(11)
    e3, offs = synth.config3_epoch(4000, rng, 0)
    blobs = [e3, e3[:int(offs[len(offs) // 2])]]  # the second cut at a record boundary
    with Engine(segment_bytes=16384, pool_segments=1 << 10, timing=True) as eng:
        logs = logs_of(eng, blobs)
        got = eng.decode_logs_async(logs, [1, 1]).wait()
        ref = eng.decode_logs(logs, [1, 1])
        same(got, ref)
        st, r, _, _ = O.decode(bytes(e3))
        assert st == 0 and got.span_rec_base[1] == len(r["tag"])
        assert eng.kernel_stats().get("decode_jser_retry", {}).get("launches", 0) >= 1


def test_repeated_shapes_new_bytes_no_timing():
    """A non-timing engine decoding the same batch shape again with other bytes (timestamps
    rewritten in place), a new shape, then the first shape again, sync and async: every
    result equals the oracle's (the reused plan, control and output buffers carry nothing
    over)."""
    rng = np.random.default_rng(21)
    shapes = {k: [synth.config2_log(n, rng) for _ in range(m)] for k, (m, n) in {"a": (4, 3000), "b": (7, 1000)}.items()}

    def fresh_values(blobs):
        out = []
        for b, offs in blobs:
            b = b.copy()
            for o in offs[b[offs] == 1]:  # Timestamp records: new 8-byte payloads
                b[o + 1:o + 9] = rng.integers(0, 256, 8, dtype=np.uint8)
            out.append((b, offs))
        return out

    with Engine(segment_bytes=4096, pool_segments=1 << 12, timing=False) as eng:
        for k in ("a", "a", "b", "a"):
            blobs = shapes[k] = fresh_values(shapes[k])
            logs = [eng.open_log(CausalLogID.main(1000 + j)) for j in range(len(blobs))]
            for lg, (b, _) in zip(logs, blobs):
                lg.processUpstreamDelta(b.tobytes(), 0, 1)
            for dec in (eng.decode_logs(logs, [1] * len(logs)), eng.decode_logs_async(logs, [1] * len(logs)).wait()):
                check_oracle(dec, [b for b, _ in blobs])
            for lg in logs:
                lg.close()


def test_third_async_before_wait_is_refused():
    """Decodes queued back to back, the first failing: up to CLG_DECODE_MAX_INFLIGHT are
    accepted, the next is refused (CLG_E_STATE) instead of dropping a status, and the waits
    return each decode's own status in queue order."""
    rng = np.random.default_rng(4)
    good = synth.random_log(500, rng, allow_serializable=False)
    bad = bytes(good) + bytes([0x7F, 1, 2, 3])
    assert _lib.CLG_DECODE_MAX_INFLIGHT == 2
    with Engine(segment_bytes=256, pool_segments=1 << 12) as eng:
        logs = logs_of(eng, [good, bad])
        pd = eng.decode_logs_async(logs, [1, 1])
        pd2 = eng.decode_logs_async(logs[:1], [1])
        with pytest.raises(ClonosError) as third:
            eng.decode_logs_async(logs[:1], [1])
        assert third.value.status == _lib.CLG_E_STATE
        with pytest.raises(ClonosError) as first:
            pd.wait()
        assert first.value.status == _lib.CLG_E_CORRUPT_TAG and first.value.err_span == 1
        assert pd2.wait().n_rec == len(O.decode(good)[1]["tag"])
        got = eng.decode_logs_async(logs[:1], [1]).wait()  # waited for: the next one is accepted
        assert got.n_rec == len(O.decode(good)[1]["tag"])


def test_later_wait_completes_earlier_host_decodes():
    """Waiting for the second of two queued decodes first: the first is completed on the way
    and keeps its own result (and error) for its own wait."""
    rng = np.random.default_rng(14)
    a = [synth.random_log(int(rng.integers(100, 2000)), rng, allow_serializable=False) for _ in range(5)]
    bad = bytes(a[0]) + bytes([0x7F, 1])
    with Engine(segment_bytes=512, pool_segments=1 << 13) as eng:
        logs = logs_of(eng, a + [bad])
        p1 = eng.decode_logs_async(logs[5:], [1])
        p2 = eng.decode_logs_async(logs[:5], [1] * 5)
        check_oracle(p2.wait(), a)
        with pytest.raises(ClonosError) as e1:
            p1.wait()
        assert e1.value.status == _lib.CLG_E_CORRUPT_TAG and e1.value.err_off == len(a[0])


class DevOut:
    """Caller-owned device output arrays (the bench's layout) and their clg_decoded."""

    def __init__(self, cap, wcap):
        self.t = [torch.empty(cap, dtype=torch.int32, device="cuda"), torch.empty(cap, dtype=torch.uint8, device="cuda"),
                  torch.empty(cap, dtype=torch.int64, device="cuda")]
        self.w = [torch.empty(wcap, dtype=t, device="cuda") for t in
                  (torch.int32, torch.int32, torch.int64, torch.int32, torch.int32, torch.uint8)]
        d = self.dec = _lib.Decoded()
        d.off, d.tag, d.v0 = [x.data_ptr() for x in self.t]
        d.w_idx, d.w_rc, d.w_v1, d.w_var_off, d.w_var_len, d.w_sub = [x.data_ptr() for x in self.w]
        d.cap, d.wcap, d.out_kind = cap, wcap, _lib.CLG_MEM_DEVICE
        self.base = None

    def check(self, ref):
        torch.cuda.synchronize()
        n, nw = int(self.dec.n_rec), int(self.dec.n_wide)
        assert n == len(ref.tag) and nw == len(ref.w_idx)
        np.testing.assert_array_equal(self.t[0][:n].cpu().numpy(), ref.off)
        np.testing.assert_array_equal(self.t[1][:n].cpu().numpy(), ref.tag)
        np.testing.assert_array_equal(self.t[2][:n].cpu().numpy(), ref.v0)
        for x, f in zip(self.w, ("w_idx", "w_rc", "w_v1", "w_var_off", "w_var_len", "w_sub")):
            np.testing.assert_array_equal(x[:nw].cpu().numpy(), getattr(ref, f), err_msg=f)
        np.testing.assert_array_equal(self.base, ref.span_rec_base)


@pytest.mark.parametrize("mix", ["config2", "config3"])
def test_two_in_flight_device_outputs(mix):
    """The pipelined bench step: decode i+1 queued (with its own device outputs) before
    decode i is waited for, slices gathered on the second stream in between; every decode
    equals the synchronous one (and the oracle), including a batch whose first fast run
    aborts for want of Serializable tables while the next one is already queued (both are
    decoded again: the redo path)."""
    rng = np.random.default_rng(31)
    if mix == "config2":
        blobs = [synth.config2_log(int(rng.integers(5000, 40000)), rng)[0] for _ in range(9)]
    else:
        blobs = [synth.config3_epoch(int(rng.integers(2000, 6000)), rng, 0)[0] for _ in range(5)]
    with Engine(segment_bytes=16384, pool_segments=1 << 12, async_slice=True, timing=True) as eng:
        logs = logs_of(eng, blobs)
        n = len(logs)
        total = sum(int(b.size) for b in blobs)
        sets = [DevOut(total // 2 + n + 1, total // 6 + n + 1) for _ in range(2)]
        h = np.array([lg.handle for lg in logs], np.uint32)
        groups = [h, h[::-1].copy(), h[: n // 2 + 1].copy()]  # batches of other shapes and orders
        creq = (_lib.SliceReq * n)()
        cres = (_lib.SliceRes * n)()
        for i, lg in enumerate(logs):
            creq[i].log, creq[i].consumer, creq[i].epoch = lg.handle, _lib.ChannelId(7, i), 1
        sl = torch.empty(total + 64, dtype=torch.uint8, device="cuda")
        refs = [eng.decode_logs([logs[int(np.nonzero(h == x)[0][0])] for x in g], [1] * len(g)) for g in groups]
        if mix == "config3":  # a fresh engine state for the abort: the table hint off again
            eng.close()
            eng = Engine(segment_bytes=16384, pool_segments=1 << 12, async_slice=True, timing=True)
            logs = logs_of(eng, blobs)
            h2 = np.array([lg.handle for lg in logs], np.uint32)
            groups = [h2[[int(np.nonzero(h == x)[0][0]) for x in g]] for g in groups]
            for i, lg in enumerate(logs):
                creq[i].log = lg.handle
        queued = []
        for k in range(7):
            g = groups[k % 3]
            so = sets[k % 2]
            if len(queued) == 2:
                j, o = queued.pop(0)
                eng.decode_wait()
                o.check(refs[j % 3])
            so.base = np.zeros(len(g) + 1, np.uint64)
            eng.decode_logs_device_async(g, np.ones(len(g), np.int64), so.dec, so.base)
            queued.append((k, so))
            eng.seek_consumers_raw(creq, np.zeros(n, np.int32), n)
            assert eng.slice_batch_raw(creq, cres, n, sl.data_ptr(), sl.numel(), device=True) == total
        while queued:
            j, o = queued.pop(0)
            eng.decode_wait()
            o.check(refs[j % 3])
        eng.sync()
        assert sl[:total].cpu().numpy().tobytes() == b"".join(bytes(b) for b in blobs)
        if mix == "config3":
            assert eng.kernel_stats().get("decode_async_redo", {}).get("launches", 0) >= 1
        eng.close()


@pytest.mark.parametrize("kind", ["config2", "config3"])
def test_truncate_beside_queued_decode(kind):
    """clg_truncate_all while an asynchronous decode from the checkpoint epoch is queued (config
    4's step): the decode's records equal the oracle's decode of the epochs it asked for, the
    segments the truncation freed go back to the pool only once the decode is waited for, and a
    fast run that aborts (config 3: the Serializable tables first) re-plans over the rebased
    logs.  A truncation above a queued decode's start epoch completes that decode first."""
    rng = np.random.default_rng(11)
    if kind == "config2":
        gen = lambda n: synth.config2_log(n, rng)[0]  # noqa: E731
    else:
        gen = lambda n: synth.config3_epoch(n, rng)[0]  # noqa: E731
    n_logs, n_ep = 6, 4
    with Engine(segment_bytes=1024, pool_segments=1 << 14) as eng:
        logs = [eng.open_log(CausalLogID.main(v)) for v in range(n_logs)]
        parts = [[] for _ in range(n_logs)]
        for ep in range(n_ep):
            for v, lg in enumerate(logs):
                b = bytes(gen(int(rng.integers(200, 3000))))
                lg.processUpstreamDelta(b, 0, ep)
                parts[v].append(b)
        used0, _ = eng.pool_stats()
        pd = eng.decode_logs_async(logs, [2] * n_logs)
        assert eng.truncate_all(2)
        got = pd.wait()
        check_oracle(got, [b"".join(p[2:]) for p in parts])
        used1, _ = eng.pool_stats()
        assert used1 < used0
        same(eng.decode_logs(logs, [2] * n_logs), got)
        pd = eng.decode_logs_async(logs, [2] * n_logs)
        assert eng.truncate_all(3)  # above the queued decode's start: it completes first
        same(pd.wait(), got)
        check_oracle(eng.decode_logs(logs, [3] * n_logs), [b"".join(p[3:]) for p in parts])
