"""GPU: the engine's ThreadCausalLog (HBM segments + host metadata) == the oracle's
ThreadCausalLogImpl model, op by op, bytes and state.  Also the batched slice path."""
import numpy as np
import pytest

import _oracle as O
from clonos_amd import ClonosError, CausalLogID, Engine
from clonos_amd import determinants as D
from clonos_amd import synth

pytestmark = pytest.mark.gpu


def status_of(fn, *a):
    try:
        return 0, fn(*a)
    except ClonosError as e:
        return e.status, None


@pytest.mark.parametrize("tail", [0, 100, 16384])  # host tail: none (every slice gathers), short, default
@pytest.mark.parametrize("seed,comp", [(0, 16), (1, 32), (2, 64), (3, 256), (4, 16384)])
def test_log_ops_match_oracle(seed, comp, tail):
    rng = np.random.default_rng(1000 + seed)
    with Engine(segment_bytes=comp, pool_segments=1 << 14, host_tail_bytes=tail) as eng:
        log = eng.open_log(CausalLogID.main(1))
        ref = O.OracleLog(comp)
        epoch, last_cp = 0, 0
        chans = [(1, 9), (2, 9), (3, 9), (4, 9)]
        for step in range(1500):
            op = int(rng.integers(0, 12))
            if op <= 4:
                rec = D.encode(synth.random_determinant(rng))
                log.appendDeterminant(rec, epoch)
                assert ref.append(epoch, rec) == 0
            elif op == 5:
                # upstream delta overlapping what we have (dedup) or extending it
                cur = ref.state()
                rec = b"".join(D.encode(synth.random_determinant(rng)) for _ in range(int(rng.integers(1, 6))))
                back = int(rng.integers(0, 3))
                have = ref.get_determinants(epoch)[1] if epoch in dict(cur["epochs"]) else b""
                delta = have[len(have) - min(back * 2, len(have)):] + rec if back else rec
                off = len(have) - (len(delta) - len(rec))
                if rng.integers(0, 6) == 0:
                    # a gap: components are added before the reader index throws (:136-143)
                    off += int(rng.integers(1, 40))
                st1, _ = status_of(log.processUpstreamDelta, delta, off, epoch)
                assert st1 == ref.upstream(delta, off, epoch)
            elif op == 6:
                ch = chans[int(rng.integers(0, len(chans)))]
                e = epoch - int(rng.integers(0, 2))
                st1, v1 = status_of(log.hasDeltaForConsumer, ch, e)
                st2, v2 = ref.has_delta(ch, e)
                assert (st1, bool(v1) if st1 == 0 else False) == (st2, v2 if st2 == 0 else False)
                if st1 == 0 and v1:
                    assert log.getOffsetFromEpochForConsumer(ch, e) == ref.offset(ch)[1]
                    st1, d1 = status_of(log.getDeltaForConsumer, ch, e)
                    st2, d2 = ref.get_delta(ch, e)
                    assert st1 == st2 and (st1 != 0 or d1 == d2)
            elif op == 7:
                epoch += 1
            elif op == 8 and epoch - 1 > last_cp:
                cp = epoch - int(rng.integers(0, 2))
                last_cp = cp
                st1, _ = status_of(log.notifyCheckpointComplete, cp)
                assert st1 == ref.checkpoint_complete(cp)
            elif op == 9:
                e = epoch - int(rng.integers(0, 3))
                st1, d1 = status_of(log.getDeterminants, e)
                st2, d2 = ref.get_determinants(e)
                assert st1 == st2 and (st1 != 0 or d1 == d2)
            elif op == 10:
                assert log.logLength() == ref.log_length()
            else:
                ch = chans[int(rng.integers(0, len(chans)))]
                log.unregisterConsumer(ch)
                ref.unregister(ch)
            s1, s2 = log.state(), ref.state()
            assert s1 == s2, (step, s1, s2)
            for ch in chans:
                assert log.consumer_state(ch) == ref.consumer(ch)
        # physical bytes identical
        s = ref.state()
        if s["writer"]:
            assert log.read_phys(0, s["writer"]) == ref.read_phys(0, s["writer"])[1]


def test_nettytests_delta_over_components():
    """NettyTests.CompositeFromCompositeComponentsTest (:144-186) with 16-byte components:
    a delta straddling three components; truncation drops whole components only."""
    with Engine(segment_bytes=16, pool_segments=64) as eng:
        log = eng.open_log(CausalLogID.main(0))
        for _ in range(5):
            log.appendDeterminant(b"Hello world, hi!", 0)  # exactly one component each
        ch = (7, 7)
        assert log.hasDeltaForConsumer(ch, 0)
        log.seek_consumer(ch, 0, 5)
        assert log.getDeltaForConsumer(ch, 0) == (b"Hello world, hi!" * 5)[5:]
        log.appendDeterminant(b"X" * 12, 1)  # epoch 1 starts at physical 80
        log.notifyCheckpointComplete(1)
        st = log.state()
        assert st["capacity"] == 16 and st["n_components"] == 1 and st["epochs"] == [(1, 0)]


def test_slice_batch_matches_sequential():
    rng = np.random.default_rng(77)
    with Engine(segment_bytes=512, pool_segments=1 << 14) as eng:
        logs = [eng.open_log(CausalLogID.sub(v, 11, 22, v % 3)) for v in range(16)]
        refs = [O.OracleLog(512) for _ in logs]
        for ep in range(3):
            for log, ref in zip(logs, refs):
                for _ in range(int(rng.integers(0, 300))):
                    rec = D.encode(synth.random_determinant(rng))
                    log.appendDeterminant(rec, ep)
                    ref.append(ep, rec)
            reqs, expect = [], []
            for i, (log, ref) in enumerate(zip(logs, refs)):
                for c in range(4):
                    ch = (c, i)
                    reqs.append((log, ch, ep))
                    st, has = ref.has_delta(ch, ep)
                    if has:
                        off = ref.offset(ch)[1]
                        d = ref.get_delta(ch, ep)[1]
                        expect.append((True, off, d))
                    else:
                        expect.append((False, 0, b""))
            res, out, total = eng.slice_batch(reqs)
            for (st, has, off, n, oo), (h2, off2, d2) in zip(res, expect):
                assert st == 0 and has == h2
                if has:
                    assert off == off2 and out[oo:oo + n].tobytes() == d2


def test_consumer_went_backwards():
    with Engine(segment_bytes=64, pool_segments=64) as eng:
        log = eng.open_log(CausalLogID.main(0))
        log.appendDeterminant(D.OrderDeterminant(1), 0)
        log.appendDeterminant(D.OrderDeterminant(2), 1)
        assert log.hasDeltaForConsumer(1, 1)
        with pytest.raises(ClonosError) as ex:
            log.hasDeltaForConsumer(1, 0)
        assert ex.value.status == -7


def test_truncate_all_cas_and_pool_reuse():
    with Engine(segment_bytes=64, pool_segments=256) as eng:
        logs = [eng.open_log(CausalLogID.main(v)) for v in range(8)]
        for ep in range(1, 6):
            for log in logs:
                for _ in range(40):
                    log.appendDeterminant(D.TimestampDeterminant(ep), ep)
        used0, _ = eng.pool_stats()
        assert eng.truncate_all(4)
        assert not eng.truncate_all(3)  # CAS: older checkpoint ignored (JobCausalLogImpl :234-235)
        used1, _ = eng.pool_stats()
        assert used1 < used0
        for log in logs:
            assert log.state()["epochs"][0][0] == 4
            assert log.getDeterminants(4) == D.encode(D.TimestampDeterminant(4)) * 40 + D.encode(D.TimestampDeterminant(5)) * 40


@pytest.mark.parametrize("seg,shuffle", [(16, False), (512, False), (16384, False), (65536, False), (512, True),
                                         (16384, True)])
def test_seek_batch_then_slice(seg, shuffle):
    """clg_consumer_seek_batch positions consumers exactly like clg_consumer_seek; the
    batched slice (one gather block per segment of a log, serving all of that log's
    requests) returns each consumer's suffix, packed in request order also when the requests
    of a log are scattered through the batch (shuffle)."""
    from clonos_amd import _lib
    rng = np.random.default_rng(seg + 3 + shuffle)
    with Engine(segment_bytes=seg, pool_segments=(1 << 21) // seg + 64) as eng:
        logs, bufs = [], []
        for v in range(6):
            log = eng.open_log(CausalLogID.main(v))
            b, _ = synth.config2_log(int(rng.integers(10, 30000)), rng)
            log.processUpstreamDelta(b.tobytes(), 0, 4)
            logs.append(log)
            bufs.append(b.tobytes())
        reqs = []
        for i in range(len(logs)):
            for c in range(5):
                reqs.append((i, (c + 1, i), int(rng.integers(0, len(bufs[i]) + 1))))
        if shuffle:
            reqs = [reqs[j] for j in rng.permutation(len(reqs))]
        creq = (_lib.SliceReq * len(reqs))()
        cres = (_lib.SliceRes * len(reqs))()
        for k, (i, ch, _) in enumerate(reqs):
            creq[k].log = logs[i].handle
            creq[k].consumer = _lib.ChannelId(*ch)
            creq[k].epoch = 4
        eng.seek_consumers_raw(creq, np.array([o for _, _, o in reqs], np.int32), len(reqs))
        for i, ch, off in reqs:
            assert logs[i].consumer_state(ch)[1] == off
        total = sum(len(bufs[i]) - off for i, _, off in reqs)
        out = np.zeros(total + 16, np.uint8)
        got = eng.slice_batch_raw(creq, cres, len(reqs), out.ctypes.data, out.size, device=False)
        assert got == total
        for k, (i, ch, off) in enumerate(reqs):
            r = cres[k]
            assert r.status == 0
            exp = bufs[i][off:]
            assert r.len == len(exp) and out[r.out_off:r.out_off + r.len].tobytes() == exp


@pytest.mark.parametrize("seg", [512, 1024, 16384])
def test_async_slice_many_consumers_per_log(seg):
    """The asynchronous device-output slice of config 2's shape -- eight consumers of each log
    at random offsets, requests shuffled, the call repeated (descriptor sets reused): each
    request's bytes equal its suffix of the log."""
    import ctypes
    from clonos_amd import _lib
    hip = ctypes.CDLL("libamdhip64.so.7")
    rng = np.random.default_rng(seg)
    with Engine(segment_bytes=seg, pool_segments=(1 << 22) // seg + 64, async_slice=True) as eng:
        logs, bufs = [], []
        for v in range(7):
            log = eng.open_log(CausalLogID.main(v))
            b, _ = synth.config2_log(int(rng.integers(10, 40000)), rng)
            log.processUpstreamDelta(b.tobytes(), 0, 2)
            logs.append(log)
            bufs.append(b.tobytes())
        reqs = [(i, (c + 1, i), int(rng.integers(0, len(bufs[i]) + 1))) for i in range(len(logs)) for c in range(8)]
        reqs = [reqs[j] for j in rng.permutation(len(reqs))]
        creq = (_lib.SliceReq * len(reqs))()
        cres = (_lib.SliceRes * len(reqs))()
        for k, (i, ch, _) in enumerate(reqs):
            creq[k].log = logs[i].handle
            creq[k].consumer = _lib.ChannelId(*ch)
            creq[k].epoch = 2
        total = sum(len(bufs[i]) - off for i, _, off in reqs)
        dptr = ctypes.c_void_p()
        assert hip.hipMalloc(ctypes.byref(dptr), ctypes.c_size_t(total + 64)) == 0
        try:
            for _ in range(2):  # twice: the second call reuses the descriptor sets
                eng.seek_consumers_raw(creq, np.array([o for _, _, o in reqs], np.int32), len(reqs))
                got = eng.slice_batch_raw(creq, cres, len(reqs), dptr.value, total + 64, device=True)
                assert got == total
                eng.sync()
                host = np.empty(total + 1, np.uint8)
                assert hip.hipMemcpy(ctypes.c_void_p(host.ctypes.data), dptr, ctypes.c_size_t(total), 2) == 0
                for k, (i, ch, off) in enumerate(reqs):
                    r = cres[k]
                    assert r.status == 0 and r.len == len(bufs[i]) - off
                    assert host[r.out_off:r.out_off + r.len].tobytes() == bufs[i][off:]
        finally:
            hip.hipFree(dptr)


def test_capacity_reports_required_size():
    """clg_get_delta / clg_get_determinants with a short buffer: CLG_E_CAPACITY, *n = the
    size needed, consumer not advanced (the JNI layer sizes its direct buffer this way)."""
    import ctypes as C
    from clonos_amd._lib import lib
    with Engine(segment_bytes=64, pool_segments=256) as eng:
        log = eng.open_log(CausalLogID.main(3))
        for i in range(40):
            log.appendDeterminant(D.TimestampDeterminant(i), 0)
        ch = (5, 6)
        assert log.hasDeltaForConsumer(ch, 0)
        n = C.c_uint32()
        st = lib.clg_get_delta(eng.handle, log.handle, _lib_ch(ch), 0, None, 0, 0, C.byref(n))
        assert st == -11 and n.value == 40 * 9
        assert log.consumer_state(ch) == (0, 0)
        st = lib.clg_get_determinants(eng.handle, log.handle, 0, None, 10, 0, C.byref(n))
        assert st == -11 and n.value == 40 * 9
        assert log.getDeltaForConsumer(ch, 0) == D.encode(D.TimestampDeterminant(0))[:0] + b"".join(
            D.encode(D.TimestampDeterminant(i)) for i in range(40))


def _lib_ch(ch):
    from clonos_amd import _lib
    return _lib.ChannelId(*ch)


def test_async_slice_overlaps_and_orders():
    """CLG_F_ASYNC_SLICE: device-output gathers queue on the gather stream; appends after
    them wait (the scatter must not overwrite segments a gather still reads), decodes run
    beside them, and sync() makes the output visible.  Bytes == the oracle's deltas.
    Device memory comes from the engine's own HIP runtime (ctypes), not torch's bundled one."""
    import ctypes
    hip = ctypes.CDLL("libamdhip64.so.7")
    rng = np.random.default_rng(91)
    with Engine(segment_bytes=1024, pool_segments=1 << 14, async_slice=True) as eng:
        logs = [eng.open_log(CausalLogID.main(v)) for v in range(8)]
        refs = [O.OracleLog(1024) for _ in logs]
        cap = 1 << 22
        dptr = ctypes.c_void_p()
        assert hip.hipMalloc(ctypes.byref(dptr), ctypes.c_size_t(cap)) == 0
        try:
            for rnd in range(4):
                for log, ref in zip(logs, refs):
                    b = synth.random_log(int(rng.integers(50, 2000)), rng, allow_serializable=False)
                    log.appendDeterminant(b, 0)
                    ref.append(0, b)
                reqs, want = [], []
                for i, (log, ref) in enumerate(zip(logs, refs)):
                    ch = (rnd % 2, i)
                    reqs.append((log, ch, 0))
                    st, has = ref.has_delta(ch, 0)
                    want.append(ref.get_delta(ch, 0)[1] if has else b"")
                res, _, total = eng.slice_batch(reqs, out=dptr.value, cap=cap)
                dec = eng.decode_logs(logs, [0] * len(logs))  # runs beside the gather
                assert dec.n_rec > 0
                eng.sync()
                host = np.empty(max(1, total), np.uint8)
                assert hip.hipMemcpy(ctypes.c_void_p(host.ctypes.data), dptr, ctypes.c_size_t(total), 2) == 0
                host = host[:total].tobytes()
                for (st, has, ofe, n, oo), w in zip(res, want):
                    assert st == 0 and host[oo:oo + n] == w
        finally:
            hip.hipFree(dptr)


def test_async_decode_device_output():
    """Decode into device memory on an engine with CLG_F_ASYNC_SLICE (the decode itself stays
    synchronous): counts final on return, SoA equal to the oracle's decode."""
    import ctypes
    from clonos_amd import _lib
    hip = ctypes.CDLL("libamdhip64.so.7")
    rng = np.random.default_rng(92)
    with Engine(segment_bytes=16384, pool_segments=1 << 12, async_slice=True) as eng:
        bufs = [synth.config2_log(int(rng.integers(1000, 200_000)), rng)[0].tobytes() for _ in range(6)]
        logs = []
        for v, b in enumerate(bufs):
            lg = eng.open_log(CausalLogID.main(v))
            lg.appendDeterminant(b, 0)
            logs.append(lg)
        cap = sum(len(b) for b in bufs) // 2 + 8
        sizes = dict(off=4 * cap, tag=cap, v0=8 * cap, w_idx=64, w_rc=64, w_v1=64, w_var_off=64, w_var_len=64, w_sub=64)
        ptrs = {}
        for k, n in sizes.items():
            p = ctypes.c_void_p()
            assert hip.hipMalloc(ctypes.byref(p), ctypes.c_size_t(n)) == 0
            ptrs[k] = p
        try:
            dec = _lib.Decoded()
            for k, p in ptrs.items():
                setattr(dec, k, p.value)
            dec.cap, dec.wcap, dec.out_kind = cap, 8, _lib.CLG_MEM_DEVICE
            base = np.zeros(len(logs) + 1, np.uint64)
            eng.decode_logs_device(np.array([l.handle for l in logs], np.uint32), np.zeros(len(logs), np.int64), dec,
                                   base)
            want = [O.decode(b)[1] for b in bufs]
            assert dec.n_rec == sum(len(w["tag"]) for w in want)
            eng.sync()
            got = {}
            for k, dt in (("off", np.uint32), ("tag", np.uint8), ("v0", np.int64)):
                a = np.empty(dec.n_rec, dt)
                assert hip.hipMemcpy(ctypes.c_void_p(a.ctypes.data), ptrs[k], ctypes.c_size_t(a.nbytes), 2) == 0
                got[k] = a
            for s, w in enumerate(want):
                sl = slice(int(base[s]), int(base[s + 1]))
                for k in ("off", "tag", "v0"):
                    np.testing.assert_array_equal(got[k][sl], w[k])
        finally:
            for p in ptrs.values():
                hip.hipFree(p)


def test_two_jobs_on_one_engine():
    """JobCausalLogImpl is per job (JobCausalLogFactory.java:56-67): two jobs on one
    TaskManager's engine keep separate logs for the same CausalLogID, separate sharing
    depths, and separate latestCompletedCheckpoint CAS states (:230-246)."""
    with Engine(segment_bytes=64, pool_segments=1 << 10) as eng:
        ja = 0
        jb = eng.open_job((0xA, 0xB), sharing_depth=-1)
        jz = eng.open_job((0xC, 0xD), sharing_depth=0)  # logging switched off for this job
        cid = CausalLogID.main(3)
        la, lb, lz = eng.open_log(cid, ja), eng.open_log(cid, jb), eng.open_log(cid, jz)
        assert len({la.handle, lb.handle, lz.handle}) == 3
        ra, rb = O.OracleLog(64), O.OracleLog(64)
        for e in range(4):
            for k in range(30):
                a = bytes([0, k % 4])
                b = bytes([1]) + (e * 1000 + k).to_bytes(8, "big")
                la.appendDeterminant(a, e)
                ra.append(e, a)
                lb.appendDeterminant(b, e)
                rb.append(e, b)
                lz.appendDeterminant(b, e)  # depth 0: a no-op (:160-161)
        assert lz.state()["writer"] == 0
        assert eng.get_log(cid, jb).handle == lb.handle and eng.get_log(cid, ja).handle == la.handle
        # job A completes checkpoint 3: only its logs are truncated
        assert eng.truncate_all(3, ja)
        assert ra.checkpoint_complete(3) == 0
        assert la.state() == ra.state() and lb.state() == rb.state()
        # job B has not seen any checkpoint yet: an older id than A's still fans out
        assert eng.truncate_all(2, jb)
        assert rb.checkpoint_complete(2) == 0
        assert lb.state() == rb.state()
        assert not eng.truncate_all(2, jb) and not eng.truncate_all(1, ja)  # CAS per job
        assert la.getDeterminants(3) == ra.get_determinants(3)[1]
        assert lb.getDeterminants(2) == rb.get_determinants(2)[1]
        eng.close_job(jb)
        assert eng.get_log(cid, jb) is None and eng.get_log(cid, ja) is not None


def test_get_delta_with_concurrent_appender():
    """getDeltaForConsumer on one thread while appendDeterminant runs on another (the
    Netty thread vs the task thread, ThreadCausalLogImpl's epochReadLock + synchronized(buf)):
    the size probe and the fetch are two calls, so a delta that grew in between must be
    re-fetched (CLG_E_CAPACITY never advances the consumer).  The deltas a consumer receives
    concatenate to exactly the log."""
    import threading
    with Engine(segment_bytes=256, pool_segments=1 << 12) as eng:
        log = eng.open_log(CausalLogID.main(9))
        recs = [bytes([1]) + i.to_bytes(8, "big") for i in range(4000)]
        log.appendDeterminant(recs[0], 0)
        done = threading.Event()

        def appender():
            for r in recs[1:]:
                log.appendDeterminant(r, 0)
            done.set()

        t = threading.Thread(target=appender)
        t.start()
        ch = (5, 5)
        got = []
        assert log.hasDeltaForConsumer(ch, 0)
        while True:
            fin = done.is_set()
            got.append(log.getDeltaForConsumer(ch, 0))
            if fin:
                break
        t.join()
        got.append(log.getDeltaForConsumer(ch, 0))
        assert b"".join(got) == b"".join(recs)


@pytest.mark.parametrize("tail", [0, 64, 16384])
def test_many_threads_many_logs(tail):
    """Eight task/Netty thread pairs on eight logs at once (the lock split: per-log calls
    take the engine lock shared + the log's stripe) while another thread keeps forcing
    whole-engine work (sync = flush + GPU, log_lengths).  Every consumer's deltas
    concatenate to exactly its log, and every log ends byte-identical to the oracle's
    ThreadCausalLogImpl fed the same records."""
    import threading
    import _oracle as O
    T, N = 8, 1500
    with Engine(segment_bytes=256, pool_segments=1 << 13, host_tail_bytes=tail) as eng:
        logs = [eng.open_log(CausalLogID.main(100 + t)) for t in range(T)]
        recs = [[bytes([1]) + (t * N + i).to_bytes(8, "big") for i in range(N)] for t in range(T)]
        got = [[] for _ in range(T)]
        errs = []
        stop = threading.Event()

        done_n = [0] * T

        def appender(t):
            try:
                for i, r in enumerate(recs[t]):
                    logs[t].appendDeterminant(r, i // 500)
                    done_n[t] += 1
            except Exception as ex:  # pragma: no cover - surfaced below
                errs.append(ex)

        def slicer(t, app):
            # moves to epoch ep+1 only once a record of it was appended before the last
            # drain of ep (a consumer moving on abandons the rest of its epoch, :204-214)
            try:
                ch = (7, t)
                ep = 0
                while True:
                    n = done_n[t]
                    if logs[t].hasDeltaForConsumer(ch, ep):
                        got[t].append(logs[t].getDeltaForConsumer(ch, ep))
                    if n >= N and ep == (N - 1) // 500:
                        break
                    if n > 500 * (ep + 1):
                        ep += 1
            except Exception as ex:  # pragma: no cover
                errs.append(ex)

        def whole_engine():
            while not stop.is_set():
                eng.sync()
                eng.log_lengths(np.array([lg.handle for lg in logs], np.uint32))

        apps = [threading.Thread(target=appender, args=(t,)) for t in range(T)]
        slis = [threading.Thread(target=slicer, args=(t, apps[t])) for t in range(T)]
        w = threading.Thread(target=whole_engine)
        for th in apps + slis + [w]:
            th.start()
        for th in apps + slis:
            th.join(timeout=120)
        stop.set()
        w.join(timeout=60)
        assert not errs, errs
        for t in range(T):
            assert b"".join(got[t]) == b"".join(recs[t]), t
            ol = O.OracleLog(256)
            for i, r in enumerate(recs[t]):
                ol.append(i // 500, r)
            assert logs[t].getDeterminants(0) == ol.get_determinants(0)[1]


def test_many_logs_batched_upstream_and_truncation():
    """A device-input upstream batch over 6000 logs, each receiving its epoch as two
    overlapping deltas in ONE batch (the second re-delivers part of the first: dedup), three
    epochs, then the job's truncation.  Every log's state and bytes == the oracle's
    ThreadCausalLogImpl fed the same calls (pooled epoch objects, flat epoch maps)."""
    import torch
    from clonos_amd import _lib
    from clonos_amd import dist as X
    n_logs, seg = 6000, 256
    rng = np.random.default_rng(77)
    with Engine(segment_bytes=seg, pool_segments=n_logs * 8, ifl_pool_segments=16) as eng:
        logs = [eng.open_log(CausalLogID.main(v)) for v in range(n_logs)]
        oracle = [O.OracleLog(seg) for _ in range(n_logs)]
        for ep in range(3):
            blobs = [synth.random_log(int(rng.integers(0, 40)), rng, allow_serializable=False) for _ in range(n_logs)]
            host = bytearray()
            reqs = np.zeros(2 * n_logs, X.DELTA_REQ)
            k = 0
            for i, b in enumerate(blobs):
                cut = int(rng.integers(0, len(b) + 1))
                for off, part in ((0, b[:max(cut, len(b) // 2)]), (cut // 2, b[cut // 2:])):
                    reqs[k] = (logs[i].handle, off, ep, len(host), len(part), 0)
                    host += part
                    k += 1
                    assert oracle[i].upstream(part, off, ep) == 0
            d = torch.frombuffer(bytearray(host or b"\0"), dtype=torch.uint8).to("cuda")
            _lib.check(_lib.lib.clg_upstream_delta_batch(eng.handle, reqs.ctypes.data, len(reqs), d.data_ptr(),
                                                         _lib.CLG_MEM_DEVICE))
            assert (reqs["status"] == 0).all()
        assert eng.truncate_all(2)
        for i in range(n_logs):
            assert oracle[i].checkpoint_complete(2) == 0
        for i in rng.choice(n_logs, 400, replace=False):
            assert logs[i].state() == oracle[i].state(), i
            assert logs[i].getDeterminants(2) == oracle[i].get_determinants(2)[1], i


def _parallel_upstream_round(eng, logs, rng, ep, gap_at, n_recs=(1, 6), prev=None):
    """One device-input batch, one request per log (the engine's per-part path above 8192
    logs): fresh epochs, some empty, one gap, and (prev: the previous round's parts) every
    third log re-delivering its previous delta (nothing new: the dedup)."""
    import torch
    from clonos_amd import _lib
    from clonos_amd import dist as X
    host = bytearray()
    reqs = np.zeros(len(logs), X.DELTA_REQ)
    parts = []
    for i, l in enumerate(logs):
        e, off = ep, 0
        b = synth.random_log(int(rng.integers(*n_recs)), rng, allow_serializable=False)
        if prev is not None and i % 3 == 0:
            b, off, e = prev[i]
        elif i % 97 == 5:
            b = b""  # empty delta
        elif i == gap_at:
            off = 3  # offsetFromEpoch past the epoch's end in the log: a gap
        reqs[i] = (l.handle, off, e, len(host), len(b), 0)
        host += b
        parts.append((b, off, e))
    d = torch.frombuffer(bytearray(host or b"\0"), dtype=torch.uint8).to("cuda")
    _lib.lib.clg_upstream_delta_batch(eng.handle, reqs.ctypes.data, len(reqs), d.data_ptr(), _lib.CLG_MEM_DEVICE)
    torch.cuda.synchronize()
    return reqs["status"].copy(), parts


def test_parallel_upstream_batch_matches_oracle_and_serial():
    """A device-input upstream batch of 9000 logs (one request each, so the engine places
    segments and scatter chunks per part of the requests) with a gap, empty deltas and
    re-deliveries: every status and every log's bytes equal the oracle's
    ThreadCausalLogImpl.processUpstreamDelta (:117-154) and the one-thread engine's; then a
    batch the pool cannot serve whole gives the same statuses in both engines (the
    request-order path)."""
    import os
    n_logs, seg = 9000, 256
    res = {}
    for threads in ("8", "1"):
        old = os.environ.get("CLONOS_HOST_THREADS")
        os.environ["CLONOS_HOST_THREADS"] = threads
        try:
            rng = np.random.default_rng(91)
            with Engine(segment_bytes=seg, pool_segments=n_logs * 4 + 100, ifl_pool_segments=16) as eng:
                logs = [eng.open_log(CausalLogID.main(v)) for v in range(n_logs)]
                oracle = [O.OracleLog(seg) for _ in range(n_logs)]
                sts, prev = [], None
                for ep in range(2):
                    # epoch 0 with a gap (the request-order path), epoch 1 without (per part)
                    st, parts = _parallel_upstream_round(eng, logs, rng, ep, gap_at=1234 if ep == 0 else -1,
                                                         prev=prev)
                    for i, (b, off, e) in enumerate(parts):
                        assert int(st[i]) == oracle[i].upstream(b, off, e), (threads, ep, i)
                    assert (st != 0).sum() == (1 if ep == 0 else 0)
                    sts.append(st)
                    prev = parts
                for i in range(0, n_logs, 37):
                    assert logs[i].getDeterminants(0) == oracle[i].get_determinants(0)[1], i
                    assert logs[i].state() == oracle[i].state(), i
                # the pool cannot hold this batch: request order decides who gets segments
                st_big, _ = _parallel_upstream_round(eng, logs, rng, 2, gap_at=-1, n_recs=(100, 200))
                assert (st_big != 0).any() and (st_big == 0).any()
                res[threads] = (sts, st_big, [logs[i].getDeterminants(0) for i in range(0, n_logs, 53)])
        finally:
            if old is None:
                os.environ.pop("CLONOS_HOST_THREADS", None)
            else:
                os.environ["CLONOS_HOST_THREADS"] = old
    a, b = res["8"], res["1"]
    assert all((x == y).all() for x, y in zip(a[0], b[0]))
    assert (a[1] == b[1]).all() and a[2] == b[2]


def test_many_span_decode_chunked_on_host_threads():
    """A decode of 9000 logs (the count pass's equal-cost chunk boundaries placed per part of
    the spans on the host threads): bit-exact against the oracle on a sample and on the fast
    path (a wrong chunk table would leave tiles uncounted and send the batch robust)."""
    rng = np.random.default_rng(93)
    n_logs, seg = 9000, 4096
    with Engine(segment_bytes=seg, pool_segments=n_logs * 4, timing=True, ifl_pool_segments=16) as eng:
        logs, blobs = [], []
        for v in range(n_logs):
            l = eng.open_log(CausalLogID.main(v))
            n = int(rng.integers(1, 400)) if v % 50 else int(rng.integers(2000, 6000))  # a few long logs
            b = synth.random_log(n, rng, allow_serializable=False)
            l.processUpstreamDelta(b, 0, 0)
            logs.append(l)
            blobs.append(b)
        eng.kernel_stats_reset()
        dec = eng.decode_logs(logs, [0] * n_logs)
        ks = eng.kernel_stats()
        assert "decode_count" in ks and "decode_fallback" not in ks and "decode_span_fallback" not in ks, ks
        from test_gpu_decode import assert_span_equal
        for s in list(range(0, n_logs, 97)) + [n_logs - 1]:
            assert_span_equal(dec, s, blobs[s])
        assert dec.n_rec == sum(len(O.decode(b)[1]["tag"]) for b in blobs[::1])
        # the asynchronous decode of the same batch plans on the host threads too (twice: the
        # second reuses the first's recycled plan): the same records
        for _ in range(2):
            got = eng.decode_logs_async(logs, [0] * n_logs).wait()
            for f in ("off", "tag", "v0", "w_idx", "w_rc", "w_v1", "w_var_off", "w_var_len", "w_sub", "span_rec_base"):
                np.testing.assert_array_equal(getattr(got, f), getattr(dec, f), err_msg=f)


@pytest.mark.parametrize("case", ["error", "serializable"])
def test_many_span_staged_plan_fallbacks(case):
    """A 9000-log decode whose plan is staged straight into the decode slot's pinned buffer
    (engine.cpp plan_parallel, DecodePlan::staged), synchronous and queued, when the fast run
    aborts and the fallbacks plan the batch again from its builder: a decode error in one log
    (the oracle's status, span, offset and tag; kept on the fast path or decoded by the per-span
    fallback), or Serializable records in a few logs while the engine's last batches had none
    (the fast run without tables aborts, the batch goes again with them): every sampled span
    equals the oracle's."""
    from test_gpu_decode import assert_span_equal
    rng = np.random.default_rng(94 if case == "error" else 95)
    n_logs, seg = 9000, 4096
    with Engine(segment_bytes=seg, pool_segments=n_logs * 4, timing=True, ifl_pool_segments=16) as eng:
        logs, blobs = [], []
        for v in range(n_logs):
            lg = eng.open_log(CausalLogID.main(v))
            b = synth.random_log(int(rng.integers(1, 300)), rng, allow_serializable=False)
            if case == "error" and v == 4321:
                b = b[:len(b) // 2] + b"\x08" + b[len(b) // 2:]  # tag 8: decodeNext rejects it
            if case == "serializable" and v % 1500 == 7:
                b = b + synth.random_log(40, rng, allow_serializable=True) + D.encode(
                    D.SerializableDeterminant(D.jser_string("s" * 20)))
            lg.processUpstreamDelta(b, 0, 0)
            logs.append(lg)
            blobs.append(b)
        bad = [(s, O.decode(b)) for s, b in enumerate(blobs)]
        bad = [(s, r) for s, r in bad if r[0] != 0]
        sample = sorted(set(list(range(0, n_logs, 89)) + [7, 1507, 4321, n_logs - 1]))
        for mode in ("async", "sync", "async"):  # (the first decode of the Serializable case aborts)
            if case == "error":
                s, (st, _, eo, et) = bad[0]
                with pytest.raises(ClonosError) as ex:
                    if mode == "sync":
                        eng.decode_logs(logs, [0] * n_logs)
                    else:
                        eng.decode_logs_async(logs, [0] * n_logs).wait()
                assert (ex.value.status, ex.value.err_span, ex.value.err_off, ex.value.err_tag) == (st, s, eo, et)
            else:
                assert not bad
                dec = eng.decode_logs(logs, [0] * n_logs) if mode == "sync" else \
                    eng.decode_logs_async(logs, [0] * n_logs).wait()
                for s in sample:
                    assert_span_equal(dec, s, blobs[s])
        ks = eng.kernel_stats()
        if case == "error":  # the fallbacks ran: the error kept, or its span decoded apart
            assert "decode_kept_errors" in ks or "decode_span_fallback" in ks, sorted(ks)
        else:  # the fast run without tables aborted, and ran again with them
            assert "decode_jser_retry" in ks, sorted(ks)
