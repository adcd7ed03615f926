"""GPU: the engine's in-flight (data) log (HBM segments, batched replay gather) == the
oracle's literal simulation of InMemorySubpartitionInFlightLogger + ReplayIterator
(oracle/inflight_ref.py), byte for byte, over random logs, truncations, skips and gaps."""
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "oracle"))

from inflight_ref import InFlightLogRef  # noqa: E402
from clonos_amd import ClonosError, Engine, _lib  # noqa: E402
from clonos_amd import inflight as IF  # noqa: E402

pytestmark = pytest.mark.gpu

STATUS = {"ok": _lib.CLG_OK, "gap": _lib.CLG_E_EPOCH_GAP, "state": _lib.CLG_E_STATE}
EDGE_SIZES = [0, 1, 15, 16, 255, 256, 257, 4095, 4096, 32768]


def _check(reps, refs, reqs):
    for rep, (ref, start, ign) in zip(reps, [(refs[f], s, i) for f, s, i in reqs]):
        st, bufs, rem, eps, end = ref.replay_full(start, ign)
        assert rep.status == STATUS[st], (start, ign, rep.status, st)
        assert rep.buffers == bufs
        if st != "state":
            assert rep.remaining == rem and rep.epochs == eps and rep.end_epoch == end


@pytest.mark.parametrize("seg", [256, 16384])
@pytest.mark.parametrize("seed", [0, 1, 2])
def test_inflight_random_vs_oracle(seg, seed):
    rng = np.random.default_rng(0x1F1 + seed)
    with Engine(segment_bytes=seg, pool_segments=(64 << 20) // seg, timing=True) as eng:
        logs = [IF.InFlightLog(eng) for _ in range(6)]
        refs = {f: InFlightLogRef() for f in logs}
        epoch = 0
        for rnd in range(8):
            items = []
            for f in logs:
                skip_epoch = rng.random() < 0.15  # some subpartitions send nothing this epoch
                if skip_epoch:
                    continue
                for _ in range(int(rng.integers(1, 6))):
                    n = int(rng.choice(EDGE_SIZES)) if rng.random() < 0.3 else int(rng.integers(0, 40000))
                    items.append((f, epoch, rng.integers(0, 256, n, dtype=np.uint8).tobytes()))
            IF.log_batch(eng, items)
            for f, e, b in items:
                refs[f].log(b, e)
            if rnd in (3, 6):
                cp = epoch - 1
                for f in logs:
                    f.notify_checkpoint_complete(cp)
                    refs[f].notify_checkpoint_complete(cp)
            epoch += 1
            for f in logs:
                assert f.epochs() == [(k, len(v)) for k, v in sorted(refs[f].sliced.items())]
            reqs = []
            for f in logs:
                for _ in range(3):
                    start = int(rng.integers(max(0, epoch - 5), epoch + 1))
                    reqs.append((f, start, int(rng.integers(0, 8))))
            _check(IF.replay_batch(eng, reqs), refs, reqs)
        for f in logs:
            f.close()
        used, _ = eng.ifl_pool_stats()
        assert used == 0 and eng.pool_stats()[0] == 0  # the determinant pool was never touched


def test_inflight_reference_scenario_and_gap():
    with Engine(segment_bytes=16384, pool_segments=256) as eng:
        f = IF.InFlightLog(eng)
        ref = InFlightLogRef()
        for epoch in range(3):  # InFlightLogTest.populate
            for i in range(6):
                b = bytes([epoch, i]) * 32
                f.log(b, epoch)
                ref.log(b, epoch)
        assert f.get_in_flight_iterator(0, 0).number_remaining() == 18  # iteratorCountTest
        f.notify_checkpoint_complete(1)
        ref.notify_checkpoint_complete(1)
        it = f.get_in_flight_iterator(0, 0)
        assert it.number_remaining() == 0 and not it.has_next()  # code, not the test's 12 / true
        assert list(f.get_in_flight_iterator(1, 2)) == ref.replay(1, 2)[1]
        f.log(b"late", 4)  # epoch 3 never logged: a gap
        ref.log(b"late", 4)
        reqs = [(f, 1, 0), (f, 1, 11), (f, 1, 12), (f, 4, 0), (f, 3, 0), (f, 3, 1)]
        _check(IF.replay_batch(eng, reqs), {f: ref}, reqs)
        it = f.get_in_flight_iterator(1, 0)
        got = []
        with pytest.raises(ClonosError):
            while it.has_next():
                got.append(it.next())
        assert got == ref.replay(1, 0)[1] and len(got) == 11


def test_inflight_device_output_and_capacity():
    """Device memory from the engine's own HIP runtime (ctypes), as in test_gpu_log.py."""
    import ctypes
    hip = ctypes.CDLL("libamdhip64.so.7")
    rng = np.random.default_rng(7)
    with Engine(segment_bytes=16384, pool_segments=1 << 12) as eng:
        logs = [IF.InFlightLog(eng) for _ in range(32)]
        items = [(f, e, rng.integers(0, 256, int(rng.integers(1, 32769)), dtype=np.uint8).tobytes())
                 for e in range(3) for f in logs for _ in range(2)]
        IF.log_batch(eng, items)
        reqs = [(f, 0, 1) for f in logs]
        st, cres, out, sizes, total, nbuf = IF.replay_batch_raw(eng, reqs, out=np.zeros(16, np.uint8))
        assert st == _lib.CLG_E_CAPACITY and total > 16 and nbuf == 32 * 5
        dptr = ctypes.c_void_p()
        assert hip.hipMalloc(ctypes.byref(dptr), ctypes.c_size_t(total)) == 0
        try:
            st, cres, _, sizes, total2, _ = IF.replay_batch_raw(eng, reqs, out=dptr.value, cap=total)
            assert st == _lib.CLG_OK and total2 == total
            hb = np.empty(total, np.uint8)
            assert hip.hipMemcpy(ctypes.c_void_p(hb.ctypes.data), dptr, ctypes.c_size_t(total), 2) == 0
            host = hb.tobytes()
        finally:
            hip.hipFree(dptr)
        # per log: drop the first buffer (ignore_buffers=1)
        exp = b"".join(b"".join([b for (g, ee, b) in items if g is f][1:]) for f in logs)
        assert host == exp


def test_inflight_golden_fixture():
    """The engine replays tests/golden/inflight_ops.json byte for byte (64-B segments, so
    buffers span several segments)."""
    import json
    d = json.load(open(os.path.join(ROOT, "tests", "golden", "inflight_ops.json")))
    with Engine(segment_bytes=d["segment_bytes"], pool_segments=1 << 14) as eng:
        for c in d["cases"]:
            logs = [IF.InFlightLog(eng) for _ in range(c["n_sub"])]
            got = []
            for op in c["ops"]:
                if op[0] == "log":
                    logs[op[1]].log(bytes.fromhex(op[3]), op[2])
                elif op[0] == "cp":
                    logs[op[1]].notify_checkpoint_complete(op[2])
                else:
                    reps = IF.replay_batch(eng, [(logs[s], st, ign) for s, st, ign in op[1]])
                    got.append([[{v: k for k, v in STATUS.items()}[r.status], [b.hex() for b in r.buffers],
                                 r.remaining if r.status != _lib.CLG_E_STATE else None,
                                 r.epochs if r.status != _lib.CLG_E_STATE else [],
                                 r.end_epoch if r.status != _lib.CLG_E_STATE else None] for r in reps])
            assert got == c["expect"]
            for f in logs:
                f.close()
        assert eng.ifl_pool_stats()[0] == 0


def test_inflight_pool_is_separate_and_reports_nospace():
    """The in-flight log has its own pool: a full in-flight pool is CLG_E_NOSPACE with
    nothing logged (the caller waits for a checkpoint: backpressure), and it never takes
    the segments appendDeterminant needs."""
    with Engine(segment_bytes=64, pool_segments=8, ifl_segment_bytes=1024, ifl_pool_segments=4) as eng:
        f = IF.InFlightLog(eng)
        f.log(b"a" * 2048, 0)  # two segments
        with pytest.raises(ClonosError) as ei:
            f.log(b"b" * 3000, 1)  # three more: the pool holds four
        assert ei.value.status == _lib.CLG_E_NOSPACE
        assert f.epochs() == [(0, 1)] and eng.ifl_pool_stats() == (2, 2)
        from clonos_amd import CausalLogID
        log = eng.open_log(CausalLogID.main(1))  # the determinant pool is untouched
        for _ in range(7):
            log.appendDeterminant(b"\x00\x01" * 32, 0)
        f.notify_checkpoint_complete(1)  # frees epoch 0: the retry fits
        f.log(b"b" * 3000, 1)
        assert f.epochs() == [(1, 1)] and eng.ifl_pool_stats() == (3, 1)


def test_inflight_log_from_device_memory():
    """clg_ifl_log_batch with CLG_MEM_DEVICE input (a buffer already in HBM, e.g. the
    network stack's output) == the same buffers logged from host memory."""
    import ctypes
    hip = ctypes.CDLL("libamdhip64.so.7")
    rng = np.random.default_rng(11)
    bufs = [rng.integers(0, 256, int(n), dtype=np.uint8).tobytes() for n in (0, 1, 16383, 16384, 16385, 40000, 7)]
    blob = np.frombuffer(b"".join(bufs), np.uint8).copy()
    lens = np.array([len(b) for b in bufs], np.uint32)
    offs = np.zeros(len(bufs), np.uint64)
    offs[1:] = np.cumsum(lens[:-1], dtype=np.uint64)
    with Engine(segment_bytes=16384, pool_segments=256) as eng:
        f = IF.InFlightLog(eng)
        dptr = ctypes.c_void_p()
        assert hip.hipMalloc(ctypes.byref(dptr), ctypes.c_size_t(blob.size)) == 0
        try:
            assert hip.hipMemcpy(dptr, ctypes.c_void_p(blob.ctypes.data), ctypes.c_size_t(blob.size), 1) == 0
            h = np.full(len(bufs), f.handle, np.uint32)
            ep = np.array([0, 0, 0, 1, 1, 2, 2], np.int64)
            _lib.check(_lib.lib.clg_ifl_log_batch(eng.handle, h.ctypes.data, ep.ctypes.data, offs.ctypes.data,
                                                  lens.ctypes.data, len(bufs), dptr.value, _lib.CLG_MEM_DEVICE))
        finally:
            hip.hipFree(dptr)
        assert f.epochs() == [(0, 3), (1, 2), (2, 2)]
        rep = f.replay(0, 0)
        assert rep.status == _lib.CLG_OK and rep.buffers == bufs and rep.remaining == len(bufs)
        f.close()
        assert eng.ifl_pool_stats()[0] == 0
