"""GPU: the engine's spillable in-flight log (the reference's default logger,
SpillableSubpartitionInFlightLogger + SpilledReplayIterator, InFlightLogConfig.java:44) == the
oracle's literal simulation (oracle/inflight_ref.py SpillableInFlightLogRef), byte for byte:
tailMap iterators, null iterators, skips, gaps, partial drains, buffers logged during a replay
reaching the live iterator, truncation during a replay and log() after a null first iterator."""
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "oracle"))

from inflight_ref import IteratorNPE, SpillableInFlightLogRef  # noqa: E402
from clonos_amd import ClonosError, Engine, _lib  # noqa: E402
from clonos_amd import inflight as IF  # noqa: E402

pytestmark = pytest.mark.gpu

STATUS = {"ok": _lib.CLG_OK, "gap": _lib.CLG_E_EPOCH_GAP, "state": _lib.CLG_E_STATE, "null": _lib.CLG_OK}


def _same(rep, ref_res, replaying=None):
    st, bufs, rem, eps, end = ref_res
    assert rep.status == STATUS[st], (rep.status, st)
    if replaying is not None:
        assert bool(rep.flags & _lib.CLG_IFL_REPLAYING) == replaying
    assert rep.null_iterator == (st == "null")
    assert rep.buffers == bufs
    if st not in ("state", "null"):
        assert rep.remaining == rem and rep.epochs == eps and rep.end_epoch == end, (rep.remaining, rem, rep.epochs,
                                                                                     eps, rep.end_epoch, end)


def _log(eng, f, ref, epoch, data):
    """log() on both; the engine reports the reference's NullPointerException as CLG_E_STATE."""
    try:
        ref.log(data, epoch)
        npe = False
    except IteratorNPE:
        npe = True
    if npe:
        with pytest.raises(ClonosError) as ex:
            f.log(data, epoch)
        assert ex.value.status == _lib.CLG_E_STATE
    else:
        f.log(data, epoch)


def test_reference_inflightlogtest_expectations_hold_for_spillable():
    """InFlightLogTest.logCheckpointCompleteTest / logIterationTest (12 remaining, hasNext after
    truncating epoch 0 and replaying from 0) hold for the spillable logger's tailMap iterator."""
    with Engine(segment_bytes=256, pool_segments=1024) as eng:
        f = IF.InFlightLog(eng, "spillable")
        for epoch in range(3):
            for i in range(6):
                f.log(bytes([epoch, i]) * 32, epoch)
        it = f.get_in_flight_iterator(0, 0)
        assert it.number_remaining() == 15 + 3  # iteratorCountTest
        f.notify_checkpoint_complete(1)
        it = f.get_in_flight_iterator(0, 0)
        assert it.number_remaining() == 10 + 2 and it.has_next()
        got = list(it)
        assert got == [bytes([e, i]) * 32 for e in (1, 2) for i in range(6)]
        f.close()


@pytest.mark.parametrize("seed", range(6))
def test_spillable_random_script_vs_oracle(seed):
    rng = np.random.default_rng(0x5B111 + seed)
    with Engine(segment_bytes=256, pool_segments=4096, ifl_segment_bytes=256, ifl_pool_segments=1 << 15) as eng:
        logs = [IF.InFlightLog(eng, "spillable") for _ in range(3)]
        refs = {f: SpillableInFlightLogRef() for f in logs}
        epoch = 0
        for step in range(120):
            f = logs[int(rng.integers(0, len(logs)))]
            ref = refs[f]
            op = rng.random()
            if op < 0.45:  # log a buffer (sometimes skipping an epoch: gaps)
                if rng.random() < 0.25:
                    epoch += int(rng.integers(1, 3))
                n = int(rng.integers(0, 700))
                _log(eng, f, ref, epoch, rng.integers(0, 256, n, dtype=np.uint8).tobytes())
            elif op < 0.55:  # checkpoint complete (possibly during a replay)
                cp = int(rng.integers(max(0, epoch - 3), epoch + 1))
                f.notify_checkpoint_complete(cp)
                ref.notify_checkpoint_complete(cp)
            elif op < 0.8:  # a new iterator, partially drained
                start = int(rng.integers(max(0, epoch - 4), epoch + 2))
                ign = int(rng.integers(0, 4))
                mx = int(rng.integers(0, 4))
                want = ref.replay_full(start, ign, mx)
                _same(f.replay(start, ign, mx), want, ref.replaying)
            else:  # continue the current iterator
                mx = int(rng.integers(0, 4))
                rep = f.replay_continue(mx)
                want = ref.continue_full(mx)
                if want[0] == "state":
                    assert rep.status == _lib.CLG_E_STATE
                else:
                    _same(rep, want, ref.replaying)
            assert f.epochs() == [(k, len(v)) for k, v in sorted(ref.sliced.items())]
        for f in logs:
            f.close()
        assert eng.ifl_pool_stats()[0] == 0


def test_live_iterator_sees_buffers_logged_during_replay():
    with Engine(segment_bytes=256, pool_segments=1024) as eng:
        f = IF.InFlightLog(eng, "spillable")
        ref = SpillableInFlightLogRef()
        for e, b in ((3, b"a"), (3, b"b"), (4, b"c")):
            f.log(b, e)
            ref.log(b, e)
        it = f.get_in_flight_iterator(3, 0, chunk=2)
        rit = ref.get_in_flight_iterator(3, 0)
        assert it.next() == rit.next() == b"a"
        for e, b in ((4, b"d"), (5, b"e")):  # during the replay: they reach the iterator
            f.log(b, e)
            ref.log(b, e)
        got = list(it)
        want = []
        while rit.has_next():
            want.append(rit.next())
        assert got == want == [b"b", b"c", b"d", b"e"]
        assert not ref.replaying
        f.log(b"f", 5)  # after the drain: no longer replaying, the old iterator is not told
        ref.log(b"f", 5)
        assert f.replay_continue().buffers == [] and ref.continue_full()[1] == []
        f.close()


def test_null_iterator_then_log_throws_npe():
    """getInFlightIterator on an empty tailMap returns null but sets isReplaying (:132-135): with
    no iterator ever built, the next log() appends and then throws a NullPointerException."""
    with Engine(segment_bytes=256, pool_segments=1024) as eng:
        f = IF.InFlightLog(eng, "spillable")
        assert f.get_in_flight_iterator(0, 0) is None
        with pytest.raises(ClonosError) as ex:
            f.log(b"x", 0)
        assert ex.value.status == _lib.CLG_E_STATE
        assert f.epochs() == [(0, 1)]  # appended before the exception
        it = f.get_in_flight_iterator(0, 0)
        assert list(it) == [b"x"]
        f.close()


def test_in_memory_rejects_spillable_requests():
    with Engine(segment_bytes=256, pool_segments=1024) as eng:
        f = IF.InFlightLog(eng)
        f.log(b"x", 0)
        assert f.replay(0, 0, 1).status == _lib.CLG_E_INVALID_ARG
        assert f.replay_continue().status == _lib.CLG_E_INVALID_ARG
        f.close()
