"""CPU: the in-flight log oracle (oracle/inflight_ref.py) against the reference's own
InFlightLogTest (flink-runtime/src/test/java/org/apache/flink/runtime/inflightlogging/
InFlightLogTest.java) and hand-derived iterator cases; the host mirror's API surface."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "oracle"))

from inflight_ref import InFlightLogRef, IteratorNPE  # noqa: E402
import pytest  # noqa: E402


def populate(log):  # InFlightLogTest.populate: 3 epochs x (5 + 1) buffers of 64 B
    for epoch in range(3):
        for i in range(6):
            log.log(bytes([epoch, i]) * 32, epoch)


def test_iterator_count():  # InFlightLogTest.iteratorCountTest
    log = InFlightLogRef()
    populate(log)
    assert log.get_in_flight_iterator(0, 0).number_remaining() == 15 + 3


def test_checkpoint_complete_then_iterate_from_truncated_epoch():
    # InFlightLogTest.logCheckpointCompleteTest / logIterationTest assert 12 remaining and
    # hasNext() == true here, but InMemorySubpartitionInFlightLogger.ReplayIterator
    # (:121-127) builds an empty iterator when the start epoch is not a key: the code
    # yields 0 / false, and that code is what the engine follows.
    log = InFlightLogRef()
    populate(log)
    log.notify_checkpoint_complete(1)
    assert sorted(log.sliced) == [1, 2]
    it = log.get_in_flight_iterator(0, 0)
    assert it.number_remaining() == 0 and not it.has_next()
    it = log.get_in_flight_iterator(1, 0)
    assert it.number_remaining() == 12 and it.has_next()


def test_replay_order_and_skip():
    log = InFlightLogRef()
    populate(log)
    st, bufs, rem = log.replay(1, 4)
    assert st == "ok" and rem == 12 - 4
    assert bufs == [bytes([1, i]) * 32 for i in range(4, 6)] + [bytes([2, i]) * 32 for i in range(6)]
    assert log.replay(2, 6) == ("ok", [], 0)
    assert log.replay(2, 7)[0] == "state"
    assert log.replay(5, 0) == ("ok", [], 0)
    assert log.replay(5, 1)[0] == "state"


def test_epoch_gap_loses_last_buffer_before_it():
    log = InFlightLogRef()
    for e, n in ((0, 3), (2, 2)):
        for i in range(n):
            log.log(bytes([e, i]), e)
    st, bufs, rem = log.replay(0, 0)
    assert st == "gap" and bufs == [bytes([0, 0]), bytes([0, 1])] and rem == 5
    st, bufs, rem = log.replay(0, 3)  # the skip loop inside getInFlightIterator reaches the gap
    assert st == "state" and bufs == [] and rem == 0
    # a skip that stops right before the gap succeeds; only the next next() throws
    st, bufs, rem, eps, end = log.replay_full(0, 2)
    assert (st, bufs, rem, eps, end) == ("gap", [], 3, [], 0)
    assert log.replay(2, 0) == ("ok", [bytes([2, 0]), bytes([2, 1])], 2)
    # one buffer before the gap (K = 1): the iterator is built, and next() throws at once
    one = InFlightLogRef()
    one.log(b"a", 0)
    one.log(b"b", 2)
    assert one.replay_full(0, 0) == ("gap", [], 2, [], 0)
    assert one.replay_full(0, 1)[0] == "state"
    it = log.get_in_flight_iterator(0, 0)
    it.next()
    it.next()
    with pytest.raises(IteratorNPE):  # fetches buffer 2, then advances into the gap
        it.next()


def test_host_mirror_exports():
    from clonos_amd import inflight
    for name in ("InFlightLog", "InFlightLogIterator", "log_batch", "replay_batch", "replay_batch_raw"):
        assert hasattr(inflight, name)


def test_golden_fixture_matches_oracle():
    """tests/golden/inflight_ops.json (committed) == a fresh run of the oracle."""
    import json
    sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))
    from make_inflight_golden import run_script
    d = json.load(open(os.path.join(ROOT, "tests", "golden", "inflight_ops.json")))
    kinds = set()
    for c in d["cases"]:
        assert run_script(c["ops"], c["n_sub"]) == c["expect"]
        for e in c["expect"]:  # every replay carries one epoch per buffer, non-decreasing
            for r in e:
                assert r[0] == "state" or (len(r[3]) == len(r[1]) and r[3] == sorted(r[3]))
        kinds |= {r[0] for e in c["expect"] for r in e}
    assert kinds == {"ok", "state", "gap"}


def test_host_iterator_mirrors_reference_iterator():
    """clonos_amd.inflight.InFlightLogIterator over a replay result behaves like the
    oracle's ReplayIterator: same buffers, numberRemaining, and the throw at a gap."""
    from clonos_amd import ClonosError, _lib
    from clonos_amd.inflight import InFlightLogIterator, InFlightReplay
    log = InFlightLogRef()
    for e, n in ((0, 3), (1, 2), (3, 2)):
        for i in range(n):
            log.log(bytes([e, i]), e)
    code = {"ok": _lib.CLG_OK, "gap": _lib.CLG_E_EPOCH_GAP}
    for start, ign in ((0, 0), (0, 2), (0, 4), (3, 0), (3, 1), (1, 0), (1, 1)):
        st, bufs, rem, eps, end = log.replay_full(start, ign)
        mine = InFlightLogIterator(InFlightReplay(code[st], bufs, rem, eps, end), start)
        ref = log.get_in_flight_iterator(start, ign)
        while True:
            assert mine.number_remaining() == ref.number_remaining()
            assert mine.get_epoch() == ref.current_key  # getEpoch() (:181-183)
            try:
                has = ref.has_next()
            except IteratorNPE:
                with pytest.raises(ClonosError):
                    mine.has_next()
                break
            assert mine.has_next() == has
            if not has:
                break
            try:
                want = ref.next()
            except IteratorNPE:  # the reference loses this buffer; the engine never hands it out
                with pytest.raises(ClonosError):
                    mine.next()
                break
            assert mine.next() == want


# ---- the spillable logger (the reference's default, InFlightLogConfig.java:44) ------------------
def test_spillable_satisfies_inflightlogtest():
    """InFlightLogTest's three assertions (iteratorCountTest 18; logCheckpointCompleteTest 12 and
    logIterationTest hasNext after truncating epoch 0 and replaying from 0) all hold for
    SpillableSubpartitionInFlightLogger's tailMap iterator (:133) -- the two the in-memory code
    fails (test_checkpoint_complete_then_iterate_from_truncated_epoch) pin this oracle."""
    from inflight_ref import SpillableInFlightLogRef
    log = SpillableInFlightLogRef()
    populate(log)
    assert log.get_in_flight_iterator(0, 0).number_remaining() == 15 + 3
    log = SpillableInFlightLogRef()
    populate(log)
    log.notify_checkpoint_complete(1)
    it = log.get_in_flight_iterator(0, 0)
    assert it.number_remaining() == 10 + 2 and it.has_next()
    got = []
    while it.has_next():
        got.append(it.next())
    assert got == [bytes([e, i]) * 32 for e in (1, 2) for i in range(6)]
    assert not log.replaying


def test_spillable_gap_throws_before_any_buffer():
    """The prefetch cursor runs into the missing epoch inside the constructor (the exception is
    swallowed there, SpilledReplayIterator :155-157); the consumer's first next() then throws
    from behind() (:175) -- no buffer is delivered.  A skip across the gap throws in the
    constructor (getInFlightIterator fails)."""
    from inflight_ref import SpillableInFlightLogRef
    log = SpillableInFlightLogRef()
    for e, b in ((5, b"a"), (5, b"b"), (7, b"c")):
        log.log(b, e)
    assert log.replay_full(5, 0) == ("gap", [], 3, [], 5)
    assert log.replay_full(5, 2)[0] == "gap"
    assert log.replay_full(5, 3)[0] == "state"
    assert log.replay_full(6, 0) == ("ok", [b"c"], 1, [7], 7)  # tailMap(6) starts at 7
    assert log.replay_full(8, 0)[0] == "null"


def test_spillable_live_append_and_npe():
    from inflight_ref import IteratorNPE, SpillableInFlightLogRef
    log = SpillableInFlightLogRef()
    assert log.get_in_flight_iterator(0, 0) is None and log.replaying
    with pytest.raises(IteratorNPE):  # currentIterator == null (:98-99), after the append
        log.log(b"x", 0)
    assert log.sliced == {0: [b"x"]}
    it = log.get_in_flight_iterator(0, 0)
    log.log(b"y", 0)  # reaches the live iterator
    log.log(b"z", 1)
    assert [it.next() for _ in range(3)] == [b"x", b"y", b"z"] and not log.replaying
    log.log(b"w", 1)  # replay over: not delivered to the old iterator
    assert not it.has_next()
