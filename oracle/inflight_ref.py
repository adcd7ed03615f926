"""TEST INFRASTRUCTURE ONLY -- CPU oracle for the in-flight (data) log.  Only tests/ may
import this; the product path (clonos_amd/) never does.

Restates, step by step, InMemorySubpartitionInFlightLogger
(R = /root/reference/flink-runtime/src/main/java/org/apache/flink/runtime/inflightlogging/
InMemorySubpartitionInFlightLogger.java):
  log            :44-48    slicedLog.computeIfAbsent(epoch, LinkedList).add(buffer)
  notifyCheckpointComplete :51-70  remove every epoch < checkpointId
  getInFlightIterator      :73-82  ReplayIterator(start, slicedLog) then next() x ignoreBuffers
  ReplayIterator           :114-183 (tailMap(start); currentIterator only if start is a key;
                                     numberOfBuffersLeft = sum of tailMap list sizes;
                                     advance: while !hasNext && currentKey < lastKey:
                                     get(++currentKey) -- a missing key is a NullPointerException)
The iterator is simulated literally (no closed form), so it is an independent check of the
engine's batched replay.  Pinned by the reference's own InFlightLogTest
(flink-runtime/src/test/java/org/apache/flink/runtime/inflightlogging/InFlightLogTest.java:
iteratorCountTest; see tests/test_inflight.py for the two tests whose asserts the code
above does not satisfy).
"""
from __future__ import annotations


class IteratorNPE(Exception):
    """NullPointerException / NoSuchElementException inside ReplayIterator."""


class ReplayIterator:
    def __init__(self, start: int, full_log: dict):
        self.current_key = start
        self.log = {k: full_log[k] for k in sorted(full_log) if k >= start}  # tailMap (:119)
        if start in self.log:                                              # :121-127
            self.cur = self.log[start]
            self.pos = 0
            self.left = sum(len(v) for v in self.log.values())
        else:
            self.cur = None
            self.pos = 0
            self.left = 0

    def _advance(self):  # advanceToNextNonEmptyIteratorIfNeeded :131-136
        while self.cur is not None and self.pos >= len(self.cur) and self.current_key < max(self.log):
            self.current_key += 1
            nxt = self.log.get(self.current_key)
            if nxt is None:
                raise IteratorNPE(f"no epoch {self.current_key}")
            self.cur, self.pos = nxt, 0

    def has_next(self) -> bool:  # :146-149
        self._advance()
        return self.cur is not None and self.pos < len(self.cur)

    def next(self):  # :152-158
        self._advance()
        if self.cur is None or self.pos >= len(self.cur):
            raise IteratorNPE("next() past the end")
        b = self.cur[self.pos]
        self.pos += 1
        self.left -= 1
        self._advance()
        return b

    def number_remaining(self) -> int:
        return self.left


class InFlightLogRef:
    def __init__(self):
        self.sliced = {}

    def log(self, buf: bytes, epoch: int):
        self.sliced.setdefault(epoch, []).append(bytes(buf))

    def notify_checkpoint_complete(self, cp: int):
        for k in [k for k in self.sliced if k < cp]:
            del self.sliced[k]

    def get_in_flight_iterator(self, start: int, ignore: int) -> ReplayIterator:
        it = ReplayIterator(start, self.sliced)
        for _ in range(ignore):
            it.next()
        return it

    def replay(self, start: int, ignore: int):
        """(status, buffers, remaining) as clg_ifl_replay_batch reports them:
        status 'ok', 'gap' (the iterator threw after `buffers`) or 'state' (the skip inside
        getInFlightIterator threw, :78-79)."""
        return self.replay_full(start, ignore)[:3]

    def replay_full(self, start: int, ignore: int):
        """(status, buffers, remaining, epochs, end_epoch): epochs[i] is getEpoch()
        (:181-183, currentKey) right before the next() that returned buffers[i] -- the value
        PipelinedSubpartition.getReplayedBufferUnsafe (:306-320) reads; end_epoch is
        getEpoch() after the last successful next() (or after the skip)."""
        try:
            it = ReplayIterator(start, self.sliced)
            for _ in range(ignore):
                it.next()
        except IteratorNPE:
            return "state", [], 0, [], None
        remaining = it.number_remaining()
        out, eps = [], []
        end = it.current_key
        try:
            while it.has_next():
                e = it.current_key
                b = it.next()
                out.append(b)
                eps.append(e)
                end = it.current_key
        except IteratorNPE:
            return "gap", out, remaining, eps, end
        return "ok", out, remaining, eps, it.current_key


# ---- SpillableSubpartitionInFlightLogger (the reference's default, InFlightLogConfig.java:44) ----
# S = SpillableSubpartitionInFlightLogger.java, SI = SpilledReplayIterator.java (same directory).
# The spill files are not modelled: no flush ever completes, so every buffer stays in memory
# (never "recycled") and the prefetcher never waits for a read -- the deterministic case.
# Java exceptions are IteratorNPE here (NullPointerException / IndexOutOfBoundsException).
class _View:
    """tailMap(view) of the logger's live epoch map (S:133): keys >= view."""

    def __init__(self, log: dict, view: int):
        self.log, self.view = log, view

    def get(self, e):
        if e < self.view or e not in self.log:
            raise IteratorNPE(f"log.get({e}) == null")
        return self.log[e]


class EpochCursor:  # SI:306-394
    def __init__(self, view: _View):
        keys = sorted(k for k in view.log if k >= view.view)
        self.v = view
        self.next_epoch = keys[0]      # :316 firstKey
        self.next_off = 0
        self.last_epoch = keys[-1]     # :318 lastKey
        self.remaining = sum(len(view.log[k]) for k in keys)

    def copy(self):
        c = EpochCursor.__new__(EpochCursor)
        c.__dict__.update(self.__dict__)
        return c

    def has_next(self):  # :324-326
        return self.remaining > 0

    def _advance(self):  # :353-358
        if self.next_off == len(self.v.get(self.next_epoch)) and self.next_epoch != self.last_epoch:
            self.next_epoch += 1
            self.next_off = 0

    def get_next_epoch(self):  # :328-331
        self._advance()
        return self.next_epoch

    def get_next_epoch_offset(self):  # :333-336
        self._advance()
        return self.next_off

    def next(self):  # :342-351
        self._advance()
        bufs = self.v.get(self.next_epoch)
        if self.next_off >= len(bufs):
            raise IteratorNPE("buffers.get(offset) past the epoch (IndexOutOfBoundsException)")
        b = bufs[self.next_off]
        self.next_off += 1
        self.remaining -= 1
        self._advance()
        return b

    def behind(self, other):  # :364-367
        return (self.get_next_epoch() < other.get_next_epoch() or
                (self.get_next_epoch() == other.get_next_epoch() and
                 self.get_next_epoch_offset() < other.get_next_epoch_offset()))

    def notify_new_buffer(self, epoch):  # :389-393
        self.remaining += 1
        if epoch > self.last_epoch:
            self.last_epoch = epoch


class SpilledReplayIterator:  # SI:60-277
    def __init__(self, owner, view: _View, ignore: int):
        self.owner = owner
        self.consumer = EpochCursor(view)   # :92
        self.prefetch = EpochCursor(view)   # :93
        for _ in range(ignore):             # :98-101
            self.consumer.next()
            self.prefetch.next()
        self._prefetch()                    # :123

    def _prefetch(self):  # :126-158, exceptions printed and swallowed
        try:
            while self.prefetch.has_next():
                self.prefetch.get_next_epoch()
                self.prefetch.next()   # in memory: retainBuffer only
        except IteratorNPE:
            pass

    def number_remaining(self):  # :160-163
        return self.consumer.remaining

    def get_epoch(self):  # :165-168
        return self.consumer.get_next_epoch()

    def has_next(self):  # :255-260
        return self.consumer.has_next()

    def next(self):  # :170-203
        while not self.consumer.behind(self.prefetch):
            self._prefetch()
            if not self.consumer.behind(self.prefetch):
                raise IteratorNPE("next() would wait forever (nothing left to prefetch)")
        b = self.consumer.next()
        if not self.consumer.has_next():
            self.owner.replaying = False    # :186-187
        self._prefetch()
        return b

    def notify_new_buffer_added(self, epoch):  # :262-277
        self.prefetch.notify_new_buffer(epoch)
        self.consumer.notify_new_buffer(epoch)


class SpillableInFlightLogRef:
    """SpillableSubpartitionInFlightLogger (S:45-341) without the disk: log, notifyCheckpointComplete,
    getInFlightIterator (a live iterator over tailMap(epochID)) and the isReplaying flag."""

    def __init__(self):
        self.sliced = {}
        self.replaying = False   # S:58
        self.current = None      # S:60
        self.closed = False

    def log(self, buf: bytes, epoch: int):  # S:84-103
        if self.closed:
            return
        self.sliced.setdefault(epoch, []).append(bytes(buf))
        if self.replaying:
            if self.current is None:
                raise IteratorNPE("currentIterator == null in log()")  # S:98-99, after the append
            self.current.notify_new_buffer_added(epoch)

    def notify_checkpoint_complete(self, cp: int):  # S:106-123
        for k in [k for k in self.sliced if k < cp]:
            del self.sliced[k]

    def get_in_flight_iterator(self, start: int, ignore: int):  # S:126-142
        if self.closed:
            return None
        self.replaying = True
        if not any(k >= start for k in self.sliced):
            return None
        self.current = SpilledReplayIterator(self, _View(self.sliced, start), ignore)  # may raise (constructor)
        return self.current

    def take(self, it, max_buffers: int = 0):
        """(status, buffers, remaining, epochs, end_epoch) for draining `it` (at most max_buffers,
        0: all), as clg_ifl_replay_batch reports one request: 'ok' or 'gap' (next() threw)."""
        remaining = it.number_remaining()
        out, eps = [], []
        try:
            while it.has_next() and (max_buffers == 0 or len(out) < max_buffers):
                e = it.get_epoch()
                out.append(it.next())
                eps.append(e)
        except IteratorNPE:
            return "gap", out, remaining, eps, it.consumer.next_epoch
        try:
            end = it.get_epoch()
        except IteratorNPE:
            end = it.consumer.next_epoch
        return "ok", out, remaining, eps, end

    def replay_full(self, start: int, ignore: int, max_buffers: int = 0):
        """A new iterator and its first `max_buffers` buffers: (status, buffers, remaining,
        epochs, end_epoch); status 'null' (no iterator) or 'state' (the constructor threw)."""
        try:
            it = self.get_in_flight_iterator(start, ignore)
        except IteratorNPE:
            return "state", [], 0, [], None
        if it is None:
            return "null", [], 0, [], None
        return self.take(it, max_buffers)

    def continue_full(self, max_buffers: int = 0):
        """The next buffers of the current iterator (CLG_IFL_CONTINUE)."""
        if self.current is None:
            return "state", [], 0, [], None
        return self.take(self.current, max_buffers)
