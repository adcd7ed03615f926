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
