"""In-flight (data) log on the engine: host-side mirror of the reference's InFlightLog.

Reference (I/ = flink-runtime/src/main/java/org/apache/flink/runtime/inflightlogging/):
  InFlightLog                          I/InFlightLog.java:32-55
  InMemorySubpartitionInFlightLogger   I/InMemorySubpartitionInFlightLogger.java:28-207
    log(buffer, epochID, isFinished)   :44-48
    notifyCheckpointComplete(cp)       :51-70
    getInFlightIterator(epoch, ignore) :73-82   (ReplayIterator :107-201)
    close()                            :90-94
  SpillableSubpartitionInFlightLogger  I/SpillableSubpartitionInFlightLogger.java:45-341 (the
                                       default, I/InFlightLogConfig.java:44; spill files not modelled)
    log                                :84-103  (a buffer logged while replaying reaches the live
                                                 iterator, I/SpilledReplayIterator.java:262-277)
    getInFlightIterator                :126-142 (tailMap(epoch); null when empty;
                                                 SpilledReplayIterator :60-401)

The buffers live in HBM (the engine's segment pool); replays of many subpartitions are one
batched gather on the GPU (clg_ifl_replay_batch).  The Java refcount bookkeeping
(retainBuffer / recycleBuffer) stays on the Java side: the engine owns the bytes until the
epoch is truncated or the log is closed.
"""
from __future__ import annotations

import ctypes as C
from typing import List, Optional, Sequence, Tuple

import numpy as np

from . import _lib
from ._lib import ClonosError, check, lib


class InFlightReplay:
    """Result of one replay request: the buffers getInFlightIterator(start, ignore) yields.

    `status` is CLG_OK, CLG_E_EPOCH_GAP (the reference's iterator throws after the buffers
    listed here) or a request error.  `remaining` is numberRemaining() right after the skip.
    `epochs[i]` is getEpoch() right before the next() that returns buffers[i] (the epoch
    PipelinedSubpartition.getReplayedBufferUnsafe :306-320 stamps on it); `end_epoch` is
    getEpoch() once the last buffer was taken."""

    def __init__(self, status: int, buffers: List[bytes], remaining: int, epochs: Optional[List[int]] = None,
                 end_epoch: int = 0, flags: int = 0):
        self.status = status
        self.buffers = buffers
        self.remaining = remaining
        self.epochs = list(epochs) if epochs is not None else []
        self.end_epoch = end_epoch
        self.flags = flags  # CLG_IFL_NULL_ITERATOR | CLG_IFL_REPLAYING (spillable)

    @property
    def null_iterator(self) -> bool:
        return bool(self.flags & _lib.CLG_IFL_NULL_ITERATOR)


class InFlightLogIterator:
    """ReplayIterator (:107-201) over a replay already gathered from HBM: next / hasNext /
    peekNext / numberRemaining / getEpoch; raises where the reference's iterator throws (an
    epoch gap)."""

    def __init__(self, rep: InFlightReplay, start_epoch: int):
        self._rep = rep
        self._i = 0
        self._left = rep.remaining
        self._start = start_epoch

    def has_next(self) -> bool:
        # at a gap the reference still sees the last buffer before it (:146-149) ...
        return self._i < len(self._rep.buffers) or self._rep.status == _lib.CLG_E_EPOCH_GAP

    def next(self) -> bytes:
        if self._i >= len(self._rep.buffers):
            if self._rep.status == _lib.CLG_E_EPOCH_GAP:  # ... and next() throws taking it (:156 -> :133)
                raise ClonosError(_lib.CLG_E_EPOCH_GAP, "in-flight log epoch gap (ReplayIterator :133)")
            raise StopIteration
        b = self._rep.buffers[self._i]
        self._i += 1
        self._left -= 1
        return b

    def peek_next(self) -> bytes:
        if self._i >= len(self._rep.buffers):
            raise StopIteration
        return self._rep.buffers[self._i]

    def number_remaining(self) -> int:
        return self._left

    def get_epoch(self) -> int:  # :181-183 currentKey
        if self._i < len(self._rep.epochs):
            return self._rep.epochs[self._i]
        return self._rep.end_epoch

    def __iter__(self):  # raises ClonosError at an epoch gap, like draining the reference's iterator
        while self.has_next():
            yield self.next()


class LiveInFlightLogIterator:
    """The spillable logger's SpilledReplayIterator (:60-401) over the engine's current iterator:
    `chunk` buffers per engine call, each exhausted chunk continued (CLG_IFL_CONTINUE) so that
    buffers logged meanwhile are delivered too (notifyNewBufferAdded :262-277)."""

    def __init__(self, log: "InFlightLog", first: InFlightReplay, chunk: int):
        self._log, self._chunk = log, chunk
        self._rep, self._i = first, 0
        self._left = first.remaining

    def _refill(self):
        if self._i < len(self._rep.buffers) or self._rep.status != _lib.CLG_OK:
            return
        rep = replay_batch(self._log.engine, [(self._log, 0, 0, self._chunk, _lib.CLG_IFL_CONTINUE)])[0]
        if rep.status not in (_lib.CLG_OK, _lib.CLG_E_EPOCH_GAP):
            check(rep.status)
        self._rep, self._i, self._left = rep, 0, rep.remaining

    def has_next(self) -> bool:  # consumerCursor.hasNext()
        self._refill()
        return self._i < len(self._rep.buffers) or self._rep.status == _lib.CLG_E_EPOCH_GAP

    def next(self) -> bytes:
        self._refill()
        if self._i >= len(self._rep.buffers):
            if self._rep.status == _lib.CLG_E_EPOCH_GAP:  # EpochCursor: log.get(epoch) == null
                raise ClonosError(_lib.CLG_E_EPOCH_GAP, "in-flight log epoch gap (SpilledReplayIterator)")
            raise StopIteration
        b = self._rep.buffers[self._i]
        self._i += 1
        self._left -= 1
        return b

    def number_remaining(self) -> int:
        return self._left

    def get_epoch(self) -> int:  # consumerCursor.getNextEpoch() :166-168
        self._refill()
        if self._i < len(self._rep.epochs):
            return self._rep.epochs[self._i]
        return self._rep.end_epoch

    def __iter__(self):
        while self.has_next():
            yield self.next()


class InFlightLog:
    """InMemorySubpartitionInFlightLogger (kind "in_memory") or SpillableSubpartitionInFlightLogger
    (kind "spillable", the reference's default) over the engine's HBM pool."""

    KINDS = {"in_memory": _lib.CLG_IFL_IN_MEMORY, "spillable": _lib.CLG_IFL_SPILLABLE}

    def __init__(self, engine, kind: str = "in_memory"):
        if kind not in self.KINDS:
            raise ValueError(f"kind must be one of {sorted(self.KINDS)}")
        self.engine = engine
        self.kind = kind
        h = C.c_uint32()
        check(lib.clg_ifl_open_typed(engine.handle, self.KINDS[kind], C.byref(h)))
        self.handle = h.value

    def log(self, buffer: bytes, epoch_id: int, is_finished: bool = True) -> None:  # :44-48
        log_batch(self.engine, [(self, epoch_id, buffer)])

    def notify_checkpoint_complete(self, checkpoint_id: int) -> None:  # :51-70
        check(lib.clg_ifl_notify_checkpoint_complete(self.engine.handle, self.handle, checkpoint_id))

    def epochs(self) -> List[Tuple[int, int]]:
        """[(epochID, buffers)] ascending (the slicedLog map)."""
        n = C.c_uint32()
        check(lib.clg_ifl_state(self.engine.handle, self.handle, None, None, 0, C.byref(n)))
        ids = np.zeros(max(n.value, 1), np.int64)
        cnt = np.zeros(max(n.value, 1), np.uint32)
        check(lib.clg_ifl_state(self.engine.handle, self.handle, ids.ctypes.data, cnt.ctypes.data, n.value,
                                C.byref(n)))
        return [(int(ids[i]), int(cnt[i])) for i in range(n.value)]

    def replay(self, start_epoch: int, ignore_buffers: int = 0, max_buffers: int = 0) -> InFlightReplay:
        return replay_batch(self.engine, [(self, start_epoch, ignore_buffers, max_buffers, 0)])[0]

    def replay_continue(self, max_buffers: int = 0) -> InFlightReplay:
        """Spillable: the next buffers of the current iterator (CLG_IFL_CONTINUE)."""
        return replay_batch(self.engine, [(self, 0, 0, max_buffers, _lib.CLG_IFL_CONTINUE)])[0]

    def get_in_flight_iterator(self, epoch_id: int, ignore_buffers: int = 0, chunk: int = 64):
        """in-memory :73-82 (the drained ReplayIterator); spillable :126-142 (None when tailMap(epoch)
        is empty, else a live iterator taking `chunk` buffers per engine call)."""
        spill = self.kind == "spillable"
        rep = self.replay(epoch_id, ignore_buffers, chunk if spill else 0)
        if rep.status not in (_lib.CLG_OK, _lib.CLG_E_EPOCH_GAP):
            check(rep.status)  # CLG_E_STATE: the skip inside getInFlightIterator threw
        if spill:
            return None if rep.null_iterator else LiveInFlightLogIterator(self, rep, chunk)
        return InFlightLogIterator(rep, epoch_id)

    def close(self) -> None:  # :90-94 (a no-op once the engine itself is closed)
        if self.handle is not None and self.engine.handle:
            check(lib.clg_ifl_close(self.engine.handle, self.handle))
            self.handle = None


def log_batch(engine, items: Sequence[Tuple[InFlightLog, int, bytes]]) -> None:
    """log() for many (log, epoch, buffer) at once: one upload + one scatter kernel."""
    n = len(items)
    if n == 0:
        return
    h = np.array([it[0].handle for it in items], np.uint32)
    ep = np.array([it[1] for it in items], np.int64)
    lens = np.array([len(it[2]) for it in items], np.uint32)
    offs = np.zeros(n, np.uint64)
    if n > 1:
        offs[1:] = np.cumsum(lens[:-1], dtype=np.uint64)
    blob = np.frombuffer(b"".join(bytes(it[2]) for it in items) or b"\0", np.uint8)
    check(lib.clg_ifl_log_batch(engine.handle, h.ctypes.data, ep.ctypes.data, offs.ctypes.data, lens.ctypes.data,
                                n, blob.ctypes.data, _lib.CLG_MEM_HOST))


def make_requests(reqs: Sequence[Tuple]):
    """The C request array for (log, start_epoch, ignore_buffers[, max_buffers, flags]) tuples;
    build it once to replay the same subpartitions repeatedly."""
    creq = (_lib.IflReplayReq * max(len(reqs), 1))()
    for i, r in enumerate(reqs):
        f, start, ign = r[:3]
        creq[i].ifl = f.handle
        creq[i].start_epoch = start
        creq[i].ignore_buffers = ign
        if len(r) > 3:
            creq[i].max_buffers, creq[i].flags = r[3], r[4]
    return creq


def replay_batch_raw(engine, reqs: Sequence[Tuple[InFlightLog, int, int]], out=None, sizes=None, cap: int = 0,
                     epochs=None):
    """One batched replay.  Returns (status, res array, out, sizes, total, total_buffers);
    out / sizes are host numpy arrays unless given; an int `out` is a device pointer
    (hipMalloc on the engine's device) of `cap` bytes, written in place.  `epochs` (int64,
    sized like `sizes`) optionally receives each buffer's epoch."""
    creq = reqs if isinstance(reqs, C.Array) else make_requests(reqs)
    n = len(creq) if len(reqs) else 0
    cres = (_lib.IflReplayRes * max(n, 1))()
    total, nbuf = C.c_uint64(), C.c_uint64()
    if out is None or sizes is None:
        # sizing pass: capacity 0 reports the totals without gathering
        st = lib.clg_ifl_replay_batch(engine.handle, creq, n, cres, None, 0, _lib.CLG_MEM_HOST, None, None, 0,
                                      C.byref(total), C.byref(nbuf))
        if st not in (_lib.CLG_OK, _lib.CLG_E_CAPACITY):
            check(st)
    kind = _lib.CLG_MEM_HOST
    if out is None:
        out = np.zeros(max(total.value, 1), np.uint8)
        out_ptr, cap = out.ctypes.data, out.size
    elif isinstance(out, np.ndarray):
        out_ptr, cap = out.ctypes.data, out.nbytes
    else:  # device pointer
        out_ptr, kind = int(out), _lib.CLG_MEM_DEVICE
    if sizes is None:
        sizes = np.zeros(max(nbuf.value, 1), np.uint32)
    if epochs is not None:
        assert epochs.dtype == np.int64 and epochs.size >= sizes.size
    st = lib.clg_ifl_replay_batch(engine.handle, creq, n, cres, out_ptr, cap, kind, sizes.ctypes.data,
                                  epochs.ctypes.data if epochs is not None else None, sizes.size,
                                  C.byref(total), C.byref(nbuf))
    return st, cres, out, sizes, total.value, nbuf.value


def replay_batch(engine, reqs: Sequence[Tuple[InFlightLog, int, int]]) -> List[InFlightReplay]:
    """getInFlightIterator + drain for many subpartitions: one gather kernel for all of them."""
    creq = make_requests(reqs)
    n = len(reqs)
    cres = (_lib.IflReplayRes * max(n, 1))()
    total, nbuf = C.c_uint64(), C.c_uint64()
    st = lib.clg_ifl_replay_batch(engine.handle, creq, n, cres, None, 0, _lib.CLG_MEM_HOST, None, None, 0,
                                  C.byref(total), C.byref(nbuf))
    if st not in (_lib.CLG_OK, _lib.CLG_E_CAPACITY):
        check(st)
    epochs = np.zeros(max(nbuf.value, 1), np.int64)
    st, cres, out, sizes, _, _ = replay_batch_raw(engine, creq if n else [], sizes=np.zeros(max(nbuf.value, 1),
                                                  np.uint32), out=np.zeros(max(total.value, 1), np.uint8),
                                                  epochs=epochs)
    check(st)
    reps = []
    for i in range(n):
        r = cres[i]
        bufs, o = [], r.out_off
        for k in range(r.n_buffers):
            sz = int(sizes[r.sizes_off + k])
            bufs.append(out[o:o + sz].tobytes())
            o += sz
        eps = [int(x) for x in epochs[r.sizes_off:r.sizes_off + r.n_buffers]]
        reps.append(InFlightReplay(r.status, bufs, r.remaining, eps, int(r.end_epoch), int(r.flags)))
    return reps
