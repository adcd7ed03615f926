"""Host-side mirror of DeterminantResponseEvent and of the replay preparation done by the
recovery states, on top of the C-ABI (libclonos_engine.so).

  DeterminantResponseEvent  reference flink-runtime/.../causal/DeterminantResponseEvent.java:36-148
                            (write :93-107, read :109-125, merge :128-148) -> clg_response_*
  WaitingDeterminantsState  .../causal/recovery/WaitingDeterminantsState.java:57,97-108
                            (accumulator (found=true, vertex), merge every direct response)
  ReplayingState            .../causal/recovery/ReplayingState.java:58-214 and
  LogReplayerImpl           .../causal/recovery/LogReplayerImpl.java:51-158
                            -> clg_replay_prepare (main logs decoded on the GPU; subpartition
                               recovery buffers turned into BufferBuilt size lists on the GPU)

The event's map keeps java.util.HashMap iteration order (see include/clonos_engine.h), so
write() produces the reference's bytes.  Entries reference Python-owned byte buffers that
this object keeps alive.
"""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass
from typing import Dict, List, Optional, Sequence, Tuple

import time

import numpy as np

from . import _lib
from ._lib import check, lib
from .engine import CausalLogID, DecodedBatch, Engine, _np_ptr


# numpy views of the C structs (include/clonos_engine.h)
LOG_ID = np.dtype([("vertex_id", "<i2"), ("is_main", "u1"), ("subpartition", "i1"), ("reserved", "<u4"),
                   ("irp_lower", "<i8"), ("irp_upper", "<i8")])
ENTRY = np.dtype([("id", LOG_ID), ("bytes", "<u8"), ("len", "<u8")])
assert LOG_ID.itemsize == C.sizeof(_lib.CausalLogIdC) and ENTRY.itemsize == C.sizeof(_lib.ResponseEntry)


def log_id_array(ids: Sequence[CausalLogID]) -> np.ndarray:
    """CausalLogIDs as a packed clg_causal_log_id array."""
    a = np.zeros(len(ids), LOG_ID)
    for i, c in enumerate(ids):
        a[i] = (c.vertex_id, 1 if c.is_main else 0, 0 if c.is_main else c.subpartition, 0,
                0 if c.is_main else c.irp_lower, 0 if c.is_main else c.irp_upper)
    return a


def table_ids(table) -> np.ndarray:
    """The job's log table (job.LogTable) as a clg_causal_log_id array, built once per table."""
    arr = getattr(table, "_c_ids", None)
    if arr is None:
        arr = log_id_array(table.ids)
        table._c_ids = arr
    return arr


def _from_c(c: _lib.CausalLogIdC) -> CausalLogID:
    if c.is_main:
        return CausalLogID.main(c.vertex_id)
    return CausalLogID.sub(c.vertex_id, c.irp_lower, c.irp_upper, c.subpartition)


def causal_log_id_hash(lid: CausalLogID) -> int:
    """CausalLogID.hashCode (CausalLogID.java:151-163)."""
    c = lid.to_c()
    return lib.clg_causal_log_id_hash(C.byref(c))


class DeterminantResponseEvent:
    """DeterminantResponseEvent (found, vertexID, correlationID, Map<CausalLogID, ByteBuf>)."""

    def __init__(self, found: bool = False, vertex_id: int = 0, correlation_id: int = 0, capacity: int = 256):
        self._entries = (_lib.ResponseEntry * max(1, capacity))()
        self._c = _lib.Response(1 if found else 0, vertex_id, 0, correlation_id, 0, capacity, 0, 0, self._entries)
        self._keep: List[object] = []  # buffers the entries point into
        self._bytes: Optional[Tuple[int, int]] = None  # (main log bytes, all bytes) when known (merged_responses)

    # ---- accessors (:71-89)
    def isFound(self) -> bool:
        return bool(self._c.found)

    def getVertexID(self) -> int:
        return int(self._c.vertex_id)

    def getCorrelationID(self) -> int:
        return int(self._c.correlation_id)

    def setCorrelationID(self, v: int) -> None:
        self._c.correlation_id = v

    def getDeterminants(self) -> Dict[CausalLogID, bytes]:
        """The map, in java.util.HashMap iteration order."""
        out = {}
        for i in range(self._c.n):
            e = self._entries[i]
            out[_from_c(e.id)] = C.string_at(e.bytes, e.len) if e.len else b""
        return out

    def __len__(self) -> int:
        return int(self._c.n)

    def _grow(self, need: int) -> None:
        if need <= self._c.cap:
            return
        cap = max(need, 2 * self._c.cap)
        new = (_lib.ResponseEntry * cap)()
        C.memmove(new, self._entries, C.sizeof(_lib.ResponseEntry) * self._c.n)
        self._entries, self._c.entries, self._c.cap = new, new, cap

    # ---- map building (JobCausalLogImpl.respondToDeterminantRequest :197-199)
    def put(self, lid: CausalLogID, data: bytes) -> None:
        self._bytes = None
        buf = np.frombuffer(bytes(data), np.uint8) if len(data) else np.zeros(1, np.uint8)
        self._keep.append(buf)
        self._grow(self._c.n + 1)
        c = lid.to_c()
        check(lib.clg_response_put(C.byref(self._c), C.byref(c), _np_ptr(buf), len(data)))

    def put_device(self, lid: CausalLogID, ptr: int, n: int, keep=None) -> None:
        """An entry whose bytes live in device memory (replay-prep over a cross-GPU merge's
        receive buffer, clg_replay_prepare_device); `keep` is held while the event lives."""
        self._bytes = None
        if keep is not None:
            self._keep.append(keep)
        self._grow(self._c.n + 1)
        c = lid.to_c()
        check(lib.clg_response_put(C.byref(self._c), C.byref(c), C.c_void_p(ptr), n))

    def put_device_batch(self, ids: np.ndarray, ptrs: np.ndarray, lens: np.ndarray, keep=None) -> None:
        """Many device-memory entries in one call (clg_response_put_batch); ids: LOG_ID array."""
        if keep is not None:
            self._keep.append(keep)
        self._bytes = None
        n = len(ids)
        self._grow(self._c.n + n)
        ids = np.ascontiguousarray(ids, LOG_ID)
        ptrs = np.ascontiguousarray(ptrs, np.uint64)
        lens = np.ascontiguousarray(lens, np.uint64)
        self._keep.extend((ids, ptrs, lens))
        check(lib.clg_response_put_batch(C.byref(self._c), ids.ctypes.data, ptrs.ctypes.data, lens.ctypes.data, n))

    def entries(self) -> np.ndarray:
        """The map's entries as an ENTRY array view (iteration order)."""
        if not self._c.n:
            return np.zeros(0, ENTRY)
        return np.frombuffer((C.c_char * (ENTRY.itemsize * self._c.n)).from_address(C.addressof(self._entries)),
                             ENTRY, self._c.n)

    # ---- wire format
    def write(self) -> bytes:
        n = C.c_uint64()
        st = lib.clg_response_write(C.byref(self._c), None, 0, C.byref(n))
        if st not in (_lib.CLG_OK, _lib.CLG_E_CAPACITY):
            check(st)
        out = np.empty(max(1, n.value), np.uint8)
        check(lib.clg_response_write(C.byref(self._c), _np_ptr(out), n.value, C.byref(n)))
        return out[:n.value].tobytes()

    @staticmethod
    def read(data: bytes) -> Tuple["DeterminantResponseEvent", int]:
        buf = np.frombuffer(bytes(data), np.uint8) if len(data) else np.zeros(0, np.uint8)
        ev = DeterminantResponseEvent(capacity=max(1, len(data) // 7 + 1))
        ev._keep.append(buf)
        used = C.c_uint64()
        check(lib.clg_response_read(_np_ptr(buf) if buf.size else None, len(data), C.byref(ev._c), C.byref(used)))
        return ev, int(used.value)

    def merge(self, other: "DeterminantResponseEvent") -> None:
        self._bytes = None
        self._grow(self._c.n + other._c.n)
        self._keep.extend(other._keep)
        check(lib.clg_response_merge(C.byref(self._c), C.byref(other._c)))


def accumulate(vertex_id: int, responses: Sequence[DeterminantResponseEvent]) -> DeterminantResponseEvent:
    """WaitingDeterminantsState: new DeterminantResponseEvent(true, vertex) (:57), then merge
    every direct response in arrival order (:102)."""
    acc = DeterminantResponseEvent(True, vertex_id)
    for r in responses:
        acc.merge(r)
    return acc


@dataclass
class SubpartitionReplay:
    """What SubpartitionRecoveryThread.run (ReplayingState.java:157-214) would rebuild."""
    log_id: CausalLogID
    buffer_sizes: np.ndarray  # buildAndLogBuffer(n) arguments, in order
    status: int               # CLG_OK or the error the thread hits after those buffers
    err_off: int
    err_tag: int


@dataclass
class VertexReplay:
    vertex_id: int
    main: DecodedBatch          # LogReplayerImpl's record sequence (span 0 of this batch view)
    main_slice: slice
    subpartitions: List[SubpartitionReplay]


def merged_responses(merged, table, vertices: Sequence[int]) -> Dict[int, DeterminantResponseEvent]:
    """The accumulated responses of failed vertices whose copies arrived by the cross-GPU merge
    (dist.merge_responses): entries point into the merge's receive buffer, in HBM under RCCL
    (prepare_replay(..., device_input=True)).  One batched put per vertex."""
    gids = np.asarray(merged.gids, np.int64)
    ids = table_ids(table)
    # the entries grouped by vertex once (a stable sort keeps each vertex's entries in the
    # merge's order), then one contiguous slice per vertex
    vert = table.vertex[gids] if len(gids) else np.zeros(0, np.int64)
    order = np.argsort(vert, kind="stable")
    vs = vert[order]
    # (rows moved as raw words: fancy indexing the structured array took 0.13 ms for 2 k rows)
    ids_o = np.take(ids.view(np.uint64).reshape(len(ids), -1), gids[order], axis=0).view(LOG_ID).reshape(-1)
    ptr_o = np.ascontiguousarray(np.asarray(merged.offs, np.uint64)[order] + np.uint64(merged.buf.data_ptr()))
    len_o = np.ascontiguousarray(np.asarray(merged.lens, np.uint64)[order])
    out = {}
    va = np.asarray(list(vertices), np.int64)
    lo_a = np.searchsorted(vs, va, "left")
    hi_a = np.searchsorted(vs, va, "right")
    los, his = lo_a.tolist(), hi_a.tolist()
    # each vertex's byte totals, for prepare_replay_raw's output sizes (prefix sums, once)
    c_all = np.zeros(len(len_o) + 1, np.uint64)
    np.cumsum(len_o, out=c_all[1:])
    c_main = np.zeros(len(len_o) + 1, np.uint64)
    np.cumsum(np.where(ids_o["is_main"] != 0, len_o, np.uint64(0)), out=c_main[1:])
    t_all = (c_all[hi_a] - c_all[lo_a]).tolist()
    t_main = (c_main[hi_a] - c_main[lo_a]).tolist()
    # one put per vertex into the three arrays above (pointer arithmetic, no per-vertex views)
    pi, pp, pl, isz = ids_o.ctypes.data, ptr_o.ctypes.data, len_o.ctypes.data, ids_o.itemsize
    keep = (merged.buf, ids_o, ptr_o, len_o)
    for v, lo, hi, tm, ta in zip(va.tolist(), los, his, t_main, t_all):
        ev = DeterminantResponseEvent(True, v, capacity=max(1, hi - lo))
        if hi > lo:
            ev._keep.append(keep)
            check(lib.clg_response_put_batch(C.byref(ev._c), pi + lo * isz, pp + lo * 8, pl + lo * 8, hi - lo))
        ev._bytes = (tm, ta)
        out[v] = ev
    return out


def merged_response(vertex_id: int, merged, table) -> DeterminantResponseEvent:
    """merged_responses for one vertex."""
    return merged_responses(merged, table, [vertex_id])[vertex_id]


@dataclass
class ReplayArrays:
    """clg_replay_prepare's outputs as arrays (prepare_replay_raw): per subpartition (global
    order: vertex order, then table order) its size list is sizes[base[j] : base[j] + count[j]]."""
    main: DecodedBatch
    sizes: np.ndarray
    base: np.ndarray
    count: np.ndarray
    status: np.ndarray
    err_off: np.ndarray
    err_tag: np.ndarray


def prepare_replay_raw(engine: Engine, jobs: Sequence[Tuple[int, DeterminantResponseEvent, np.ndarray]],
                       device_input: bool = False, timing: Optional[Dict[str, float]] = None) -> ReplayArrays:
    """clg_replay_prepare over jobs (vertex_id, merged response, subpartition table as a
    LOG_ID array in the task's order), without per-subpartition Python objects.  timing:
    (developer) seconds added per part -- build, alloc, call, finish."""
    t0 = time.perf_counter()
    n = len(jobs)
    vs = (_lib.ReplayVertex * max(1, n))()
    tables = []
    main_bytes, sub_bytes, n_sub = 0, 0, 0
    for i, (vid, acc, subs) in enumerate(jobs):
        t = np.ascontiguousarray(subs, LOG_ID)
        tables.append(t)
        n_sub += len(t)
        vs[i] = _lib.ReplayVertex(C.pointer(acc._c), C.cast(t.ctypes.data, C.POINTER(_lib.CausalLogIdC)), len(t), vid, 0)
        if acc._bytes is not None:
            mb, ab = acc._bytes
        else:
            e = acc.entries()
            ln = e["len"]
            mb, ab = int(ln[e["id"]["is_main"] != 0].sum()), int(ln.sum())
        main_bytes += mb
        sub_bytes += ab - mb  # a bound: the table may name fewer
    t1 = time.perf_counter()
    cap = main_bytes // 2 + n + 1
    d, arrs, _ = engine._pooled_outputs(cap, main_bytes // 6 + n + 1)
    base = np.zeros(n + 1, np.uint64)
    sizes = np.empty(max(1, sub_bytes // 5), np.int32)
    sbase = np.zeros(n_sub + 1, np.uint64)
    cnt = np.zeros(max(1, n_sub), np.uint64)
    sst = np.zeros(max(1, n_sub), np.int32)
    soff = np.zeros(max(1, n_sub), np.int64)
    stag = np.zeros(max(1, n_sub), np.int32)
    out = _lib.ReplayOut(C.pointer(d), _np_ptr(base), _np_ptr(sizes), sizes.size, _np_ptr(sbase), _np_ptr(cnt),
                         _np_ptr(sst), _np_ptr(soff), _np_ptr(stag))
    fn = lib.clg_replay_prepare_device if device_input else lib.clg_replay_prepare
    t2 = time.perf_counter()
    st = fn(engine.handle, vs, n, C.byref(out))
    t3 = time.perf_counter()
    main = engine._finish(st, d, arrs, base, n, None)
    res = ReplayArrays(main, sizes, sbase[:n_sub], cnt[:n_sub], sst[:n_sub], soff[:n_sub], stag[:n_sub])
    if timing is not None:
        for k, v in (("build", t1 - t0), ("alloc", t2 - t1), ("call", t3 - t2), ("finish", time.perf_counter() - t3)):
            timing[k] = timing.get(k, 0.0) + v
    return res


def prepare_replay(engine: Engine, jobs: Sequence[Tuple[int, DeterminantResponseEvent, Sequence[CausalLogID]]],
                   device_input: bool = False) -> Tuple[DecodedBatch, List[VertexReplay]]:
    """ReplayingState construction for a batch of failed vertices: jobs are
    (vertex_id, merged response, subpartition table in the task's order).  device_input:
    the responses' bytes are in device memory (clg_replay_prepare_device)."""
    n = len(jobs)
    vs = (_lib.ReplayVertex * max(1, n))()
    tables = []
    main_bytes, sub_bytes = 0, 0
    for i, (vid, acc, subs) in enumerate(jobs):
        t = (_lib.CausalLogIdC * max(1, len(subs)))(*[s.to_c() for s in subs])
        tables.append(t)
        vs[i] = _lib.ReplayVertex(C.pointer(acc._c), t, len(subs), vid, 0)
        sizes_of = {_from_c(acc._entries[k].id): int(acc._entries[k].len) for k in range(acc._c.n)}
        main_bytes += sizes_of.get(CausalLogID.main(vid), 0)
        sub_bytes += sum(sizes_of.get(CausalLogID.sub(vid, s.irp_lower, s.irp_upper, s.subpartition), 0)
                         for s in subs)
    n_sub = sum(len(j[2]) for j in jobs)
    cap = main_bytes // 2 + n + 1
    d, arrs, _ = engine._pooled_outputs(cap, main_bytes // 6 + n + 1)
    base = np.zeros(n + 1, np.uint64)
    sizes = np.empty(max(1, sub_bytes // 5), np.int32)
    sbase = np.zeros(n_sub + 1, np.uint64)
    cnt = np.zeros(max(1, n_sub), np.uint64)
    sst = np.zeros(max(1, n_sub), np.int32)
    soff = np.zeros(max(1, n_sub), np.int64)
    stag = np.zeros(max(1, n_sub), np.int32)
    out = _lib.ReplayOut(C.pointer(d), _np_ptr(base), _np_ptr(sizes), sizes.size, _np_ptr(sbase), _np_ptr(cnt),
                         _np_ptr(sst), _np_ptr(soff), _np_ptr(stag))
    fn = lib.clg_replay_prepare_device if device_input else lib.clg_replay_prepare
    st = fn(engine.handle, vs, n, C.byref(out))
    main = engine._finish(st, d, arrs, base, n, None)
    res, j = [], 0
    for i, (vid, acc, subs) in enumerate(jobs):
        sp = []
        for s in subs:
            lid = CausalLogID.sub(vid, s.irp_lower, s.irp_upper, s.subpartition)
            b0 = int(sbase[j])
            sp.append(SubpartitionReplay(lid, sizes[b0:b0 + int(cnt[j])].copy(), int(sst[j]), int(soff[j]),
                                         int(stag[j])))
            j += 1
        res.append(VertexReplay(vid, main, main.span_slice(i), sp))
    return main, res
