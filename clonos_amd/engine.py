"""Host-side mirror of Clonos' ThreadCausalLog / DeterminantEncoder (decode) on top of the
C-ABI of libclonos_engine.so.

Method names follow the reference Java interfaces so parity tests read like the
reference's own code:
  ThreadCausalLog  reference flink-runtime/.../causal/log/thread/ThreadCausalLog.java:33-96
  JobCausalLog     reference flink-runtime/.../causal/log/job/JobCausalLog.java:50-78 (see job.py)
Errors surface as ClonosError carrying the C status (the Java side throws the matching
exception: CorruptDeterminantArrayException, RuntimeException("Consumer went backwards"), ...).
"""
from __future__ import annotations

import collections
import ctypes as C
import mmap
import sys
import threading
from dataclasses import dataclass
from typing import Iterable, List, Optional, Sequence, Tuple, Union

import numpy as np

from . import _lib
from ._lib import ClonosError, check, lib
from . import determinants as D

ChannelLike = Union[Tuple[int, int], int]


def _ch(c: ChannelLike) -> _lib.ChannelId:
    if isinstance(c, tuple):
        return _lib.ChannelId(c[0] & 0xFFFFFFFFFFFFFFFF, c[1] & 0xFFFFFFFFFFFFFFFF)
    return _lib.ChannelId(int(c) & 0xFFFFFFFFFFFFFFFF, 0)


@dataclass(frozen=True)
class CausalLogID:
    """CausalLogID.java:38-198: main-thread log or (partition, subpartition) log of a vertex."""
    vertex_id: int
    is_main: bool = True
    irp_lower: int = 0
    irp_upper: int = 0
    subpartition: int = 0

    @staticmethod
    def main(vertex_id: int) -> "CausalLogID":
        return CausalLogID(vertex_id, True)

    @staticmethod
    def sub(vertex_id: int, lower: int, upper: int, index: int) -> "CausalLogID":
        return CausalLogID(vertex_id, False, lower, upper, index)

    def key(self):
        """equals/hashCode semantics (:128-163): main logs compare by vertex only."""
        return (self.vertex_id, True) if self.is_main else (self.vertex_id, False, self.irp_lower, self.irp_upper,
                                                            self.subpartition)

    def to_c(self) -> _lib.CausalLogIdC:
        return _lib.CausalLogIdC(self.vertex_id, 1 if self.is_main else 0, 0 if self.is_main else self.subpartition, 0,
                                 0 if self.is_main else self.irp_lower, 0 if self.is_main else self.irp_upper)

    def is_for_vertex(self, v: int) -> bool:
        return self.vertex_id == v


class DecodedBatch:
    """Dense SoA produced by the GPU decode (layout: include/clonos_engine.h clg_decoded)."""

    def __init__(self, off, tag, v0, w_idx, w_rc, w_v1, w_var_off, w_var_len, w_sub, span_rec_base, spans_bytes=None):
        self.off, self.tag, self.v0 = off, tag, v0
        self.w_idx, self.w_rc, self.w_v1 = w_idx, w_rc, w_v1
        self.w_var_off, self.w_var_len, self.w_sub = w_var_off, w_var_len, w_sub
        self.span_rec_base = span_rec_base
        self.spans_bytes = spans_bytes  # optional: the raw span bytes, to materialise var fields

    @property
    def n_rec(self) -> int:
        return int(self.tag.shape[0])

    def span_slice(self, s: int) -> slice:
        return slice(int(self.span_rec_base[s]), int(self.span_rec_base[s + 1]))

    def determinants(self, s: int) -> List[D.Determinant]:
        """Rebuild Determinant objects for span s (LogReplayer consumption order)."""
        raw = self.spans_bytes[s] if self.spans_bytes is not None else None
        sl = self.span_slice(s)
        widx = {int(i): k for k, i in enumerate(self.w_idx)}
        out: List[D.Determinant] = []
        for i in range(sl.start, sl.stop):
            t = int(self.tag[i])
            v0 = int(self.v0[i])
            if t == D.ORDER:
                out.append(D.OrderDeterminant(v0))
            elif t == D.TIMESTAMP:
                out.append(D.TimestampDeterminant(v0))
            elif t == D.RNG:
                out.append(D.RNGDeterminant(v0))
            elif t == D.BUFFER_BUILT:
                out.append(D.BufferBuiltDeterminant(v0))
            else:
                k = widx[i]
                rc, v1, vo, vl, sub = (int(self.w_rc[k]), int(self.w_v1[k]), int(self.w_var_off[k]),
                                       int(self.w_var_len[k]), int(self.w_sub[k]))
                var = bytes(raw[vo:vo + vl]) if raw is not None and vo else None
                if t == D.IGNORE_CHECKPOINT:
                    out.append(D.IgnoreCheckpointDeterminant(rc, v0))
                elif t == D.TIMER_TRIGGER:
                    out.append(D.TimerTriggerDeterminant(rc, v0, sub, var if sub == D.INTERNAL else None))
                elif t == D.SOURCE_CHECKPOINT:
                    out.append(D.SourceCheckpointDeterminant(rc, v0, v1, sub & 0x7F, var if sub & 0x80 else None))
                elif t == D.SERIALIZABLE:
                    out.append(D.SerializableDeterminant(var if var is not None else b""))
        return out


def _np_ptr(a: np.ndarray) -> int:
    return a.ctypes.data if a.size else 0


class Engine:
    """One engine per GPU (one process per GPU).  Owns the HBM segment pool."""

    def __init__(self, segment_bytes: int = 16384, pool_segments: int = 16384, device: int = 0,
                 sharing_depth: int = _lib.CLG_FULL_SHARING, timing: bool = False, decode: str = "auto",
                 async_slice: bool = False, ifl_segment_bytes: Optional[int] = None,
                 ifl_pool_segments: Optional[int] = None, host_tail_bytes: Optional[int] = None):
        """decode: "auto" = single-launch decode for small batches, else the fast three-pass
        decode, robust multi-pass pipeline on abort; "three_pass" = no single-launch path
        (CLG_F_NO_SMALL_DECODE); "robust" = the robust pipeline only (CLG_F_ROBUST_DECODE).  async_slice: device-output
        slices return once queued on the gather stream (CLG_F_ASYNC_SLICE); sync() before
        reading them.  ifl_*: the in-flight log's own pool (default: the same geometry as the
        determinant pool)."""
        if decode not in ("auto", "three_pass", "robust"):
            raise ValueError(f"decode must be 'auto', 'three_pass' or 'robust', not {decode!r}")
        cfg = _lib.Config()
        lib.clg_config_default(C.byref(cfg))
        cfg.segment_bytes = segment_bytes
        cfg.pool_segments = pool_segments
        cfg.device = device
        cfg.sharing_depth = sharing_depth
        if host_tail_bytes is not None:
            cfg.host_tail_bytes = host_tail_bytes
        cfg.ifl_segment_bytes = ifl_segment_bytes if ifl_segment_bytes is not None else segment_bytes
        cfg.ifl_pool_segments = ifl_pool_segments if ifl_pool_segments is not None else pool_segments
        cfg.flags = ((_lib.CLG_F_TIMING if timing else 0) | (_lib.CLG_F_ROBUST_DECODE if decode == "robust" else 0)
                     | (_lib.CLG_F_NO_SMALL_DECODE if decode == "three_pass" else 0)
                     | (_lib.CLG_F_ASYNC_SLICE if async_slice else 0))
        h = C.c_void_p()
        check(lib.clg_engine_create(C.byref(cfg), C.byref(h)))
        self._h = h
        self._out_slots: List[dict] = []  # _pooled_outputs
        self._in_sc = None  # _in_scratch
        self._in_mu = threading.Lock()  # its user
        self._pool_mu = threading.Lock()  # slot picks (a picked slot is busy until _finish)
        self.segment_bytes = segment_bytes
        self.sharing_depth = sharing_depth
        self.async_slice = async_slice
        self.device = device
        self._logs = {}
        self._queued = collections.deque()  # queued asynchronous decodes, oldest first (clg_decode_wait is FIFO)

    # ---- lifecycle ----------------------------------------------------------------
    def close(self):
        if self._h:
            self._out_release()
            lib.clg_engine_destroy(self._h)
            self._h = None

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    @property
    def handle(self):
        return self._h

    @property
    def stream(self) -> int:
        return lib.clg_engine_stream(self._h) or 0

    def sync(self):
        check(lib.clg_sync(self._h))

    def pool_stats(self) -> Tuple[int, int]:
        u, f = C.c_uint32(), C.c_uint32()
        check(lib.clg_pool_stats(self._h, C.byref(u), C.byref(f)))
        return u.value, f.value

    def ifl_pool_stats(self) -> Tuple[int, int]:
        u, f = C.c_uint32(), C.c_uint32()
        check(lib.clg_ifl_pool_stats(self._h, C.byref(u), C.byref(f)))
        return u.value, f.value

    # ---- jobs (JobCausalLogImpl scope) ----------------------------------------------------
    def open_job(self, job_id: Tuple[int, int], sharing_depth: int = _lib.CLG_FULL_SHARING) -> int:
        """A further JobCausalLog on this engine (job 0 is the engine's default job): its own
        logs, sharing depth and latestCompletedCheckpoint CAS."""
        j = C.c_uint32()
        check(lib.clg_job_open(self._h, job_id[0], job_id[1], sharing_depth, C.byref(j)))
        return j.value

    def close_job(self, job: int) -> None:
        check(lib.clg_job_close(self._h, job))
        self._logs = {k: v for k, v in self._logs.items() if k[0] != job}

    # ---- logs -----------------------------------------------------------------------
    def open_log(self, cid: CausalLogID, job: int = 0) -> "ThreadCausalLog":
        h = C.c_uint32()
        check(lib.clg_log_open(self._h, job, C.byref(cid.to_c()), C.byref(h)))
        log = ThreadCausalLog(self, h.value, cid, job)
        self._logs[(job, cid.key())] = log
        return log

    def get_log(self, cid: CausalLogID, job: int = 0) -> Optional["ThreadCausalLog"]:
        """The open log for `cid` (also logs the engine opened itself, e.g. by processCausalLogDelta)."""
        log = self._logs.get((job, cid.key()))
        if log is None:
            h = C.c_uint32()
            if lib.clg_log_find(self._h, job, C.byref(cid.to_c()), C.byref(h)) == _lib.CLG_OK:
                log = self._logs[(job, cid.key())] = ThreadCausalLog(self, h.value, cid, job)
        return log

    def append_batch(self, logs: np.ndarray, epochs: np.ndarray, offs: np.ndarray, lens: np.ndarray,
                     data: np.ndarray):
        logs = np.ascontiguousarray(logs, np.uint32)
        epochs = np.ascontiguousarray(epochs, np.int64)
        offs = np.ascontiguousarray(offs, np.uint64)
        lens = np.ascontiguousarray(lens, np.uint32)
        data = np.ascontiguousarray(data, np.uint8)
        check(lib.clg_append_batch(self._h, _np_ptr(logs), _np_ptr(epochs), _np_ptr(offs), _np_ptr(lens),
                                   len(logs), _np_ptr(data)))

    # ---- batched slicing ----------------------------------------------------------------
    def slice_batch(self, reqs: Sequence[Tuple["ThreadCausalLog", ChannelLike, int]], out=None,
                    cap: Optional[int] = None):
        """Batched hasDelta/getOffset/getDelta.  `out`: None (host bytes returned), a numpy
        uint8 array, or a device pointer (int, CLG_MEM_DEVICE) with `cap`."""
        n = len(reqs)
        creq = (_lib.SliceReq * max(n, 1))()
        for i, (log, ch, ep) in enumerate(reqs):
            creq[i].log = log.handle
            creq[i].consumer = _ch(ch)
            creq[i].epoch = ep
        cres = (_lib.SliceRes * max(n, 1))()
        total = C.c_uint64()
        if out is None or isinstance(out, np.ndarray):
            if out is None:
                out = np.empty(cap if cap is not None else self._slice_bound(reqs), np.uint8)
            st = lib.clg_slice_batch(self._h, C.cast(creq, C.c_void_p), n, C.cast(cres, C.c_void_p), _np_ptr(out),
                                     out.size, _lib.CLG_MEM_HOST, C.byref(total))
        else:
            st = lib.clg_slice_batch(self._h, C.cast(creq, C.c_void_p), n, C.cast(cres, C.c_void_p), int(out),
                                     int(cap), _lib.CLG_MEM_DEVICE, C.byref(total))
        check(st)
        res = [(cres[i].status, bool(cres[i].has_delta), cres[i].offset_from_epoch, cres[i].len, cres[i].out_off)
               for i in range(n)]
        return res, out, total.value

    def _slice_bound(self, reqs) -> int:
        b = 0
        for log in {id(r[0]): r[0] for r in reqs}.values():
            b += log.state()["writer"] * sum(1 for r in reqs if r[0] is log)
        return max(b, 1)

    def slice_batch_raw(self, creq, cres, n: int, out_ptr: int, cap: int, device: bool = True) -> int:
        """Zero-overhead variant for benchmarks: prebuilt ctypes request/result arrays."""
        total = C.c_uint64()
        check(lib.clg_slice_batch(self._h, C.cast(creq, C.c_void_p), n, C.cast(cres, C.c_void_p), out_ptr, cap,
                                  _lib.CLG_MEM_DEVICE if device else _lib.CLG_MEM_HOST, C.byref(total)))
        return total.value

    def log_lengths(self, handles: np.ndarray) -> Tuple[np.ndarray, int]:
        """logLength of many logs in one call: (per-log lengths, sum)."""
        h = np.ascontiguousarray(handles, np.uint32)
        out = np.zeros(max(h.size, 1), np.int32)
        tot = C.c_uint64()
        check(lib.clg_log_length_batch(self._h, _np_ptr(h), h.size, _np_ptr(out), C.byref(tot)))
        return out[:h.size], tot.value

    def upstream_delta_batch(self, reqs, n: int, src_ptr: int, in_kind: int) -> None:
        """Batched processUpstreamDelta over one buffer (host or device pointer); each
        request's status is written back into `reqs` (clg_delta_req)."""
        check(lib.clg_upstream_delta_batch(self._h, C.cast(reqs, C.c_void_p), n, src_ptr, in_kind))

    def seek_consumers_raw(self, creq, offsets: np.ndarray, n: int) -> None:
        """Batched consumer positioning over a prebuilt ctypes request array."""
        offs = np.ascontiguousarray(offsets, dtype=np.int32)
        check(lib.clg_consumer_seek_batch(self._h, C.cast(creq, C.c_void_p), offs.ctypes.data, n))

    # ---- checkpoint completion ---------------------------------------------------------
    def truncate_all(self, checkpoint_id: int, job: int = 0) -> bool:
        """JobCausalLogImpl.notifyCheckpointComplete (:230-246) for `job`: CAS, then every log of it."""
        applied = C.c_int32()
        check(lib.clg_truncate_all(self._h, job, checkpoint_id, C.byref(applied)))
        return bool(applied.value)

    # ---- decode -------------------------------------------------------------------------
    # (name, dtype, itemsize, side table?) of clg_decoded's host arrays
    _OUT_FIELDS = (("off", np.uint32, 4, 0), ("tag", np.uint8, 1, 0), ("v0", np.int64, 8, 0), ("w_idx", np.uint32, 4, 1),
                   ("w_rc", np.int32, 4, 1), ("w_v1", np.int64, 8, 1), ("w_var_off", np.uint32, 4, 1),
                   ("w_var_len", np.uint32, 4, 1), ("w_sub", np.uint8, 1, 1))

    @staticmethod
    def _out_bytes(cap: int, wcap: int, bcap: int = 0) -> Tuple[List[int], int]:
        """Offsets of the nine arrays (16-byte aligned), then of span_rec_base (bcap entries)."""
        offs, at = [], 0
        for _, _, isz, wide in Engine._OUT_FIELDS:
            offs.append(at)
            at = (at + isz * (wcap if wide else cap) + 15) & ~15
        offs.append(at)
        return offs, at + 8 * bcap

    @staticmethod
    def _host_outputs(cap: int, wcap: int, buf: Optional[np.ndarray] = None, bcap: int = 0):
        """The SoA output arrays as views of one host buffer (one allocation, one pointer),
        and their clg_decoded.  buf: a buffer to carve them from (large enough), else a new one.
        bcap: also a span_rec_base array ("base") of that many entries."""
        offs, at = Engine._out_bytes(cap, wcap, bcap)
        if buf is None or buf.size < at:
            buf = np.empty(max(at, 16), np.uint8)
        b0 = buf.ctypes.data
        d = _lib.Decoded()
        arrs = {}
        for (k, dt, isz, wide), o in zip(Engine._OUT_FIELDS, offs):
            arrs[k] = buf[o:o + isz * (wcap if wide else cap)].view(dt)
            setattr(d, k, b0 + o)
        if bcap:
            arrs["base"] = buf[offs[-1]:offs[-1] + 8 * bcap].view(np.uint64)
        d.cap, d.wcap, d.out_kind = cap, wcap, _lib.CLG_MEM_HOST
        return d, arrs

    @staticmethod
    def _slot_capacity(size: int, cap: int, wcap: int, bcap: int) -> Tuple[int, int, int]:
        """The largest capacities in the proportions of (cap, wcap) -- and at least 256 span
        entries -- whose arrays fit a slot of `size` bytes; (cap, wcap, bcap) when they do not."""
        b = max(bcap, 256)
        k = (size - 8 * b - 160) / max(13 * cap + 25 * wcap, 1)  # 160: more than the padding
        if k < 1.0:
            return cap, wcap, bcap
        return int(cap * k), int(wcap * k), b

    _OUT_SLOTS = 3  # pooled output buffers (a caller usually keeps one batch while asking for the next)

    @staticmethod
    def _slot_free(sl) -> bool:
        # not between its pick and _finish, and references when free: the slot, getrefcount's
        # argument, and the cached views
        return not sl["busy"] and sys.getrefcount(sl["buf"]) <= 2 + (
            len(sl["cache"][2]) if sl["cache"] is not None else 0)

    def _slot_done(self, arrs) -> None:
        """The decode that picked the slot of `arrs` has made its result (or failed)."""
        for sl in self._out_slots:
            if sl["cache"] is not None and sl["cache"][2] is arrs:
                sl["busy"] = False

    def _slot_use(self, pick):
        """The slot becomes busy and the most recent (by identity: the slots hold arrays); its
        cached clg_decoded, views and byref, counts reset."""
        pick["busy"] = True
        if self._out_slots[-1] is not pick:
            self._out_slots = [sl for sl in self._out_slots if sl is not pick] + [pick]
        _, d, arrs, ref = pick["cache"]
        d.n_rec = d.n_wide = 0
        return d, arrs, ref

    def _pooled_outputs(self, cap: int, wcap: int, bcap: int = 0):
        """_host_outputs from one of the engine's reusable buffers that no earlier result still
        holds (every returned array is a view of its buffer, so a live batch keeps the buffer's
        reference count up): the pages stay mapped -- not faulted in on every call -- and
        registered for the device (clg_host_register), so the single-launch small decode writes
        the outputs straight into them (CLG_MEM_MAPPED).  The views are carved at the slot's
        whole capacity (_slot_capacity) and serve again for every request they cover.
        Returns (clg_decoded, arrays, byref(clg_decoded))."""
        with self._pool_mu:
            return self._pooled_pick(cap, wcap, bcap)

    def _pooled_pick(self, cap: int, wcap: int, bcap: int):
        need = self._out_bytes(cap, wcap, bcap)[1]
        pick = None
        for sl in self._out_slots:
            c = sl["cache"]
            if c is not None and c[0][0] >= cap and c[0][1] >= wcap and c[0][2] >= bcap and self._slot_free(sl):
                return self._slot_use(sl)
            if pick is None and sl["buf"].size >= need and self._slot_free(sl):
                pick = sl
        if pick is None:
            idle = [i for i, sl in enumerate(self._out_slots) if not sl["busy"]]
            if len(self._out_slots) >= self._OUT_SLOTS and idle:  # all held (or too small): the oldest
                self._slot_release(self._out_slots.pop(idle[0]))  # not being decoded into leaves the pool
            size = (max(need, 1 << 16) + 4095) & ~4095  # page-aligned: an anonymous mapping
            buf = np.frombuffer(mmap.mmap(-1, size), np.uint8)
            mapped = self._h is not None and lib.clg_host_register(_np_ptr(buf), size) == _lib.CLG_OK
            pick = {"buf": buf, "mapped": mapped, "cache": None, "busy": False}
            self._out_slots.append(pick)
        pick["cache"] = None  # (its views would hold the buffer)
        key = self._slot_capacity(pick["buf"].size, cap, wcap, bcap)
        d, arrs = self._host_outputs(*key[:2], pick["buf"], key[2])
        if pick["mapped"]:
            d.out_kind = _lib.CLG_MEM_MAPPED
        pick["cache"] = (key, d, arrs, C.byref(d))
        pick["bptr"] = arrs["base"].ctypes.data if "base" in arrs else 0
        return self._slot_use(pick)

    def _slot_release(self, sl):
        """A pooled buffer leaves the pool: unregistered (a batch the caller keeps stays valid as
        ordinary host memory)."""
        if sl["mapped"]:
            lib.clg_host_unregister(_np_ptr(sl["buf"]))
        sl["cache"] = None

    def _out_release(self):
        while self._out_slots:
            self._slot_release(self._out_slots.pop())

    @property
    def _out_buf(self):  # the most recently used pooled buffer (tests)
        return self._out_slots[-1]["buf"] if self._out_slots else None

    @property
    def _out_cache(self):
        return self._out_slots[-1]["cache"] if self._out_slots else None

    @property
    def _out_mapped(self):
        return bool(self._out_slots) and self._out_slots[-1]["mapped"]

    def _finish(self, st, d, arrs, base, n_spans, spans_bytes):
        """The batch as slices of the slot's views (they hold its buffer); the slot's pick ends."""
        try:
            if st != _lib.CLG_OK:
                err = _lib.ClonosError(st, lib.clg_last_error().decode(errors="replace"))
                err.err_span, err.err_off, err.err_tag = d.err_span, d.err_off, d.err_tag
                err.n_rec = d.n_rec
                raise err
            nr, nw = d.n_rec, d.n_wide
            return DecodedBatch(arrs["off"][:nr], arrs["tag"][:nr], arrs["v0"][:nr], arrs["w_idx"][:nw],
                                arrs["w_rc"][:nw], arrs["w_v1"][:nw], arrs["w_var_off"][:nw],
                                arrs["w_var_len"][:nw], arrs["w_sub"][:nw], base[:n_spans + 1], spans_bytes)
        finally:
            self._slot_done(arrs)

    def decode_host(self, data: Union[bytes, np.ndarray], spans: Optional[Sequence[Tuple[int, int]]] = None
                    ) -> DecodedBatch:
        """DeterminantEncoder.decodeNext over whole spans of host bytes, on the GPU."""
        buf = np.frombuffer(bytes(data), np.uint8) if not isinstance(data, np.ndarray) else np.ascontiguousarray(
            data, np.uint8)
        if spans is None:
            spans = [(0, buf.size)]
        so = np.array([s[0] for s in spans], np.uint64)
        sl = np.array([s[1] for s in spans], np.uint64)
        cap = int(sl.sum()) // 2 + len(spans) + 1
        wcap = int(sl.sum()) // 6 + len(spans) + 1
        d, arrs, ref = self._pooled_outputs(cap, wcap)
        base = np.zeros(len(spans) + 1, np.uint64)
        st = lib.clg_decode_host(self._h, _np_ptr(buf), _np_ptr(so), _np_ptr(sl), len(spans), ref, _np_ptr(base))
        return self._finish(st, d, arrs, base, len(spans),
                            [buf[int(o):int(o) + int(n)] for o, n in zip(so, sl)])

    def decode_logs(self, logs: Sequence["ThreadCausalLog"], start_epochs: Sequence[int],
                    keep_bytes: bool = False) -> DecodedBatch:
        n = len(logs)
        own = self._in_mu.acquire(blocking=False)  # the reused handle / epoch arrays, else new ones
        try:
            sc = self._in_scratch(n) if own else self._in_arrays(n)
            h, ep = sc[0][:n], sc[1][:n]
            h[:] = [l.handle for l in logs]
            ep[:] = start_epochs
            # a free registered slot whose capacity covers the batch decodes without logLength;
            # a batch beyond it fails with CLG_E_CAPACITY (nothing changed) and is sized below
            fast = self._pooled_fast(n)
            st = _lib.CLG_E_CAPACITY
            if fast is not None:
                d, arrs, ref, bptr = fast
                st = lib.clg_decode_logs(self._h, sc[2], sc[3], n, ref, bptr)
                if st == _lib.CLG_E_CAPACITY:
                    self._slot_done(arrs)
            if st == _lib.CLG_E_CAPACITY:
                total = self.log_lengths(h)[1]  # logLength bounds every span (one native call for the batch)
                d, arrs, ref = self._pooled_outputs(total // 2 + n + 1, total // 6 + n + 1, n + 1)
                st = lib.clg_decode_logs(self._h, sc[2], sc[3], n, ref, arrs["base"].ctypes.data)
        finally:
            if own:
                self._in_mu.release()
        sb = [np.frombuffer(l.getDeterminants(e), np.uint8) for l, e in zip(logs, start_epochs)] if keep_bytes else None
        return self._finish(st, d, arrs, arrs["base"], n, sb)

    def _in_scratch(self, n: int):
        """Reused handle / epoch arrays of decode_logs, with their addresses."""
        sc = self._in_sc
        if sc is None or sc[0].size < n:
            sc = self._in_sc = self._in_arrays(max(64, 1 << max(n - 1, 0).bit_length()))
        return sc

    @staticmethod
    def _in_arrays(n: int):
        h, ep = np.zeros(max(n, 1), np.uint32), np.zeros(max(n, 1), np.int64)
        return h, ep, h.ctypes.data, ep.ctypes.data

    def _pooled_fast(self, n_spans: int):
        """A free registered slot with a span_rec_base of n_spans + 1 entries (its views carved at
        its whole capacity), or None."""
        with self._pool_mu:
            for sl in self._out_slots:
                c = sl["cache"]
                if c is not None and sl["mapped"] and c[0][2] > n_spans and self._slot_free(sl):
                    return self._slot_use(sl) + (sl["bptr"],)
        return None

    def decode_logs_async(self, logs: Sequence["ThreadCausalLog"], start_epochs: Sequence[int]) -> "PendingDecode":
        """clg_decode_logs_async into host arrays: returns at once; .wait() gives the batch.
        Up to CLG_DECODE_MAX_INFLIGHT may be queued; their waits complete them in queue order
        (waiting for a later one first completes the earlier ones, whose results are kept)."""
        h = np.array([l.handle for l in logs], np.uint32)
        ep = np.array(start_epochs, np.int64)
        total = self.log_lengths(h)[1]
        d, arrs, ref = self._pooled_outputs(total // 2 + len(logs) + 1, total // 6 + len(logs) + 1)
        base = np.zeros(len(logs) + 1, np.uint64)
        pd = PendingDecode(self, (h, ep, d, arrs, base), len(logs))
        st = lib.clg_decode_logs_async(self._h, _np_ptr(h), _np_ptr(ep), len(logs), ref, _np_ptr(base))
        if st != _lib.CLG_OK:
            self._slot_done(arrs)
            check(st)
        self._queued.append(pd)
        return pd

    def decode_logs_device(self, handles: np.ndarray, start_epochs: np.ndarray, dec: _lib.Decoded,
                           base: np.ndarray) -> None:
        """Benchmark variant: outputs are caller-owned device arrays described by `dec`."""
        check(lib.clg_decode_logs(self._h, _np_ptr(handles), _np_ptr(start_epochs), len(handles), C.byref(dec),
                                  _np_ptr(base)))

    def decode_logs_device_async(self, handles: np.ndarray, start_epochs: np.ndarray, dec: _lib.Decoded,
                                 base: np.ndarray) -> None:
        """clg_decode_logs_async: queues the decode and returns; `dec`, `base` and the output
        arrays stay untouched by the caller until the decode_wait() that pairs with it (FIFO;
        up to CLG_DECODE_MAX_INFLIGHT queued, each with its own outputs)."""
        keep = (handles, start_epochs, dec, base)  # kept alive until the wait
        check(lib.clg_decode_logs_async(self._h, _np_ptr(handles), _np_ptr(start_epochs), len(handles),
                                        C.byref(dec), _np_ptr(base)))
        self._queued.append(keep)

    def decode_wait(self) -> None:
        """clg_decode_wait: completes the oldest queued asynchronous decode and raises its error."""
        if self._queued and isinstance(self._queued[0], PendingDecode):
            self._queued[0].wait()
            return
        st = lib.clg_decode_wait(self._h)
        if self._queued:
            self._queued.popleft()
        check(st)

    # ---- piggybacked deltas (AbstractDeltaSerializerDeserializer) ---------------------------
    def enrich_batch(self, strategy: int, reqs):
        """enrichWithCausalLogDelta for many channels.  reqs: [(channel, epoch, [(log, send), ...])]
        with the logs in the strategy's iteration order.  Returns [(status, header+deltas bytes)]."""
        logs, flags, creq = [], [], (_lib.EnrichReq * max(1, len(reqs)))()
        for i, (ch, ep, entries) in enumerate(reqs):
            creq[i].consumer, creq[i].epoch, creq[i].first, creq[i].count = _ch(ch), ep, len(logs), len(entries)
            for log, send in entries:
                logs.append(log.handle)
                flags.append(_lib.CLG_DE_SEND if send else 0)
        la, fa = np.array(logs or [0], np.uint32), np.array(flags or [0], np.uint8)
        total = C.c_uint64()
        st = lib.clg_enrich_batch(self._h, strategy, creq, len(reqs), _np_ptr(la), _np_ptr(fa), None, 0,
                                  _lib.CLG_MEM_HOST, C.byref(total))
        if st == _lib.CLG_E_CAPACITY or (st == _lib.CLG_OK and total.value):
            out = np.empty(max(1, total.value), np.uint8)
            check(lib.clg_enrich_batch(self._h, strategy, creq, len(reqs), _np_ptr(la), _np_ptr(fa), _np_ptr(out),
                                       out.size, _lib.CLG_MEM_HOST, C.byref(total)))
        else:
            check(st)
            out = np.zeros(0, np.uint8)
        return [(creq[i].status, out[creq[i].out_off:creq[i].out_off + creq[i].out_len].tobytes())
                for i in range(len(reqs))]

    def process_delta(self, strategy: int, msg: bytes, job: int = 0):
        """processCausalLogDelta: returns (epoch, logs touched in header order, bytes consumed)."""
        buf = np.frombuffer(bytes(msg), np.uint8)
        ep, nl, used = C.c_int64(), C.c_uint32(), C.c_uint64()
        hs = np.zeros(4096, np.uint32)
        check(lib.clg_process_delta(self._h, job, strategy, _np_ptr(buf), len(msg), _lib.CLG_MEM_HOST, C.byref(ep),
                                    _np_ptr(hs), hs.size, C.byref(nl), C.byref(used)))
        return ep.value, [int(h) for h in hs[:min(nl.value, hs.size)]], used.value

    # ---- encode -----------------------------------------------------------------------------
    def encode_batch(self, tag, v0, w_idx=None, w_rc=None, w_v1=None, w_var_off=None, w_var_len=None, w_sub=None,
                     var: bytes = b"") -> bytes:
        """SimpleDeterminantEncoder.encodeTo over a batch, on the GPU: records in the decode's
        SoA layout (the side-table arrays for wide records; w_var_off indexes `var`)."""
        tag = np.ascontiguousarray(tag, np.uint8)
        v0 = np.ascontiguousarray(v0, np.int64)
        nw = 0 if w_idx is None else len(w_idx)
        arr = lambda a, t: np.ascontiguousarray(a if a is not None else np.zeros(0), t)  # noqa: E731
        side = [arr(w_idx, np.uint32), arr(w_rc, np.int32), arr(w_v1, np.int64), arr(w_var_off, np.uint32),
                arr(w_var_len, np.uint32), arr(w_sub, np.uint8)]
        vb = np.frombuffer(bytes(var), np.uint8) if len(var) else np.zeros(1, np.uint8)
        ein = _lib.EncodeIn(_np_ptr(tag), _np_ptr(v0), len(tag), *[_np_ptr(a) for a in side[:6]], nw,
                            _np_ptr(vb), len(var), _lib.CLG_MEM_HOST, 0)
        n_out, bad = C.c_uint64(), C.c_uint64()
        st = lib.clg_encode_batch(self._h, C.byref(ein), None, 0, _lib.CLG_MEM_HOST, C.byref(n_out), C.byref(bad))
        if st not in (_lib.CLG_OK, _lib.CLG_E_CAPACITY):
            err = _lib.ClonosError(st, lib.clg_last_error().decode(errors="replace"))
            err.bad_index = bad.value
            raise err
        out = np.empty(max(1, n_out.value), np.uint8)
        check(lib.clg_encode_batch(self._h, C.byref(ein), _np_ptr(out), out.size, _lib.CLG_MEM_HOST, C.byref(n_out),
                                   C.byref(bad)))
        return out[:n_out.value].tobytes()

    def encode_decoded(self, dec: "DecodedBatch", span_bytes: bytes) -> bytes:
        """Round trip: re-encode a decoded span (its var fields index the span bytes)."""
        return self.encode_batch(dec.tag, dec.v0, dec.w_idx, dec.w_rc, dec.w_v1, dec.w_var_off, dec.w_var_len,
                                 dec.w_sub, span_bytes)

    # ---- replay-prep ----------------------------------------------------------------------
    def replay_prep(self, copies: Sequence[Tuple[int, bytes]]):
        """DeterminantResponseEvent.merge (longest wins, ties -> later) + batched decode of
        the winners.  Returns (winner indices, DecodedBatch over the winners)."""
        keys = np.array([c[0] for c in copies], np.uint64)
        blobs = [bytes(c[1]) for c in copies]
        offs = np.zeros(len(blobs), np.uint64)
        lens = np.array([len(b) for b in blobs], np.uint64)
        if len(blobs):
            offs[1:] = np.cumsum(lens)[:-1]
        data = np.frombuffer(b"".join(blobs) or b"\0", np.uint8)
        winner = np.zeros(max(len(blobs), 1), np.uint32)
        nk = C.c_uint32()
        total = int(lens.sum())
        d, arrs, _ = self._pooled_outputs(total // 2 + len(blobs) + 1, total // 6 + len(blobs) + 1)
        base = np.zeros(len(blobs) + 1, np.uint64)
        st = lib.clg_replay_prep(self._h, _np_ptr(keys), _np_ptr(data), _np_ptr(offs), _np_ptr(lens), len(blobs),
                                 _np_ptr(winner), C.byref(nk), C.byref(d), _np_ptr(base))
        k = nk.value
        win = winner[:k].copy()
        return win, self._finish(st, d, arrs, base, k, [np.frombuffer(blobs[i], np.uint8) for i in win])

    # ---- instrumentation ---------------------------------------------------------------------
    def kernel_stats(self):
        arr = (_lib.KernelStat * 64)()
        n = C.c_uint32()
        check(lib.clg_kernel_stats(self._h, arr, 64, C.byref(n)))
        return {arr[i].name.decode(): dict(launches=arr[i].launches, ms=arr[i].total_ms, bytes=arr[i].bytes)
                for i in range(min(n.value, 64))}

    def kernel_stats_reset(self):
        check(lib.clg_kernel_stats_reset(self._h))


class PendingDecode:
    """A queued clg_decode_logs_async; holds the output arrays until wait().  The engine
    completes its queued decodes in order (clg_decode_wait is FIFO): waiting for this one
    first waits for the ones queued before it, whose results (or errors) they keep."""

    def __init__(self, engine: "Engine", keep, n_spans: int):
        self._e, self._keep, self._n = engine, keep, n_spans
        self._done = False
        self._res = None  # (result, exception)

    def _complete(self) -> None:
        q = self._e._queued
        assert q and q[0] is self
        st = lib.clg_decode_wait(self._e._h)
        q.popleft()
        self._done = True
        _, _, d, arrs, base = self._keep
        try:
            self._res = (self._e._finish(st, d, arrs, base, self._n, None), None)
        except ClonosError as ex:
            self._res = (None, ex)

    def wait(self) -> DecodedBatch:
        while not self._done:
            head = self._e._queued[0]
            if isinstance(head, PendingDecode):
                head._complete()
            else:  # an earlier device-output decode: its status is its own caller's to take
                raise RuntimeError("an earlier decode_logs_device_async is not waited for (decode_wait)")
        res, ex = self._res
        if ex is not None:
            raise ex
        return res


class ThreadCausalLog:
    """Mirror of ThreadCausalLog (ThreadCausalLog.java:33-96) backed by the engine."""

    def __init__(self, engine: Engine, handle: int, cid: CausalLogID, job: int = 0):
        self.engine = engine
        self.handle = handle
        self.cid = cid
        self.job = job

    def getCausalLogID(self) -> CausalLogID:
        return self.cid

    def appendDeterminant(self, det: Union[D.Determinant, bytes], epochID: int) -> None:
        b = det if isinstance(det, (bytes, bytearray)) else D.encode(det)
        check(lib.clg_append(self.engine.handle, self.handle, epochID, bytes(b), len(b)))

    def processUpstreamDelta(self, delta: bytes, offsetFromEpoch: int, epochID: int) -> None:
        check(lib.clg_upstream_delta(self.engine.handle, self.handle, epochID, offsetFromEpoch, bytes(delta),
                                     len(delta)))

    def logLength(self) -> int:
        v = C.c_int32()
        check(lib.clg_log_length(self.engine.handle, self.handle, C.byref(v)))
        return v.value

    def hasDeltaForConsumer(self, outputChannelID: ChannelLike, epochID: int) -> bool:
        v = C.c_int32()
        check(lib.clg_has_delta(self.engine.handle, self.handle, _ch(outputChannelID), epochID, C.byref(v)))
        return bool(v.value)

    def getOffsetFromEpochForConsumer(self, outputChannelID: ChannelLike, epochID: int) -> int:
        v = C.c_int32()
        check(lib.clg_offset_from_epoch(self.engine.handle, self.handle, _ch(outputChannelID), C.byref(v)))
        return v.value

    @staticmethod
    def _probe_fetch(call) -> bytes:
        """Size probe, then fetch; CLG_E_CAPACITY (the log grew in between: another thread
        appended) reports the new size without moving anything, so fetch again."""
        n = C.c_uint32()
        st = call(None, 0, C.byref(n))
        buf = np.empty(1, np.uint8)
        while st == _lib.CLG_E_CAPACITY:
            buf = np.empty(n.value + 256, np.uint8)
            st = call(_np_ptr(buf), buf.size, C.byref(n))
        check(st)
        return buf[:n.value].tobytes()

    def getDeltaForConsumer(self, outputChannelID: ChannelLike, epochID: int) -> bytes:
        ch = _ch(outputChannelID)
        return self._probe_fetch(lambda p, cap, n: lib.clg_get_delta(self.engine.handle, self.handle, ch, epochID, p,
                                                                     cap, _lib.CLG_MEM_HOST, n))

    def determinants_length(self, startEpochID: int) -> int:
        """len(getDeterminants(startEpochID)) without moving bytes."""
        n = C.c_uint32()
        st = lib.clg_get_determinants(self.engine.handle, self.handle, startEpochID, None, 0, _lib.CLG_MEM_HOST,
                                      C.byref(n))
        if st not in (_lib.CLG_OK, _lib.CLG_E_CAPACITY):
            check(st)
        return n.value

    def determinants_into(self, startEpochID: int, dev_ptr: int, cap: int) -> int:
        """getDeterminants(startEpochID) gathered into device memory (engine's device)."""
        n = C.c_uint32()
        check(lib.clg_get_determinants(self.engine.handle, self.handle, startEpochID, dev_ptr, cap,
                                       _lib.CLG_MEM_DEVICE, C.byref(n)))
        return n.value

    def getDeterminants(self, startEpochID: int) -> bytes:
        return self._probe_fetch(lambda p, cap, n: lib.clg_get_determinants(self.engine.handle, self.handle,
                                                                            startEpochID, p, cap, _lib.CLG_MEM_HOST,
                                                                            n))

    def notifyCheckpointComplete(self, checkpointID: int) -> None:
        check(lib.clg_notify_checkpoint_complete(self.engine.handle, self.handle, checkpointID))

    def unregisterConsumer(self, toCancel: ChannelLike) -> None:
        check(lib.clg_unregister_consumer(self.engine.handle, self.handle, _ch(toCancel)))

    def close(self) -> None:
        check(lib.clg_log_close(self.engine.handle, self.handle))
        self.engine._logs.pop((self.job, self.cid.key()), None)

    # ---- introspection (tests / safety assertions) ----
    def state(self) -> dict:
        st = _lib.LogState()
        ids = np.zeros(4096, np.int64)
        offs = np.zeros(4096, np.int32)
        check(lib.clg_log_get_state(self.engine.handle, self.handle, C.byref(st), _np_ptr(ids), _np_ptr(offs), 4096))
        n = st.n_epochs
        return dict(writer=st.writer, capacity=st.capacity, n_components=st.n_components,
                    epochs=list(zip(ids[:n].tolist(), offs[:n].tolist())))

    def consumer_state(self, ch: ChannelLike):
        ex, ep, off = C.c_int32(), C.c_int64(), C.c_int32()
        check(lib.clg_consumer_state(self.engine.handle, self.handle, _ch(ch), C.byref(ex), C.byref(ep), C.byref(off)))
        return (ep.value, off.value) if ex.value else None

    def seek_consumer(self, ch: ChannelLike, epoch: int, offset: int) -> None:
        check(lib.clg_consumer_seek(self.engine.handle, self.handle, _ch(ch), epoch, offset))

    def read_phys(self, phys: int, n: int) -> bytes:
        buf = np.empty(max(n, 1), np.uint8)
        check(lib.clg_log_read_phys(self.engine.handle, self.handle, phys, n, _np_ptr(buf)))
        return buf[:n].tobytes()
