"""Multi-GPU sharding, sharing-depth replication and the cross-GPU replay-prep merge
(SURVEY.md 8e).

One process per GPU, one Engine per process.  Logs shard by VertexID (job.owner_rank):
rank g owns the vertices v with v mod G == g and is the only writer of their logs.

Replication.  Consumers on other GPUs need replicas of upstream logs within the sharing
depth (job.replication_masks).  Every rank builds the same canonical log table
(job.LogTable: a global index `gid` per CausalLogID), so the wire carries gids and every
per-log step is a numpy gather over dense tables -- no per-log Python.  One exchange (per
epoch, or per batch of buffers):

  1. the owner slices the new bytes of every owned log for every other rank that wants it
     (each receiving rank is one consumer of the log, with its own offset): the engine's
     batched hasDelta/getOffset/getDelta (clg_slice_batch), ONE device gather into a
     payload buffer grouped by destination;
  2. two all-to-alls (RCCL over xGMI with the "nccl" backend; gloo on CPU): the header
     rows, one per planned (log, destination) request, with static split sizes every rank
     knows from the plan; then, after one read-back of the headers, the payload with the
     split sizes they carry.  A rank receives only the logs within its sharing depth (at
     depth 1 only its direct producers'), and with one rank no collective runs;
  3. every rank applies the received rows with the batched processUpstreamDelta
     (clg_upstream_delta_batch) reading straight from the receive buffer in HBM.  The dedup
     rule of ThreadCausalLogImpl.java:117-154 makes re-delivery harmless.

This replaces the reference's piggybacking of CausalLogDelta on network buffers for
GPU-to-GPU traffic (AbstractDeltaSerializerDeserializer.java:89-163,
FlatDeltaSerializerDeserializer.java:57-90): the bytes and the (offsetFromEpoch, epoch)
pairs are the same, the transport is a collective.

Replay-prep merge (concurrent / connected failures).  DeterminantResponseEvent.merge
(DeterminantResponseEvent.java:128-148) keeps, per CausalLogID, the longest copy among
the responses (WaitingDeterminantsState.java:97-109).  Across GPUs: every rank measures its
copy of each log of the failed vertices, one all-reduce(MAX) over packed
(len << 8 | rank) picks the winner per log, and one all-to-all moves each winner's bytes to
the rank hosting the failed vertex's replacement (merge_responses).
"""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass
from typing import Dict, List, Optional, Sequence, Tuple

import itertools

import numpy as np

from . import _lib
from ._lib import check, lib
from .engine import CausalLogID, Engine, ThreadCausalLog
from .job import JobGraph, LogTable, owner_rank, replication_masks

# One header row per delta (little-endian, 32 bytes): global log index, epoch,
# offsetFromEpoch, length, payload offset inside the sender's payload for this receiver.
HEADER = np.dtype([("gid", "<i4"), ("offset_from_epoch", "<i4"), ("epoch", "<i8"), ("len", "<u4"),
                   ("pad", "<u4"), ("payload_off", "<u8")])
assert HEADER.itemsize == 32
BLOB_ALIGN = 64
REPLICATION_CHANNEL = (0xC1055EED00000000, 0x5EED)  # replication consumer; destination rank in ch_hi bits 16+

# numpy views of the C request / result structs (include/clonos_engine.h)
SLICE_REQ = np.dtype([("log", "<u4"), ("reserved", "<u4"), ("ch_lo", "<u8"), ("ch_hi", "<u8"), ("epoch", "<i8")])
SLICE_RES = np.dtype([("status", "<i4"), ("has_delta", "<i4"), ("offset_from_epoch", "<i4"), ("len", "<i4"),
                      ("out_off", "<u8")])
DELTA_REQ = np.dtype([("log", "<u4"), ("offset_from_epoch", "<i4"), ("epoch", "<i8"), ("src_off", "<u8"),
                      ("len", "<u4"), ("status", "<i4")])
assert SLICE_REQ.itemsize == C.sizeof(_lib.SliceReq) and SLICE_RES.itemsize == C.sizeof(_lib.SliceRes)
assert DELTA_REQ.itemsize == C.sizeof(_lib.DeltaReq)


def _align(n: int) -> int:
    return (n + BLOB_ALIGN - 1) // BLOB_ALIGN * BLOB_ALIGN


# ---- collectives ------------------------------------------------------------------------
def _to_comm(t, backend: str):
    """gloo moves host tensors; RCCL ("nccl") moves device tensors in place."""
    return t if (backend == "nccl" or not t.is_cuda) else t.cpu()


# ---- replication ------------------------------------------------------------------------
@dataclass
class ExchangeStats:
    sent_bytes: int = 0     # header rows + payload this rank sent
    recv_bytes: int = 0     # header rows + payload this rank received
    applied: int = 0        # deltas applied to replicas
    applied_bytes: int = 0  # delta bytes those deltas carried
    skipped: int = 0        # rows for logs this rank does not want


class ReplicationPlan:
    """The static part of sharing-depth replication for one rank: which owned logs it
    sends to which rank, which logs it keeps replicas of, and the dense handle tables.
    Built once per job and rank (registerTask time), identically on every rank.

    Each receiving rank is one downstream consumer of every log it wants (its own consumer
    offset per log, as each output channel is in FlatDeltaSerializerDeserializer.java:57-90),
    so a rank receives exactly the logs within its sharing depth and nothing else: the
    requests (req_gid, req_dest) are grouped by destination rank."""

    def __init__(self, table: LogTable, depth: int, rank: int, world: int,
                 need: Optional[np.ndarray] = None):
        self.table, self.rank, self.world = table, rank, world
        g = table.graph
        need = replication_masks(g, depth, world) if need is None else need  # [rank, vertex]
        owner = np.array([owner_rank(int(v), world) for v in range(need.shape[1])], np.int64)
        lv = table.vertex
        self.owned = np.nonzero(owner[lv] == rank)[0]            # gids this rank writes
        wanted_anywhere = need.any(axis=0)
        self.send = self.owned[wanted_anywhere[lv[self.owned]]]  # owned gids some rank wants
        self.wanted = np.nonzero(need[rank][lv])[0]               # gids this rank keeps replicas of
        # one slice request per (sent log, destination rank that wants it), by destination
        per_dest = [self.owned[need[r][lv[self.owned]]] if r != rank else self.owned[:0] for r in range(world)]
        self.req_gid = np.concatenate(per_dest).astype(np.int64) if world else np.zeros(0, np.int64)
        self.req_dest = np.repeat(np.arange(world, dtype=np.int64), [len(p) for p in per_dest])
        self.n_to = np.array([len(p) for p in per_dest], np.int64)  # requests per destination
        # header rows every other rank sends here (one per its planned request for this rank):
        # static, so the header all-to-all needs no count exchange first
        mine_needed = need[rank][lv]
        src_of = owner[lv]
        self.n_from = np.array([int(((src_of == r) & mine_needed).sum()) if r != rank else 0 for r in range(world)],
                               np.int64)


class EngineIO:
    """The byte work of replication on the engine (HBM): batched slices into a device
    blob, batched device-input processUpstreamDelta into replicas."""

    def __init__(self, engine: Engine, job: int = 0):
        self.engine, self.job = engine, job

    def open_replica(self, cid: CausalLogID) -> int:
        return self.engine.open_log(cid, self.job).handle

    def payload_bound(self, handles: np.ndarray) -> int:
        return self.engine.log_lengths(handles)[1]

    def slice(self, sreq: np.ndarray, sres: np.ndarray, n: int, out_ptr: int, cap: int) -> int:
        total = C.c_uint64()
        check(lib.clg_slice_batch(self.engine.handle, sreq.ctypes.data, n, sres.ctypes.data, out_ptr, cap,
                                  _lib.CLG_MEM_DEVICE, C.byref(total)))
        if self.engine.async_slice:  # the collective reads the payload: order it after the gather
            import torch
            gs = lib.clg_gather_stream(self.engine.handle)
            torch.cuda.current_stream().wait_stream(torch.cuda.ExternalStream(gs))
        return total.value

    def apply(self, req: np.ndarray, recv) -> None:
        kind = _lib.CLG_MEM_DEVICE if recv.is_cuda else _lib.CLG_MEM_HOST
        check(lib.clg_upstream_delta_batch(self.engine.handle, req.ctypes.data, len(req), recv.data_ptr(), kind))

    # replay-prep merge: a copy is getDeterminants(startEpoch) of a log (owned or replica);
    # both calls are one native call for all the copies (clg_get_determinants_batch)
    def copy_lengths(self, handles: np.ndarray, start_epochs: np.ndarray) -> np.ndarray:
        h = np.ascontiguousarray(handles, np.uint32)
        ep = np.ascontiguousarray(start_epochs, np.int64)
        ln = np.zeros(max(1, len(h)), np.uint32)
        total = C.c_uint64()
        check(lib.clg_get_determinants_batch(self.engine.handle, h.ctypes.data, ep.ctypes.data, len(h), None, 0,
                                             _lib.CLG_MEM_DEVICE, None, ln.ctypes.data, C.byref(total)))
        return ln[:len(h)].astype(np.int64)

    def copy_batch(self, handles: np.ndarray, start_epochs: np.ndarray, tensor, off: int) -> int:
        """The copies back to back in the given order into tensor[off:] (one gather)."""
        h = np.ascontiguousarray(handles, np.uint32)
        ep = np.ascontiguousarray(start_epochs, np.int64)
        ln = np.zeros(max(1, len(h)), np.uint32)
        total = C.c_uint64()
        kind = _lib.CLG_MEM_DEVICE if tensor.is_cuda else _lib.CLG_MEM_HOST
        check(lib.clg_get_determinants_batch(self.engine.handle, h.ctypes.data, ep.ctypes.data, len(h),
                                             tensor.data_ptr() + off, tensor.numel() - off, kind, None,
                                             ln.ctypes.data, C.byref(total)))
        return int(total.value)


class Replicator:
    """Sharing-depth replication for one rank.  `io` does the byte work (EngineIO; the CPU
    tests pass a stand-in over the oracle).  owned_handles: gid -> handle of each owned log
    that is sent; replicas of the wanted logs are opened here.

    One exchange moves each destination only the logs it wants: the slices of all requests
    land in one payload buffer grouped by destination (one batched slice), and two
    collectives carry them -- an all-to-all of the header rows (static split sizes: one row
    per planned request) and an all-to-all of the payload (split sizes from the headers).
    With one rank there is nothing to move and no collective runs."""

    def __init__(self, io, plan: ReplicationPlan, device, owned_handles: Dict[int, int], group=None):
        self.io, self.plan, self.device, self.group = io, plan, device, group
        n = len(plan.table)
        self.handle = np.full(n, -1, np.int64)
        for gid, h in owned_handles.items():
            self.handle[gid] = h
        self.replica_handle = np.full(n, -1, np.int64)
        for gid in plan.wanted:
            self.replica_handle[gid] = io.open_replica(plan.table.ids[gid])
        missing = sorted({int(g) for g in plan.req_gid if self.handle[g] < 0})
        if missing:
            raise ValueError(f"no log handle for owned gids {missing[:8]}")
        # prebuilt slice requests: one per (sent log, destination), the destination's consumer
        nq = len(plan.req_gid)
        self._sreq = np.zeros(max(nq, 1), SLICE_REQ)
        self._sreq["log"][:nq] = self.handle[plan.req_gid]
        self._sreq["ch_lo"][:nq] = REPLICATION_CHANNEL[0]
        self._sreq["ch_hi"][:nq] = REPLICATION_CHANNEL[1] | (plan.req_dest.astype(np.uint64) << np.uint64(16))
        self._sres = np.zeros(max(nq, 1), SLICE_RES)
        self._payload = None

    def payload_bound(self) -> int:
        """Bytes the requests' slices can need at most (their logs' lengths)."""
        nq = len(self.plan.req_gid)
        return self.io.payload_bound(self._sreq["log"][:nq]) if nq else 0

    def build_payload(self, epoch: int, payload_cap: Optional[int] = None):
        """Slice every request into the payload buffer (grouped by destination).  Returns
        (payload, one header row per planned request -- len 0 where there is no delta --,
        bytes per destination)."""
        import torch
        plan = self.plan
        nq = len(plan.req_gid)
        cap = payload_cap if payload_cap is not None else self.payload_bound()
        if self._payload is None or self._payload.numel() < cap + BLOB_ALIGN:
            self._payload = torch.empty(_align(cap) + BLOB_ALIGN, dtype=torch.uint8, device=self.device)
        self._sreq["epoch"][:nq] = epoch
        if nq:
            self.io.slice(self._sreq, self._sres, nq, self._payload.data_ptr(), cap)
        res = self._sres[:nq]
        bad = np.nonzero(res["status"])[0]
        if bad.size:
            check(int(res["status"][bad[0]]))
        ln = np.where(res["has_delta"] != 0, res["len"], 0).astype(np.int64)
        # clg_slice_batch packs the slices back to back in request order (requests are grouped
        # by destination), so each destination's part is contiguous; checked, not assumed
        out_off = res["out_off"].astype(np.int64)
        packed = np.concatenate([[0], np.cumsum(ln)[:-1]]).astype(np.int64) if nq else out_off
        keep = ln > 0
        if not np.array_equal(out_off[keep], packed[keep]):
            raise RuntimeError("slice outputs are not packed in request order")
        bytes_to = np.bincount(plan.req_dest, weights=ln, minlength=plan.world).astype(np.int64)
        start = np.concatenate([[0], np.cumsum(bytes_to)[:-1]]).astype(np.int64)
        rows = np.zeros(nq, HEADER)
        rows["gid"] = plan.req_gid
        rows["offset_from_epoch"] = np.where(keep, res["offset_from_epoch"], 0)
        rows["epoch"] = epoch
        rows["len"] = ln
        rows["payload_off"] = np.where(keep, packed - start[plan.req_dest], 0)  # within its destination's part
        return self._payload, rows, bytes_to

    def exchange(self, epoch: int, payload_cap: Optional[int] = None) -> ExchangeStats:
        """One replication round for `epoch` (all ranks call it together): two all-to-alls
        and one read-back.  The header rows go first with STATIC split sizes (one row per
        planned request, ReplicationPlan.n_to / n_from, so no count exchange precedes them);
        their read-back gives the payload's split sizes and the apply requests; then the
        payload."""
        import torch
        import torch.distributed as dist
        st = ExchangeStats()
        plan = self.plan
        if plan.world == 1:
            return st
        payload, rows, bytes_to = self.build_payload(epoch, payload_cap)
        backend = dist.get_backend(self.group)
        dev = self.device if backend == "nccl" else "cpu"
        # 1. header rows, static splits
        hsend = torch.from_numpy(rows.view(np.uint8).copy()).to(dev)
        hrecv = torch.empty(int(plan.n_from.sum()) * HEADER.itemsize, dtype=torch.uint8, device=dev)
        dist.all_to_all_single(hrecv, hsend, output_split_sizes=(plan.n_from * HEADER.itemsize).tolist(),
                               input_split_sizes=(plan.n_to * HEADER.itemsize).tolist(), group=self.group)
        rr = hrecv.cpu().numpy().view(HEADER)  # the one read-back (it also orders the host after the collective)
        src_rank = np.repeat(np.arange(plan.world), plan.n_from)
        bytes_from = np.bincount(src_rank, weights=rr["len"].astype(np.int64), minlength=plan.world).astype(np.int64)
        st.sent_bytes = int(rows_sent(rows)) * HEADER.itemsize + int(bytes_to.sum())
        st.recv_bytes = int(rows_sent(rr)) * HEADER.itemsize + int(bytes_from.sum())
        # 2. payload
        nrecv = int(bytes_from.sum())
        recv = torch.empty(max(nrecv, 1) + BLOB_ALIGN, dtype=torch.uint8, device=dev)
        psend = _to_comm(payload[:int(bytes_to.sum())], backend)
        dist.all_to_all_single(recv[:nrecv], psend, output_split_sizes=bytes_from.tolist(),
                               input_split_sizes=bytes_to.tolist(), group=self.group)
        live = rr["len"] > 0
        if not live.any():
            return st
        src_start = np.concatenate([[0], np.cumsum(bytes_from)[:-1]]).astype(np.uint64)
        src = src_start[src_rank] + rr["payload_off"].astype(np.uint64)
        h = self.replica_handle[rr["gid"]]
        want = live & (h >= 0)
        st.skipped = int((live & (h < 0)).sum())
        n = int(want.sum())
        if n:
            req = np.zeros(n, DELTA_REQ)
            req["log"] = h[want]
            req["offset_from_epoch"] = rr["offset_from_epoch"][want]
            req["epoch"] = rr["epoch"][want]
            req["src_off"] = src[want]
            req["len"] = rr["len"][want]
            if str(self.device).startswith("cuda") and not recv.is_cuda:  # gloo: into HBM once
                recv = recv.to(self.device)
            self.io.apply(req, recv)
            bad = np.nonzero(req["status"])[0]
            if bad.size:
                check(int(req["status"][bad[0]]))
            st.applied = n
            st.applied_bytes = int(req["len"].sum())
        return st


def rows_sent(rows: np.ndarray) -> int:
    """Header rows that carry a delta (the rest are the static slots of requests with none)."""
    return int((rows["len"] > 0).sum())


# ---- replay-prep merge across GPUs ---------------------------------------------------------
MERGE_GUARD = 64  # bytes before and after the received winners (device gathers read aligned 16-byte words)


class MergedCopies:
    """The winners delivered to one rank: every log's winning copy inside one buffer (an RCCL
    receive buffer in HBM, or host memory over gloo) at place[gid] = (offset, length), with
    MERGE_GUARD bytes around them, ready for clg_replay_prepare_device as they lie.  Also as
    arrays (gids, offsets, lengths), which the batched consumers read."""

    def __init__(self, buf, place: Optional[Dict[int, Tuple[int, int]]] = None, gids=None, offs=None, lens=None,
                 ranks=None):
        self.buf = buf
        if place is not None:
            gids = np.fromiter(place.keys(), np.int64, len(place))
            ol = np.array(list(place.values()), np.int64).reshape(-1, 2)
            offs, lens = ol[:, 0], ol[:, 1]
        self.gids = np.asarray(gids if gids is not None else [], np.int64)
        self.offs = np.asarray(offs if offs is not None else [], np.int64)
        self.lens = np.asarray(lens if lens is not None else [], np.int64)
        self.ranks = np.asarray(ranks if ranks is not None else np.full(len(self.gids), -1), np.int64)  # winner's rank
        self._place = place

    @property
    def place(self) -> Dict[int, Tuple[int, int]]:
        if self._place is None:
            self._place = dict(zip(self.gids.tolist(), zip(self.offs.tolist(), self.lens.tolist())))
        return self._place

    def bytes_of(self, gid: int) -> bytes:
        o, n = self.place[gid]
        return self.buf[o:o + n].cpu().numpy().tobytes() if n else b""

    def as_dict(self) -> Dict[int, bytes]:
        return {g: self.bytes_of(g) for g in self.place}


_GROUP_INFO: Dict[int, tuple] = {}


def _group_info(group) -> Tuple[int, int, str]:
    """(rank, world size, backend) of a process group, looked up once per group object (each
    torch.distributed query goes through its logging wrapper: ~10 us apiece on the merge's
    critical path).  The entry holds the group itself, so a re-initialised default group
    (a new object) is looked up afresh."""
    import torch.distributed as dist
    g = group if group is not None else dist.group.WORLD
    got = _GROUP_INFO.get(id(g))
    if got is None or got[0] is not g:
        got = (g, dist.get_rank(group), dist.get_world_size(group), dist.get_backend(group))
        _GROUP_INFO[id(g)] = got
    return got[1], got[2], got[3]


def copy_arrays(copies) -> Tuple[np.ndarray, np.ndarray]:
    """merge_responses' `copies` as (gids ascending, handles): from a dict gid -> handle, or
    already such a pair (a caller that merges every step converts its dict once)."""
    if isinstance(copies, tuple):
        return copies
    kv = np.fromiter(itertools.chain.from_iterable(copies.items()), np.int64, 2 * len(copies)).reshape(-1, 2)
    ck, cv = kv[:, 0], kv[:, 1]
    if len(ck) > 1 and not (ck[1:] > ck[:-1]).all():  # (callers usually build it in gid order)
        srt = np.argsort(ck)
        ck, cv = ck[srt], cv[srt]
    return ck, cv


def merge_responses(io, table: LogTable, failed: Sequence[int], copies,
                    start_epochs: Dict[int, int], dest_of: Dict[int, int], device, group=None,
                    timing: Optional[Dict[str, float]] = None) -> MergedCopies:
    """Cross-GPU DeterminantResponseEvent.merge for the logs of the failed vertices.

    copies: gid -> io handle of this rank's copy (owned log or replica) of a log of a failed
    vertex (a dict, or copy_arrays' pair); start_epochs: failed VertexID -> the epoch the request asks from
    (respondToDeterminantRequest -> getDeterminants(startEpoch), JobCausalLogImpl.java:
    188-204); dest_of: failed VertexID -> rank hosting its replacement.

    Step 1: every rank measures all its copies in one call and reports (len << 8 | rank);
    an all-reduce(MAX) picks, per log, the longest copy (DeterminantResponseEvent.java:
    137-146; equal lengths are equal bytes -- every copy is a prefix of the same log -- so the
    rank tie-break picks identical content).  Step 2: the winners this rank holds are
    gathered in one call, grouped by destination, and one all-to-all carries them to the
    ranks hosting the replacements.  Returns this rank's MergedCopies (a log no rank holds
    is absent, as in the merged map)."""
    import time as _time
    import torch
    import torch.distributed as dist
    t_in = _time.perf_counter()
    rank, world, backend = _group_info(group)
    if world > 255:
        raise ValueError("rank must fit the packed key's low byte")
    # every per-log step below is an array operation: a failed task has 129 logs at p=128
    fv = np.unique(np.fromiter((int(v) for v in failed), np.int64))
    gids = table.gids_of(fv)
    n = len(gids)
    vslot = np.searchsorted(fv, table.vertex[gids])  # each log's failed vertex, as an index into fv
    ep_of = np.array([start_epochs[int(v)] for v in fv], np.int64)
    dest = np.array([dest_of[int(v)] for v in fv], np.int64)[vslot]
    ck, cv = copy_arrays(copies)
    pos = np.minimum(np.searchsorted(ck, gids), max(len(ck) - 1, 0))
    held = np.nonzero(ck[pos] == gids)[0] if len(ck) else np.zeros(0, np.int64)  # logs this rank holds
    handles = cv[pos[held]]
    epochs = ep_of[vslot[held]]
    key = np.full(max(n, 1), -1, np.int64)
    t0 = _time.perf_counter()
    if timing is not None:
        timing["setup"] = timing.get("setup", 0.0) + t0 - t_in
    if len(held):
        key[held] = (io.copy_lengths(handles, epochs) << 8) | rank
    if timing is not None:  # (developer: the bench's phase split)
        timing["lengths"] = timing.get("lengths", 0.0) + _time.perf_counter() - t0
    if world == 1:  # every copy is this rank's: the winners are gathered in place, nothing moves
        win = key[:n]
        mine = np.nonzero(win >= 0)[0]
        lens = (win[mine] >> 8).astype(np.int64)
        tot = int(lens.sum())
        buf = torch.empty(MERGE_GUARD + max(tot, 1) + MERGE_GUARD, dtype=torch.uint8, device=device)
        t1 = _time.perf_counter()
        if tot:
            sel = np.searchsorted(held, mine)
            got = io.copy_batch(handles[sel], epochs[sel], buf, MERGE_GUARD)
            if got != tot:
                raise RuntimeError(f"logs changed during the merge ({got} != {tot} bytes)")
        t2 = _time.perf_counter()
        if timing is not None:
            timing["gather"] = timing.get("gather", 0.0) + t2 - t1
            timing["alloc"] = timing.get("alloc", 0.0) + t1 - t0
        offs = MERGE_GUARD + np.concatenate([[0], np.cumsum(lens)[:-1]]).astype(np.int64) if len(mine) else lens
        res = MergedCopies(buf, gids=gids[mine], offs=offs, lens=lens, ranks=np.zeros(len(mine), np.int64))
        if timing is not None:
            timing["finish"] = timing.get("finish", 0.0) + _time.perf_counter() - t2
        return res
    dev = device if backend == "nccl" else "cpu"
    kt = torch.from_numpy(key).to(dev)
    dist.all_reduce(kt, op=dist.ReduceOp.MAX, group=group)
    win = kt.cpu().numpy()[:n]
    win_rank = np.where(win >= 0, win & 0xFF, -1)
    win_len = np.where(win >= 0, win >> 8, 0)
    mine = np.nonzero(win_rank == rank)[0]
    order = mine[np.argsort(dest[mine], kind="stable")]  # by destination, then log order
    send_split = np.bincount(dest[mine], weights=win_len[mine], minlength=world).astype(np.int64)
    inbound = np.nonzero((win_rank >= 0) & (dest == rank))[0]
    recv_split = np.bincount(win_rank[inbound], weights=win_len[inbound], minlength=world).astype(np.int64)
    send = torch.empty(max(int(send_split.sum()), 1), dtype=torch.uint8, device=device)
    if int(send_split.sum()):
        sel = np.searchsorted(held, order)  # (every winner of this rank is a held log)
        got = io.copy_batch(handles[sel], epochs[sel], send, 0)
        if got != int(send_split.sum()):
            raise RuntimeError(f"logs changed during the merge ({got} != {int(send_split.sum())} bytes)")
    nrecv = int(recv_split.sum())
    buf = torch.empty(MERGE_GUARD + max(nrecv, 1) + MERGE_GUARD, dtype=torch.uint8, device=dev)
    s_in = _to_comm(send, backend)
    dist.all_to_all_single(buf[MERGE_GUARD:MERGE_GUARD + nrecv], s_in[:int(send_split.sum())],
                           output_split_sizes=recv_split.tolist(), input_split_sizes=send_split.tolist(),
                           group=group)
    # received in source-rank order, each source's winners in log order
    recv = inbound[np.lexsort((inbound, win_rank[inbound]))]
    lens = win_len[recv]
    offs = MERGE_GUARD + np.concatenate([[0], np.cumsum(lens)[:-1]]).astype(np.int64) if len(recv) else lens
    return MergedCopies(buf, gids=gids[recv], offs=offs, lens=lens, ranks=win_rank[recv])
