"""Multi-GPU sharding and sharing-depth replication.

One process per GPU, one Engine per process.  Logs shard by VertexID (job.owner_rank):
rank g owns the vertices v with v mod G == g and is the only writer of their logs.
Consumers on other GPUs need replicas of upstream logs within the sharing depth
(job.replication_plan).  Once per exchange (e.g. per epoch or per batch of buffers):

  1. every rank slices the new bytes of each owned log for one replication consumer
     per log (the engine's batched getDeltaForConsumer: one device gather into a
     send blob, no host copy of the bytes);
  2. the blob = [header table | payload]; blob sizes are all-gathered, then the padded
     blobs (torch.distributed.all_gather_into_tensor: RCCL over xGMI with the "nccl"
     backend, gloo on CPU);
  3. every rank applies the deltas of the logs it needs with the batched
     processUpstreamDelta (clg_upstream_delta_batch), reading straight from the receive
     buffer in HBM.  The dedup rule of :117-154 makes re-delivery harmless.

This replaces the reference's piggybacking of CausalLogDelta on network buffers for
GPU-to-GPU traffic (AbstractDeltaSerializerDeserializer.java:89-163): the bytes and the
(offsetFromEpoch, epoch) header are the same, the transport is a collective.
"""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass
from typing import Dict, Iterable, List, Optional, Sequence, Tuple

import numpy as np

from . import _lib
from ._lib import check
from .engine import CausalLogID, Engine, ThreadCausalLog

# One header row per delta (little-endian, 48 bytes).
HEADER = np.dtype([("vertex", "<i2"), ("is_main", "u1"), ("sub", "i1"), ("pad", "<u4"),
                   ("irp_lo", "<i8"), ("irp_hi", "<i8"), ("epoch", "<i8"),
                   ("offset_from_epoch", "<i4"), ("len", "<u4"), ("payload_off", "<u8")])
assert HEADER.itemsize == 48
BLOB_ALIGN = 64
REPLICATION_CHANNEL = (0xC1055EED00000000, 0x5EED)  # the replication consumer of every log


def _align(n: int) -> int:
    return (n + BLOB_ALIGN - 1) // BLOB_ALIGN * BLOB_ALIGN


def header_bytes(n_rows: int) -> int:
    """[u64 n_rows][pad to 64][rows] rounded up to 64."""
    return _align(BLOB_ALIGN + n_rows * HEADER.itemsize)


def pack_header(rows: np.ndarray) -> bytes:
    out = bytearray(header_bytes(len(rows)))
    out[0:8] = np.uint64(len(rows)).tobytes()
    out[BLOB_ALIGN:BLOB_ALIGN + rows.nbytes] = rows.tobytes()
    return bytes(out)


def unpack_header(blob: bytes) -> np.ndarray:
    n = int(np.frombuffer(blob[:8], np.uint64)[0])
    return np.frombuffer(blob[BLOB_ALIGN:BLOB_ALIGN + n * HEADER.itemsize], HEADER).copy()


def header_row(lid: CausalLogID, epoch: int, offset_from_epoch: int, n: int, payload_off: int) -> tuple:
    return (lid.vertex_id, 1 if lid.is_main else 0, 0 if lid.is_main else lid.subpartition, 0,
            0 if lid.is_main else lid.irp_lower, 0 if lid.is_main else lid.irp_upper, epoch, offset_from_epoch, n,
            payload_off)


def row_log_id(r) -> CausalLogID:
    if r["is_main"]:
        return CausalLogID.main(int(r["vertex"]))
    return CausalLogID.sub(int(r["vertex"]), int(r["irp_lo"]), int(r["irp_hi"]), int(r["sub"]))


# ---- the collective: all-gather of variable-size blobs ------------------------------------
def allgather_blobs(send, group=None):
    """All-gather one uint8 tensor per rank (sizes differ): returns (recv, sizes, stride)
    with rank r's blob at recv[r * stride : r * stride + sizes[r]]."""
    import torch
    import torch.distributed as dist
    world = dist.get_world_size(group)
    n = torch.tensor([send.numel()], dtype=torch.int64, device=send.device)
    sizes_t = torch.empty(world, dtype=torch.int64, device=send.device)
    dist.all_gather_into_tensor(sizes_t, n, group=group)
    sizes = [int(x) for x in sizes_t.cpu()]
    stride = _align(max(sizes) if sizes else 0) or BLOB_ALIGN
    padded = torch.zeros(stride, dtype=torch.uint8, device=send.device)
    padded[:send.numel()] = send
    recv = torch.empty(world * stride, dtype=torch.uint8, device=send.device)
    dist.all_gather_into_tensor(recv, padded, group=group)
    return recv, sizes, stride


# ---- engine I/O (the product path) ------------------------------------------------------
class EngineIO:
    """Slices and applies deltas through the engine; blobs live in HBM."""

    def __init__(self, engine: Engine, device):
        self.engine = engine
        self.device = device
        self.replicas: Dict[tuple, ThreadCausalLog] = {}

    def build_blob(self, owned: Sequence[ThreadCausalLog], epoch: int):
        import torch
        n = len(owned)
        creq = (_lib.SliceReq * max(1, n))()
        cres = (_lib.SliceRes * max(1, n))()
        for k, lg in enumerate(owned):
            creq[k].log = lg.handle
            creq[k].consumer = _lib.ChannelId(*REPLICATION_CHANNEL)
            creq[k].epoch = epoch
        cap = sum(lg.logLength() for lg in owned) + BLOB_ALIGN
        hb = header_bytes(n)
        blob = torch.empty(hb + cap, dtype=torch.uint8, device=self.device)
        total = self.engine.slice_batch_raw(creq, cres, n, blob.data_ptr() + hb, cap, device=True) if n else 0
        rows = []
        for k, lg in enumerate(owned):
            r = cres[k]
            check(r.status)
            if r.has_delta and r.len:
                rows.append(header_row(lg.cid, epoch, r.offset_from_epoch, r.len, r.out_off))
        head = pack_header(np.array(rows, HEADER))
        hb2 = len(head)
        if hb2 != hb:  # fewer rows than logs: compact the header in front of the payload
            blob2 = torch.empty(hb2 + total, dtype=torch.uint8, device=self.device)
            blob2[hb2:] = blob[hb:hb + total]
            blob, hb = blob2, hb2
        blob[:hb] = torch.frombuffer(bytearray(head), dtype=torch.uint8).to(self.device)
        return blob[:hb + total]

    def replica(self, lid: CausalLogID) -> ThreadCausalLog:
        key = lid.key()
        lg = self.replicas.get(key)
        if lg is None:
            lg = self.replicas[key] = self.engine.open_log(lid)
        return lg

    def apply(self, recv, plan: List[Tuple[CausalLogID, int, int, int, int]]) -> List[int]:
        """plan rows: (log id, epoch, offsetFromEpoch, src_off in recv, len)."""
        if not plan:
            return []
        reqs = (_lib.DeltaReq * len(plan))()
        for k, (lid, epoch, ofe, src, n) in enumerate(plan):
            reqs[k].log = self.replica(lid).handle
            reqs[k].offset_from_epoch = ofe
            reqs[k].epoch = epoch
            reqs[k].src_off = src
            reqs[k].len = n
        kind = _lib.CLG_MEM_DEVICE if recv.is_cuda else _lib.CLG_MEM_HOST
        self.engine.upstream_delta_batch(reqs, len(plan), recv.data_ptr(), kind)
        return [reqs[k].status for k in range(len(plan))]


@dataclass
class ExchangeStats:
    sent_bytes: int = 0
    recv_bytes: int = 0
    applied: int = 0
    skipped: int = 0


class Replicator:
    """Sharing-depth replication for one rank.  `io` does the byte work (EngineIO on a
    GPU); `wanted` is the set of VertexIDs this rank needs from other ranks
    (job.replication_plan(...)[rank])."""

    def __init__(self, io, rank: int, world: int, wanted: Iterable[int], group=None):
        self.io = io
        self.rank = rank
        self.world = world
        self.wanted = set(int(v) for v in wanted)
        self.group = group

    def exchange(self, owned: Sequence, epoch: int) -> ExchangeStats:
        import torch
        import torch.distributed as dist
        st = ExchangeStats()
        blob = self.io.build_blob(owned, epoch)
        st.sent_bytes = int(blob.numel())
        backend = dist.get_backend(self.group)
        send = blob if (backend == "nccl" or not blob.is_cuda) else blob.cpu()
        recv, sizes, stride = allgather_blobs(send, self.group)
        recv_dev = recv if (recv.is_cuda or not blob.is_cuda) else recv.to(blob.device)
        plan = []
        for r in range(self.world):
            if r == self.rank or sizes[r] == 0:
                continue
            base = r * stride
            n_rows = int(np.frombuffer(recv[base:base + 8].cpu().numpy().tobytes(), np.uint64)[0])
            hb = header_bytes(n_rows)
            rows = unpack_header(recv[base:base + hb].cpu().numpy().tobytes())
            st.recv_bytes += sizes[r]
            for row in rows:
                if int(row["vertex"]) not in self.wanted:
                    st.skipped += 1
                    continue
                plan.append((row_log_id(row), int(row["epoch"]), int(row["offset_from_epoch"]),
                             base + hb + int(row["payload_off"]), int(row["len"])))
        statuses = self.io.apply(recv_dev, plan)
        for s in statuses:
            check(s)
        st.applied = len(plan)
        return st
