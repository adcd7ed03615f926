"""CPU, world_size 2 over gloo: the sharing-depth replication protocol of
clonos_amd/dist.py (blob packing, all-gather of variable-size blobs, the wanted-vertex
filter, per-epoch re-delivery).  The byte store is the oracle's ThreadCausalLogImpl model
(test infrastructure: it stands in for the engine, which needs a GPU; the same exchange
over real engines is tests/test_gpu_dist.py)."""
import os
import socket
import sys

import numpy as np
import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
sys.path.insert(0, os.path.dirname(HERE))

N_VERT = 6
EPOCHS = 4
SEG = 64


def free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def log_ids():
    from clonos_amd import CausalLogID
    ids = [CausalLogID.main(v) for v in range(N_VERT)]
    ids += [CausalLogID.sub(v, 100 + v, 200 + v, s) for v in range(N_VERT) for s in range(2)]
    return ids


def records(cid, epoch):
    """Deterministic content of log `cid` in `epoch` (every rank can recompute it)."""
    from clonos_amd import determinants as D, synth
    rng = np.random.default_rng(hash(cid.key()) % (1 << 30) * 31 + epoch)
    return b"".join(D.encode(synth.random_determinant(rng)) for _ in range(int(rng.integers(0, 60))))


class OracleIO:
    def __init__(self):
        import _oracle as O
        self.O = O
        self.replicas = {}

    def build_blob(self, owned, epoch):
        import torch
        from clonos_amd import dist as X
        rows, payload = [], bytearray()
        for cid, ol in owned:
            st, has = ol.has_delta(X.REPLICATION_CHANNEL, epoch)
            assert st == 0
            if has:
                ofe = ol.offset(X.REPLICATION_CHANNEL)[1]
                st, d = ol.get_delta(X.REPLICATION_CHANNEL, epoch)
                assert st == 0
                rows.append(X.header_row(cid, epoch, ofe, len(d), len(payload)))
                payload += d
        head = X.pack_header(np.array(rows, X.HEADER))
        return torch.frombuffer(bytearray(head + bytes(payload)) or bytearray(64), dtype=torch.uint8)

    def apply(self, recv, plan):
        buf = recv.numpy().tobytes()
        out = []
        for lid, epoch, ofe, src, n in plan:
            ol = self.replicas.setdefault(lid.key(), self.O.OracleLog(SEG))
            out.append(ol.upstream(buf[src:src + n], ofe, epoch))
        return out


def worker(rank, world, port, q):
    try:
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        import torch.distributed as dist
        import _oracle as O
        from clonos_amd import dist as X
        from clonos_amd.job import owner_rank
        dist.init_process_group("gloo", rank=rank, world_size=world)
        mine = [cid for cid in log_ids() if owner_rank(cid.vertex_id, world) == rank]
        owned = [(cid, O.OracleLog(SEG)) for cid in mine]
        wanted = {v for v in range(N_VERT) if owner_rank(v, world) != rank and v != 1}  # vertex 1 not wanted
        io = OracleIO()
        rep = X.Replicator(io, rank, world, wanted)
        for ep in range(EPOCHS):
            for half in range(2):  # two exchanges per epoch: re-delivery must be a no-op
                for cid, ol in owned:
                    r = records(cid, ep)
                    part = r[:len(r) // 2] if half == 0 else r[len(r) // 2:]
                    if part:
                        assert ol.append(ep, part) == 0
                rep.exchange(owned, ep)
        # every wanted replica holds exactly the owner's bytes
        got = 0
        for cid in log_ids():
            if cid.vertex_id not in wanted:
                assert cid.key() not in io.replicas or owner_rank(cid.vertex_id, world) == rank
                continue
            expect = b"".join(records(cid, ep) for ep in range(EPOCHS))
            ol = io.replicas.get(cid.key())
            have = ol.get_determinants(0)[1] if ol is not None else b""
            assert have == expect, (rank, cid)
            got += 1
        dist.barrier()
        dist.destroy_process_group()
        q.put((rank, "ok", got))
    except Exception as e:  # surface the failure in the parent
        import traceback
        q.put((rank, "fail", traceback.format_exc()))


def test_replication_gloo_world2():
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = free_port()
    procs = [ctx.Process(target=worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = [q.get(timeout=240) for _ in procs]
    for p in procs:
        p.join(timeout=60)
    for rank, status, info in res:
        assert status == "ok", info
    assert sum(info for _, _, info in res) > 0


def test_header_roundtrip():
    from clonos_amd import CausalLogID
    from clonos_amd import dist as X
    rows = np.array([X.header_row(CausalLogID.main(7), 3, 11, 5, 0),
                     X.header_row(CausalLogID.sub(-2, 1 << 40, -5, 3), 9, 0, 17, 64)], X.HEADER)
    b = X.pack_header(rows)
    assert len(b) % 64 == 0
    back = X.unpack_header(b)
    assert back.tobytes() == rows.tobytes()
    assert X.row_log_id(back[1]).key() == CausalLogID.sub(-2, 1 << 40, -5, 3).key()
