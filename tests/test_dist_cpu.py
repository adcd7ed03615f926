"""CPU, world sizes 2, 4 and 8 over gloo: the sharing-depth replication protocol of
clonos_amd/dist.py (canonical log table, per-destination consumers and requests, the
all-to-alls of counts, header rows and payload, per-epoch re-delivery, depth -1 and 1) and
the cross-GPU replay-prep merge (all-reduce MAX with ties to the highest rank, all-to-all).  The byte store is the oracle's ThreadCausalLogImpl model
(test infrastructure standing in for the engine, which needs a GPU; the same protocol
over real engines is tests/test_gpu_dist.py)."""
import os
import socket
import sys

import numpy as np
import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
sys.path.insert(0, os.path.dirname(HERE))

EPOCHS = 4
SEG = 64
STAGES, PAR = 3, 4


def free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def records(cid, epoch, scale=60):
    """Deterministic content of log `cid` in `epoch` (every rank can recompute it)."""
    from clonos_amd import determinants as D, synth
    seed = (hash(cid.key()) % (1 << 30)) * 31 + epoch
    rng = np.random.default_rng(seed)
    if not cid.is_main:  # subpartition logs hold BufferBuilt records (ReplayingState :172-177)
        return b"".join(D.encode(D.BufferBuiltDeterminant(int(rng.integers(1, 1 << 15))))
                        for _ in range(int(rng.integers(0, scale // 6 + 1))))
    return b"".join(D.encode(synth.random_determinant(rng)) for _ in range(int(rng.integers(0, scale))))


class OracleIO:
    """dist.Replicator's IO over oracle logs (handles index self.logs)."""

    def __init__(self):
        import _oracle as O
        self.O = O
        self.logs = []

    def new_log(self):
        self.logs.append(self.O.OracleLog(SEG))
        return len(self.logs) - 1

    def open_replica(self, cid):
        return self.new_log()

    def payload_bound(self, handles):
        return sum(self.logs[int(h)].state()["writer"] for h in handles)

    def slice(self, sreq, sres, n, out_ptr, cap):
        import ctypes
        from clonos_amd import dist as X
        dst = 0
        for i in range(n):
            ol = self.logs[int(sreq["log"][i])]
            ch = (int(sreq["ch_lo"][i]), int(sreq["ch_hi"][i]))
            ep = int(sreq["epoch"][i])
            st, has = ol.has_delta(ch, ep)
            sres[i] = (st, int(has), 0, 0, dst)
            if st or not has:
                continue
            ofe = ol.offset(ch)[1]
            st, d = ol.get_delta(ch, ep)
            assert dst + len(d) <= cap
            ctypes.memmove(out_ptr + dst, d, len(d))
            sres[i] = (st, 1, ofe, len(d), dst)
            dst += len(d)
        assert X.REPLICATION_CHANNEL == (int(sreq["ch_lo"][0]), int(sreq["ch_hi"][0]) & 0xFFFF)
        return dst

    def apply(self, req, recv):
        buf = recv.numpy().tobytes()
        for r in req:
            n = int(r["len"])
            src = int(r["src_off"])
            r["status"] = self.logs[int(r["log"])].upstream(buf[src:src + n], int(r["offset_from_epoch"]),
                                                            int(r["epoch"]))


def worker(rank, world, port, q, depth):
    try:
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        import torch.distributed as dist
        from clonos_amd import dist as X
        from clonos_amd import job as J
        dist.init_process_group("gloo", rank=rank, world_size=world)
        g = J.dag(STAGES, PAR)
        table = J.LogTable(g)
        plan = X.ReplicationPlan(table, depth, rank, world)
        io = OracleIO()
        owned = {int(gid): io.new_log() for gid in plan.owned}
        rep = X.Replicator(io, plan, "cpu", {gid: h for gid, h in owned.items() if gid in set(plan.send.tolist())})
        # each destination gets exactly the logs it wants, once
        need_all = J.replication_masks(g, depth, world)
        for r in range(world):
            mine_to_r = plan.req_gid[plan.req_dest == r]
            expect = [int(x) for x in plan.owned if r != rank and need_all[r][table.vertex[x]]]
            assert mine_to_r.tolist() == expect
        for ep in range(EPOCHS):
            for half in range(2):  # two exchanges per epoch: re-delivery must be a no-op
                for gid, h in owned.items():
                    r = records(table.ids[gid], ep)
                    part = r[:len(r) // 2] if half == 0 else r[len(r) // 2:]
                    if part:
                        assert io.logs[h].append(ep, part) == 0
                st = rep.exchange(ep)
                assert st.skipped == 0  # a rank is sent only the logs it wants
        # every wanted replica holds exactly the owner's bytes; nothing else was opened
        need = J.replication_masks(g, depth, world)[rank]
        got = 0
        for gid, cid in enumerate(table.ids):
            h = int(rep.replica_handle[gid])
            if not need[cid.vertex_id]:
                assert h < 0
                continue
            expect = b"".join(records(cid, ep) for ep in range(EPOCHS))
            assert io.logs[h].get_determinants(0)[1] == expect, (rank, cid)
            got += 1
        dist.barrier()
        dist.destroy_process_group()
        q.put((rank, "ok", got))
    except Exception:  # surface the failure in the parent
        import traceback
        q.put((rank, "fail", traceback.format_exc()))


def run_world(target, *args, world=2):
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = free_port()
    procs = [ctx.Process(target=target, args=(r, world, port, q) + args) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=240) for _ in procs]
    for p in procs:
        p.join(timeout=60)
    for rank, status, info in res:
        assert status == "ok", info
    return res


@pytest.mark.parametrize("world", [2, 4, 8])
@pytest.mark.parametrize("depth", [-1, 1])
def test_replication_gloo(depth, world):
    res = run_world(worker, depth, world=world)
    assert sum(info for _, _, info in res) > 0


def test_header_layout():
    from clonos_amd import dist as X
    rows = np.zeros(3, X.HEADER)
    rows["gid"] = [7, 0, 66175]
    rows["len"] = [5, 0, 17]
    assert X.HEADER.itemsize == 32
    assert np.frombuffer(rows.tobytes(), X.HEADER)["gid"].tolist() == [7, 0, 66175]


@pytest.mark.parametrize("world", [1, 2, 4, 8])
def test_plan_depth1_sends_direct_producers_only(world):
    """At depth 1 a rank receives the logs of its subtasks' direct producers only (config 1's
    sharing depth), so the requests to it are exactly those; at world 1 there are none."""
    from clonos_amd import dist as X
    from clonos_amd import job as J
    g = J.dag(4, 8)
    table = J.LogTable(g)
    need = J.replication_masks(g, 1, world)
    plans = [X.ReplicationPlan(table, 1, r, world, need) for r in range(world)]
    for dst in range(world):
        got = sorted(int(x) for p in plans for x in p.req_gid[p.req_dest == dst])
        assert got == plans[dst].wanted.tolist()
        stages = {int(table.vertex[x]) // 8 for x in got}
        own_stages = {v // 8 for v in range(32) if J.owner_rank(v, world) == dst}
        assert all(s + 1 in own_stages for s in stages)  # only a stage right below one it hosts
    if world == 1:
        assert len(plans[0].req_gid) == 0


def test_plan_partitions_logs():
    """Every log is owned by exactly one rank; a rank never wants its own logs; a log is
    sent iff some rank wants it (config 4: 5 stages x 128, 8 ranks)."""
    from clonos_amd import dist as X
    from clonos_amd import job as J
    g = J.dag(5, 128)
    table = J.LogTable(g)
    assert len(table) == 640 + 4 * 128 * 128
    need = J.replication_masks(g, -1, 8)
    plans = [X.ReplicationPlan(table, -1, r, 8, need) for r in range(8)]
    owned = np.concatenate([p.owned for p in plans])
    assert sorted(owned.tolist()) == list(range(len(table)))
    for p in plans:
        assert not set(p.owned.tolist()) & set(p.wanted.tolist())
        assert len(p.wanted) == 448 * 129  # stages 0..3 minus the 64 vertices it owns there
    sent = set(np.concatenate([p.send for p in plans]).tolist())
    wanted = set(np.concatenate([p.wanted for p in plans]).tolist())
    assert sent == wanted


def merge_worker(rank, world, port, q):
    """Cross-GPU merge over oracle copies: each rank holds a prefix (different lengths) of
    every log of the failed vertices; the winners equal DeterminantResponseEvent.merge of
    the per-rank responses in any arrival order (oracle/response_ref.py)."""
    try:
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        import torch.distributed as dist
        from clonos_amd import dist as X
        from clonos_amd import job as J
        import response_ref as R
        dist.init_process_group("gloo", rank=rank, world_size=world)
        g = J.dag(STAGES, PAR)
        table = J.LogTable(g)
        failed = [1, 5]  # a connected pair (stage 0 subtask 1 -> stage 1 subtask 1)
        dest_of = {1: 1 % world, 5: 0}
        full = {gid: records(table.ids[gid], 0, 200) for gid in range(len(table)) if table.vertex[gid] in failed}
        rng = np.random.default_rng(9)
        cut = {gid: [int(rng.integers(0, len(b) + 1)) for _ in range(world)] for gid, b in full.items()}
        for gid in list(cut)[:3]:
            cut[gid] = [len(full[gid])] * world  # ties: every rank holds the whole log
        store = OracleStore(full, cut, rank)
        merged = X.merge_responses(store, table, failed, store.handles, {1: 0, 5: 0}, dest_of, "cpu")
        got = merged.as_dict()
        # the copies as copy_arrays' pair (what a caller merging every step passes): the same
        again = X.merge_responses(store, table, failed, X.copy_arrays(store.handles), {1: 0, 5: 0}, dest_of, "cpu")
        assert again.as_dict() == got and (again.ranks == merged.ranks).all()
        # the winner is the longest copy; equal lengths go to the highest rank
        for gid, rk in zip(merged.gids.tolist(), merged.ranks.tolist()):
            lens = cut[gid]
            assert lens[rk] == max(lens) and rk == max(r for r in range(world) if lens[r] == max(lens))
        for o, nb in merged.place.values():  # guard bytes around every winner
            assert o >= X.MERGE_GUARD and o + nb + X.MERGE_GUARD <= merged.buf.numel()

        def lid(cid):
            return (R.LogId.main(cid.vertex_id) if cid.is_main else
                    R.LogId.subpartition(cid.vertex_id, cid.irp_lower, cid.irp_upper, cid.subpartition))
        # the reference: every rank's response merged in arrival order (two orders)
        for order in (list(range(world)), list(reversed(range(world)))):
            acc = R.Response(True, 0)
            for r in order:
                ev = R.Response(True, 0)
                for gid, b in full.items():
                    ev.dets.put(lid(table.ids[gid]), b[:cut[gid][r]])
                acc.merge(ev)
            want = {gid: acc.dets.get(lid(table.ids[gid])) for gid in full
                    if dest_of[int(table.vertex[gid])] == rank}
            assert got == want
        dist.destroy_process_group()
        q.put((rank, "ok", len(got)))
    except Exception:
        import traceback
        q.put((rank, "fail", traceback.format_exc()))


class OracleStore:
    """merge_responses' view of a rank's copies, over host bytes (stands in for the engine)."""

    def __init__(self, full, cut, rank):
        self.copies = {gid: b[:cut[gid][rank]] for gid, b in full.items()}
        self.handles = {gid: gid for gid in full}

    def copy_lengths(self, handles, start_epochs):
        return np.array([len(self.copies[int(h)]) for h in handles], np.int64)

    def copy_batch(self, handles, start_epochs, tensor, off):
        import torch
        for h in handles:
            b = self.copies[int(h)]
            if b:
                tensor[off:off + len(b)] = torch.frombuffer(bytearray(b), dtype=torch.uint8)
            off += len(b)
        return sum(len(self.copies[int(h)]) for h in handles)


@pytest.mark.parametrize("world", [1, 2, 4, 8])
def test_merge_gloo(world):
    sys.path.insert(0, os.path.join(os.path.dirname(HERE), "oracle"))
    res = run_world(merge_worker, world=world)
    assert sum(info for _, _, info in res) == 2 * (1 + 4)  # both failed vertices' logs
