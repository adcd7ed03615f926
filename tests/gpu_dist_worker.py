"""Launcher for tests/test_gpu_dist.py: two ranks (gloo transport), one Engine each on
cuda:0.  Config 4's shape at reduced log sizes -- the 5-stage DAG at parallelism 128 under
full sharing (640 VertexIDs, 1 main + 128 subpartition logs per producing vertex) -- is
replicated with clonos_amd.dist over real engines, then the replay-prep merge runs across
the ranks.  The launcher itself never touches the GPU; each rank is a fresh process.

Checks, per rank: every replica holds exactly the owner's bytes (all ~33k replicas, read
back in one batched slice), replica state == the oracle's ThreadCausalLogImpl fed the same
epochs (a sample), the merge winners == DeterminantResponseEvent.merge of the ranks'
responses (oracle/response_ref.py), replay preparation on the destination ranks straight
from the merge's receive buffer (clg_replay_prepare_device) == the oracle's decode and
BufferBuilt sizes of the merged logs, and truncation afterwards (job CAS) matches the oracle.
"""
import os
import socket
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
sys.path.insert(0, os.path.dirname(HERE))
sys.path.insert(0, os.path.join(os.path.dirname(HERE), "oracle"))

STAGES, PAR, EPOCHS, SEG = 5, 128, 3, 1024


def content(gid: int, epoch: int, is_main: bool) -> bytes:
    """Deterministic bytes of log `gid` in `epoch`: main logs a few Order/Timestamp/RNG
    records, subpartition logs BufferBuilt records (0-3 per epoch)."""
    rng = np.random.default_rng(gid * 131 + epoch)
    out = bytearray()
    if is_main:
        for _ in range(int(rng.integers(0, 12))):
            t = int(rng.integers(0, 3))
            out += (bytes([0, int(rng.integers(0, 4))]) if t == 0 else
                    bytes([1]) + int(rng.integers(0, 1 << 40)).to_bytes(8, "big") if t == 1 else
                    bytes([2]) + int(rng.integers(0, 1 << 31)).to_bytes(4, "big"))
    else:
        for _ in range(int(rng.integers(0, 4))):
            out += bytes([7]) + int(rng.integers(1, 1 << 15)).to_bytes(4, "big")
    return bytes(out)


def worker(rank, world, port, q):
    try:
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        import torch
        import torch.distributed as dist
        import _oracle as O
        from clonos_amd import Engine, _lib
        from clonos_amd import dist as X
        from clonos_amd.engine import ThreadCausalLog
        from clonos_amd import job as J
        dist.init_process_group("gloo", rank=rank, world_size=world)
        dev = torch.device("cuda", 0)
        g = J.dag(STAGES, PAR)
        table = J.LogTable(g)
        need = J.replication_masks(g, -1, world)
        plan = X.ReplicationPlan(table, -1, rank, world, need)
        assert len(plan.wanted) == (4 * PAR // world) * (PAR + 1) * (world - 1)
        eng = Engine(segment_bytes=SEG, pool_segments=len(plan.owned) + len(plan.wanted) + 4096, device=0,
                     ifl_pool_segments=16)
        owned = {int(gid): eng.open_log(table.ids[gid]).handle for gid in plan.owned}
        send = set(plan.send.tolist())
        rep = X.Replicator(X.EngineIO(eng), plan, dev, {k: v for k, v in owned.items() if k in send})
        gids = np.array(sorted(owned), np.int64)
        stats = []
        for ep in range(EPOCHS):
            blob = bytearray()
            reqs = np.zeros(len(gids), X.DELTA_REQ)
            for k, gid in enumerate(gids):  # the owners' new epoch, appended in one batch
                b = content(int(gid), ep, table.ids[gid].is_main)
                reqs[k] = (owned[int(gid)], 0, ep, len(blob), len(b), 0)
                blob += b
            hb = np.frombuffer(bytes(blob) or b"\0", np.uint8)
            _lib.check(_lib.lib.clg_upstream_delta_batch(eng.handle, reqs.ctypes.data, len(reqs), hb.ctypes.data,
                                                         _lib.CLG_MEM_HOST))
            stats.append(rep.exchange(ep))
        assert stats[0].applied > 0 and stats[0].skipped == 0
        # every replica == the owner's bytes (getDeterminants from the first epoch)
        wanted = plan.wanted
        got = {int(gid): ThreadCausalLog(eng, int(rep.replica_handle[gid]), table.ids[gid]).getDeterminants(0)
               for gid in wanted}
        n_bytes = 0
        for gid in wanted:
            want = b"".join(content(int(gid), ep, table.ids[gid].is_main) for ep in range(EPOCHS))
            assert bytes(got[int(gid)]) == want, (rank, int(gid))
            n_bytes += len(want)
        # replica state == the oracle's ThreadCausalLogImpl fed the same epochs (sample)
        rng = np.random.default_rng(rank)
        for gid in rng.choice(wanted, 200, replace=False):
            ol = O.OracleLog(SEG)
            for ep in range(EPOCHS):
                b = content(int(gid), ep, table.ids[gid].is_main)
                assert ol.upstream(b, 0, ep) == 0
            lg = rep.replica_handle[gid]
            assert ThreadCausalLog(eng, int(lg), table.ids[gid]).state() == ol.state()
        # replay-prep merge across the ranks: failed vertices 3 (stage 0) and 131 (stage 1),
        # a connected pair; rank r's copies are its owned logs or replicas
        failed = [3, 131]
        dest_of = {3: 1 % world, 131: 0}
        fg = np.nonzero(np.isin(table.vertex, failed))[0]
        copies = {}
        for gid in fg:
            h = owned.get(int(gid), -1)
            if h < 0:
                h = int(rep.replica_handle[gid])
            if h >= 0:
                copies[int(gid)] = h
        # the owner of vertex 3 logged one more epoch that was never replicated: its copies
        # are the longest and must win
        extra = {}
        for gid in fg:
            if int(table.vertex[gid]) == 3 and int(gid) in owned:
                b = content(int(gid), EPOCHS, table.ids[gid].is_main)
                ThreadCausalLog(eng, owned[int(gid)], table.ids[gid]).processUpstreamDelta(b, 0, EPOCHS)
        for gid in fg:
            if int(table.vertex[gid]) == 3:
                extra[int(gid)] = content(int(gid), EPOCHS, table.ids[gid].is_main)
        mc = X.merge_responses(X.EngineIO(eng), table, failed, copies, {3: 0, 131: 0}, dest_of, dev)
        merged = mc.as_dict()
        for gid in fg:
            v = int(table.vertex[gid])
            if dest_of[v] != rank:
                assert int(gid) not in merged
                continue
            want = b"".join(content(int(gid), ep, table.ids[gid].is_main) for ep in range(EPOCHS))
            assert merged.get(int(gid)) == want + extra.get(int(gid), b""), (rank, int(gid))
        # replay preparation on each failed vertex's destination rank, straight from the merge's
        # receive buffer (device input: the winners never pass through the host)
        from clonos_amd.replay import merged_response, prepare_replay
        import response_ref as R
        mine = [v for v in failed if dest_of[v] == rank]
        if mine:
            mcd = X.MergedCopies(mc.buf if mc.buf.is_cuda else mc.buf.to(dev), gids=mc.gids, offs=mc.offs, lens=mc.lens)  # gloo: lift to HBM
            jobs, sub_gids = [], []
            for v in mine:
                sg = [int(g) for g in fg if int(table.vertex[g]) == v and not table.ids[g].is_main]
                sub_gids.append(sg)
                jobs.append((v, merged_response(v, mcd, table), [table.ids[g] for g in sg]))
            main, res = prepare_replay(eng, jobs, device_input=True)
            for i, v in enumerate(mine):
                gm = [int(g) for g in fg if int(table.vertex[g]) == v and table.ids[g].is_main][0]
                st_, r, _, _ = O.decode(merged[gm])
                assert st_ == 0
                sl = main.span_slice(i)
                assert (main.tag[sl] == r["tag"]).all() and (main.v0[sl] == r["v0"]).all()
                assert (main.off[sl] == r["off"]).all() and sl.stop - sl.start == len(r["tag"])
                assert len(res[i].subpartitions) == PAR
                for sp, g in zip(res[i].subpartitions, sub_gids[i]):
                    assert sp.status == _lib.CLG_OK
                    assert sp.buffer_sizes.tolist() == R.buffer_sizes(merged[g]), (rank, g)
        # checkpoint completion afterwards: the job's CAS + truncation of owned logs and replicas
        assert eng.truncate_all(2)
        for gid in rng.choice(wanted, 50, replace=False):
            ol = O.OracleLog(SEG)
            for ep in range(EPOCHS):
                assert ol.upstream(content(int(gid), ep, table.ids[gid].is_main), 0, ep) == 0
            assert ol.checkpoint_complete(2) == 0
            assert ThreadCausalLog(eng, int(rep.replica_handle[gid]), table.ids[gid]).state() == ol.state()
        dist.barrier()
        dist.destroy_process_group()
        eng.close()
        q.put((rank, "ok", (len(wanted), n_bytes, stats[0].sent_bytes)))
    except Exception:
        import traceback
        q.put((rank, "fail", traceback.format_exc()))


if __name__ == "__main__":
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    procs = [ctx.Process(target=worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = [q.get(timeout=300) for _ in procs]
    for p in procs:
        p.join(timeout=60)
    bad = [r for r in res if r[1] != "ok"]
    for r in bad:
        print(r[2], file=sys.stderr)
    print("replicas verified:", [r[2] for r in res if r[1] == "ok"])
    sys.exit(1 if bad else 0)
