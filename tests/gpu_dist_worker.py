"""Launcher for tests/test_gpu_dist.py: two ranks (gloo), one Engine each on cuda:0,
replicating owned logs with clonos_amd.dist over real engines.  The launcher itself never
touches the GPU; each rank is a fresh process."""
import os
import socket
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
sys.path.insert(0, os.path.dirname(HERE))
import test_dist_cpu as T  # noqa: E402  (log ids and deterministic contents)


def worker(rank, world, port, q):
    try:
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        import torch
        import torch.distributed as dist
        from clonos_amd import Engine
        from clonos_amd import dist as X
        from clonos_amd.job import owner_rank
        dist.init_process_group("gloo", rank=rank, world_size=world)
        dev = torch.device("cuda", 0)
        eng = Engine(segment_bytes=T.SEG, pool_segments=1 << 14, device=0)
        mine = [cid for cid in T.log_ids() if owner_rank(cid.vertex_id, world) == rank]
        owned = [eng.open_log(cid) for cid in mine]
        wanted = {v for v in range(T.N_VERT) if owner_rank(v, world) != rank and v != 1}
        io = X.EngineIO(eng, dev)
        rep = X.Replicator(io, rank, world, wanted)
        for ep in range(T.EPOCHS):
            for half in range(2):
                for lg in owned:
                    r = T.records(lg.cid, ep)
                    part = r[:len(r) // 2] if half == 0 else r[len(r) // 2:]
                    if part:
                        lg.processUpstreamDelta(part, len(r) // 2 if half else 0, ep)
                rep.exchange(owned, ep)
        got = 0
        for cid in T.log_ids():
            if cid.vertex_id not in wanted:
                continue
            expect = b"".join(T.records(cid, ep) for ep in range(T.EPOCHS))
            lg = io.replicas.get(cid.key())
            have = lg.getDeterminants(0) if lg is not None else b""
            assert have == expect, (rank, cid, len(have), len(expect))
            got += 1
        dist.barrier()
        dist.destroy_process_group()
        eng.close()
        q.put((rank, "ok", got))
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
    print("replicas verified:", sum(r[2] for r in res if r[1] == "ok"))
    sys.exit(1 if bad else 0)
