"""bench.py -- determinants/sec for decode + per-channel delta slice (BASELINE.json metric).

Workload (BASELINE.json configs[1], SURVEY.md 8d "Config 2"), per GPU:
  64 subtask logs x 1M Order+Timestamp determinants in one epoch (~352 MB resident in HBM
  segments), 8 downstream consumers per log positioned at random record boundaries.
One step = GPU decode of all 64 logs (getDeterminants spans, SoA output in HBM) +
batched delta slice for all 512 (consumer, log) pairs (packed output in HBM).
Multi-GPU: logs shard by vertex across ranks (weak scaling), no data-path collective.

Prints ONE JSON line on rank 0 (contract in the task description), with a `roofline`
object for the dominant kernel (HIP-event durations measured inside the engine on the
stream the kernels run on) and a `cpu_baseline` object (the C++ oracle on host cores).
"""
from __future__ import annotations

import argparse
import ctypes as C
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

N_LOGS = 64
N_REC = 1_000_000
N_CONS = 8
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec peak (MI355X_MICROARCH.md: 8.0 TB/s)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--logs", type=int, default=N_LOGS)
    ap.add_argument("--records", type=int, default=N_REC)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-threads", type=int, default=0)
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    ap.add_argument("--no-config3", action="store_true", help="skip the secondary config-3 decode measurement")
    ap.add_argument("--no-inflight", action="store_true", help="skip the secondary in-flight log replay measurement")
    ap.add_argument("--inflight-only", action="store_true",
                    help="profiling aid: run only the in-flight replay leg and print its JSON object")
    ap.add_argument("--no-isolated", action="store_true", help="skip the isolated per-kernel pass (profiling runs)")
    ap.add_argument("--no-config4", action="store_true", help="skip the config-4 replication leg")
    ap.add_argument("--config4-only", action="store_true",
                    help="profiling aid: run only the config-4 leg and print its JSON object")
    ap.add_argument("--config4-steps", type=int, default=6)
    ap.add_argument("--config5-steps", type=int, default=4)
    ap.add_argument("--no-config1", action="store_true", help="skip the config-1 latency leg")
    return ap.parse_args()


def spawn(args) -> int:
    """`bench.py --gpus N` outside torch.distributed.run: N fresh child processes, rank r on
    GPU r (CLONOS_BENCH_REHEARSAL=1: all on GPU 0 over gloo), the same arguments, with
    RANK / LOCAL_RANK / WORLD_SIZE / MASTER_* set.  This parent never touches the GPU: it
    only waits, and ends the others if one rank fails."""
    import socket
    import subprocess
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    procs = []
    for r in range(args.gpus):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(args.gpus), LOCAL_WORLD_SIZE=str(args.gpus),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), HSA_ENABLE_IPC_MODE_LEGACY="0")
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:], env=env))
    rc = 0
    while procs:
        for p in list(procs):
            r = p.poll()
            if r is None:
                continue
            procs.remove(p)
            if r != 0 and rc == 0:
                rc = r
                for q in procs:  # the others would wait in a collective forever
                    q.terminate()
        time.sleep(0.05)
    return rc


def main():
    args = parse()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(spawn(args))
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    import torch
    import torch.distributed as dist

    # CLONOS_BENCH_REHEARSAL=1: every rank on cuda:0 with gloo, to rehearse the N>1 path on a
    # one-GPU box (numbers meaningless); the real multi-GPU run is one rank per GPU over RCCL
    rehearse = os.environ.get("CLONOS_BENCH_REHEARSAL") == "1"
    if rehearse:
        local = 0
    torch.cuda.set_device(local)
    if world > 1:
        os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
        if rehearse:
            dist.init_process_group("gloo")
        else:
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))

    from clonos_amd import CausalLogID, Engine, _lib, synth

    if args.inflight_only:
        print(json.dumps(inflight_replay(args, torch, torch.device("cuda", local))), flush=True)
        return
    if args.config4_only:
        c4, c5 = config4(args, torch, torch.device("cuda", local), rank, world, dist, rehearse)
        if rank == 0:
            print(json.dumps({"config4": c4, "config5": c5}), flush=True)
        if world > 1:
            dist.destroy_process_group()
        return

    # ---------------- synthetic shard (seeded per rank) ----------------
    rng = np.random.default_rng(synth.SEED_CONFIG2 + rank)
    bufs, offs = [], []
    for _ in range(args.logs):
        b, o = synth.config2_log(args.records, rng)
        bufs.append(b)
        offs.append(o)
    log_bytes = [int(b.size) for b in bufs]
    total_bytes = sum(log_bytes)
    seg = 16384
    pool = sum((n + seg - 1) // seg + 1 for n in log_bytes) + 64
    timing = os.environ.get("CLONOS_BENCH_TIMING") != "0"  # developer switch: 0 = no kernel timing events (A/B)
    eng = Engine(segment_bytes=seg, pool_segments=pool, device=local, timing=timing, async_slice=True,
                 ifl_pool_segments=16)
    logs = []
    for v, b in enumerate(bufs):
        vid = rank * args.logs + v  # VertexID sharding: this rank owns its vertices
        log = eng.open_log(CausalLogID.main(vid))
        log.processUpstreamDelta(b.tobytes(), 0, 1)  # one epoch, received whole
        logs.append(log)
    eng.sync()

    # consumers at random record boundaries
    cons = []  # (log index, channel, offset)
    for i, o in enumerate(offs):
        for c in range(N_CONS):
            r = int(rng.integers(0, len(o)))
            cons.append((i, (c + 1, rank * args.logs + i), int(o[r])))
    slice_total = sum(log_bytes[i] - off for i, _, off in cons)
    n_req = len(cons)
    creq = (_lib.SliceReq * n_req)()
    cres = (_lib.SliceRes * n_req)()
    for k, (i, ch, _) in enumerate(cons):
        creq[k].log = logs[i].handle
        creq[k].consumer = _lib.ChannelId(ch[0], ch[1])
        creq[k].epoch = 1

    # ---------------- device outputs (HBM, caller-owned) ----------------
    # two output sets: decode i+1 is queued before decode i is completed (two in flight,
    # CLG_DECODE_MAX_INFLIGHT), so neither stream waits for the host between steps
    n_det = args.logs * args.records
    dev = torch.device("cuda", local)
    depth = 1 if os.environ.get("CLONOS_BENCH_PIPELINE") == "0" else 2  # developer switch: 1 = one decode at a time
    wcap = 1024
    outs = []
    for _ in range(depth):
        o_off = torch.empty(n_det, dtype=torch.int32, device=dev)
        o_tag = torch.empty(n_det, dtype=torch.uint8, device=dev)
        o_v0 = torch.empty(n_det, dtype=torch.int64, device=dev)
        o_w = [torch.empty(wcap, dtype=t, device=dev) for t in
               (torch.int32, torch.int32, torch.int64, torch.int32, torch.int32, torch.uint8)]
        d = _lib.Decoded()
        d.off, d.tag, d.v0 = o_off.data_ptr(), o_tag.data_ptr(), o_v0.data_ptr()
        d.w_idx, d.w_rc, d.w_v1, d.w_var_off, d.w_var_len, d.w_sub = [t.data_ptr() for t in o_w]
        d.cap, d.wcap, d.out_kind = n_det, wcap, _lib.CLG_MEM_DEVICE
        outs.append((d, np.zeros(len(logs) + 1, np.uint64), [o_off, o_tag, o_v0] + o_w))
    o_slice = torch.empty(slice_total + 64, dtype=torch.uint8, device=dev)
    dec, base = outs[0][0], outs[0][1]
    handles = np.array([l.handle for l in logs], np.uint32)
    starts = np.ones(len(logs), np.int64)

    seek_offs = np.array([off for _, _, off in cons], np.int32)

    host = [0.0] * 3  # host time per call over the timed steps: decode queue, seek + slice, decode wait
    state = {"k": 0, "queued": []}

    def complete_oldest():
        d = state["queued"].pop(0)
        eng.decode_wait()
        assert d.err_status == 0 and d.n_rec == n_det, (d.err_status, d.n_rec, n_det)

    def step(acc=None):
        # decode i is queued asynchronously, then the slices of step i go to the engine's
        # gather stream (they only read log segments); only then is decode i-1 completed, so
        # both streams always hold queued work while the host plans
        d, b, _ = outs[state["k"] % depth]
        state["k"] += 1
        c0 = time.perf_counter()
        if len(state["queued"]) == depth:
            complete_oldest()  # (depth 1: the previous step's decode, before this one is queued)
        c1 = time.perf_counter()
        eng.decode_logs_device_async(handles, starts, d, b)
        state["queued"].append(d)
        c2 = time.perf_counter()
        eng.seek_consumers_raw(creq, seek_offs, n_req)  # rewind the consumers to their start offsets
        got = eng.slice_batch_raw(creq, cres, n_req, o_slice.data_ptr(), o_slice.numel(), device=True)
        c3 = time.perf_counter()
        if acc is not None:
            for k, v in enumerate((c2 - c1, c3 - c2, c1 - c0)):
                acc[k] += v
        assert got == slice_total, (got, slice_total)

    def drain():
        while state["queued"]:
            complete_oldest()

    # correctness guard on the first step: record count and status
    step()
    drain()
    torch.cuda.synchronize()
    for _ in range(max(0, args.warmup - 1)):
        step()
    drain()
    eng.sync()
    torch.cuda.synchronize()
    eng.kernel_stats_reset()

    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step(host)
    c0 = time.perf_counter()
    drain()  # every decode of the K steps completed (status and count checked) inside the timed region
    host[2] += time.perf_counter() - c0
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device="cpu" if rehearse else dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    stats = eng.kernel_stats()
    # isolated pass (after the timed region): decode, then the slices, each waited for, so
    # every kernel's duration is its own (no overlap)
    eng.kernel_stats_reset()
    for _ in range(0 if args.no_isolated else min(args.steps, 5)):
        eng.decode_logs_device(handles, starts, dec, base)
        eng.seek_consumers_raw(creq, seek_offs, n_req)
        eng.slice_batch_raw(creq, cres, n_req, o_slice.data_ptr(), o_slice.numel(), device=True)
        eng.sync()
    torch.cuda.synchronize()
    iso_stats = eng.kernel_stats()

    ms_per_step = elapsed * 1e3 / args.steps
    value = n_det * world / (elapsed / args.steps)
    if not timing:  # (developer A/B: no kernel stats to report)
        print(json.dumps({"ms_per_step": round(ms_per_step, 4), "timing": False}), flush=True)
        raise SystemExit(0)

    # ---------------- roofline of the dominant kernel ----------------
    def per_kernel(st):
        out = {}
        for name, s in st.items():
            if s["launches"]:
                avg_ms = s["ms"] / s["launches"]
                per_launch = s["bytes"] / s["launches"]
                out[name] = dict(launches=s["launches"], avg_ms=round(avg_ms, 5),
                                 algo_bytes_per_launch=int(per_launch),
                                 gbs=round(per_launch / (avg_ms * 1e-3) / 1e9, 1) if avg_ms > 0 else None)
        return out
    kern, kern_iso = per_kernel(stats), per_kernel(iso_stats)
    dom = max((k for k in kern if k != "decode_pipeline" and not k.startswith("host_")),
              key=lambda k: kern[k]["avg_ms"] * kern[k]["launches"], default=None)
    roof = None
    if dom:
        ach = kern[dom]["gbs"]
        # traffic: HBM bytes per launch from the last round profile's PMC passes (not measured
        # in this run: counters need rocprofv3 --pmc), with where and when they were collected
        traffic, tsrc = None, None
        pmc_path = os.path.join(ROOT, "profiles", "pmc_traffic.json")
        if os.path.exists(pmc_path):
            try:
                pt = json.load(open(pmc_path))
                kt = pt.get("kernels", pt)
                traffic = kt.get(dom)
                tsrc = {"file": "profiles/pmc_traffic.json", "git_head": pt.get("git_head"), "date": pt.get("date"),
                        "tag": pt.get("tag"), "measured_in_this_run": False}
            except Exception:
                traffic = None
        roof = {"bound": "hbm", "kernel": dom, "achieved": ach, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": round(ach / HBM_PEAK_GBS, 4) if ach else None, "traffic": traffic, "traffic_source": tsrc}
    # decode pipeline as a whole (HIP events from its first kernel's start to emit's end, on
    # the engine's stream) against its algorithmic bytes
    dec_ms = kern_iso["decode_pipeline"]["avg_ms"] if "decode_pipeline" in kern_iso else None
    dec_bytes = total_bytes + 13 * n_det
    # the slice's algorithmic bytes: each slice read and written once, 16 B of
    # metadata per request.  Beside it the minimum traffic: every source byte some consumer
    # reads, once (per log the union of its consumers' suffixes), plus the writes -- the 8
    # consumers of a log re-read its tail, which the caches (MALL) serve in part
    slice_bytes = 2 * slice_total + 16 * n_req
    first_off = {}
    for i, _, off in cons:
        first_off[i] = min(first_off.get(i, off), off)
    slice_min_bytes = sum(log_bytes[i] - o for i, o in first_off.items()) + slice_total + 16 * n_req
    roof_iso = None
    if dom and dom in kern_iso and kern_iso[dom]["gbs"]:
        roof_iso = {"kernel": dom, "achieved": kern_iso[dom]["gbs"], "peak": HBM_PEAK_GBS, "unit": "GB/s",
                    "frac": round(kern_iso[dom]["gbs"] / HBM_PEAK_GBS, 4)}
    step_gbs = (dec_bytes + slice_bytes) / (elapsed / args.steps) / 1e9

    # ---------------- CPU baseline (rank 0, N=1 only) ----------------
    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cpu = cpu_baseline(bufs, log_bytes, cons, args)
    # ---------------- secondary: config 1 latency (rank 0, N=1 only) ----------------
    # before the larger legs: measured after config 3 and the in-flight leg in the same process,
    # its decode took 0.60 ms instead of 0.25 ms
    c1 = None
    if rank == 0 and world == 1 and not args.no_config1:
        c1 = config1(args, torch)
    # ---------------- secondary: config 3 decode (rank 0, N=1 only) ----------------
    c3 = None
    if rank == 0 and world == 1 and not args.no_config3:
        eng.close()
        del outs, o_slice, dec
        torch.cuda.empty_cache()
        c3 = config3(args, torch, dev)
    ifl = None
    if rank == 0 and world == 1 and not args.no_inflight:
        ifl = inflight_replay(args, torch, dev)
    c4 = c5 = None
    if not args.no_config4:  # every rank: the exchange is a collective
        if world == 1:
            eng.close()
        c4, c5 = config4(args, torch, dev, rank, world, dist, rehearse)

    if rank == 0:
        line = {
            "metric": "determinants/sec decode+delta-slice",
            "value": round(value, 1),
            "unit": "determinants/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms_per_step, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u8",
            "data": "synthetic (seeded config-2 generator; SURVEY.md 8d)",
            "config": {"workload": "config2: 64 subtasks x 1M Order+Timestamp determinants/epoch, decode + "
                                   "per-channel delta slice (8 consumers/log)",
                       "logs_per_gpu": args.logs, "records_per_log": args.records, "consumers_per_log": N_CONS,
                       "log_bytes_per_gpu": total_bytes, "slice_bytes_per_gpu": slice_total,
                       "segment_bytes": seg, "parallelism": f"shard-by-vertex x{world}"},
            "log_gbs": round(total_bytes * world / (elapsed / args.steps) / 1e9, 2),
            "decode_pipeline": {"avg_ms_isolated": round(dec_ms, 4) if dec_ms else None, "algo_bytes": dec_bytes,
                                "gbs": round(dec_bytes / (dec_ms * 1e-3) / 1e9, 1) if dec_ms else None},
            "step_roofline": {"note": "decode + slice algorithmic bytes / step time (slice gather overlaps the "
                                      "next decode on a second stream)", "achieved": round(step_gbs, 1),
                              "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": round(step_gbs / HBM_PEAK_GBS, 4)},
            "slice": {"algo_bytes": slice_bytes, "min_traffic_bytes": slice_min_bytes},
            "decode_path": ("robust (fast path aborted)" if "decode_fallback" in stats else
                            "three-pass (count -> scan -> emit)"),
            "decodes_in_flight": depth,
            "host_ms_per_step": {"decode_queue": round(host[0] * 1e3 / args.steps, 4),
                                 "seek_slice_queue": round(host[1] * 1e3 / args.steps, 4),
                                 "waiting_for_gpu": round(host[2] * 1e3 / args.steps, 4),
                                 "note": "host time per timed step: planning + queueing the decode, the consumer "
                                         "seeks + slice planning + gather queueing, and blocked in decode_wait "
                                         "(the GPU was busy). The host's work overlaps the GPU's: with two decodes "
                                         "in flight the GPU does not wait for it while its work is shorter than "
                                         "a step"},
            "kernels": kern,
            "kernels_isolated": kern_iso,
            "roofline": roof,
            "roofline_isolated": roof_iso,
            "cpu_baseline": cpu,
            "config3": c3,
            "inflight_replay": ifl,
            "config4": c4,
            "config5": c5,
            "config1": c1,
            "distributed": dist_info(torch, dist, world, rehearse),
        }
        print(json.dumps(line), flush=True)
    eng.close()
    if world > 1:
        dist.destroy_process_group()


def dist_info(torch, dist, world, rehearse):
    """What the process group was, so a scaling record shows how many ranks the collectives
    saw: torch.distributed's world size and backend ("nccl" is RCCL on ROCm), and the RCCL
    version torch was built against."""
    info = {"world_size": dist.get_world_size() if dist.is_initialized() else world,
            "backend": dist.get_backend() if dist.is_initialized() else None,
            "transport": "gloo rehearsal (every rank on GPU 0)" if rehearse else
                         ("RCCL over xGMI" if world > 1 else "one rank (no collective in the config-2 step)"),
            "rccl_version": None, "hip_version": getattr(torch.version, "hip", None)}
    try:
        v = torch.cuda.nccl.version()
        info["rccl_version"] = ".".join(str(x) for x in v) if isinstance(v, tuple) else str(v)
    except Exception as e:  # (reported, not fatal: the version is a label)
        info["rccl_version"] = f"unavailable: {type(e).__name__}"
    return info


def config4(args, torch, dev, rank, world, dist, rehearse, main_records=4096, sub_records=64):
    """BASELINE.json configs[3]: full sharing depth on a 5-stage DAG at parallelism 128
    (640 VertexIDs; per producing vertex 1 main + 128 subpartition logs; 66 176 logs), logs
    sharded by VertexID across the ranks (job.owner_rank).  One step, on every rank:
      1. the new epoch of every owned log lands in HBM (batched device-input append);
      2. batched decode of that epoch of every owned log (SoA in HBM);
      3. replication (dist.Replicator.exchange): batched slice of the new bytes of every
         owned log for every rank that wants it -> all-to-alls over RCCL (counts, header
         rows, payload) -> batched device-input processUpstreamDelta into the replicas;
      4. checkpoint completion of the previous epoch (job CAS + truncation of owned logs and
         replicas).
    At N=1 every log is local: the replication has nothing to move and runs no collective.  Timing: K steps between barriers + device syncs, max over ranks."""
    import time as _t
    from clonos_amd import Engine, _lib, job as J, synth, dist as X
    own_group = None
    if world == 1:  # a one-rank group so the exchange's collectives run (and are timed)
        if not dist.is_initialized():
            os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
            os.environ.setdefault("MASTER_PORT", str(29500 + (os.getpid() % 2000)))
            dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
            own_group = True
    g = J.dag(5, 128)
    table = J.LogTable(g)
    need = J.replication_masks(g, -1, world)
    plan = X.ReplicationPlan(table, -1, rank, world, need)
    rng = np.random.default_rng(synth.SEED_CONFIG4 + rank)
    gids = plan.owned
    host, offs = synth.config4_epoch(table, gids, rng, main_records, sub_records)
    seg = 16384
    per_log = np.diff(offs).astype(np.int64)
    segs = int(((2 * per_log + seg - 1) // seg + 2).sum())
    # replicas: the owners' epoch sizes are the same shapes (main / subpartition)
    main_b = int(per_log[[table.ids[int(x)].is_main for x in gids]].max()) if len(gids) else 0
    sub_b = sub_records * 5
    rep_segs = sum(((2 * (main_b if table.ids[int(x)].is_main else sub_b) + seg - 1) // seg + 2)
                   for x in plan.wanted)
    eng = Engine(segment_bytes=seg, pool_segments=segs + rep_segs + 64, device=dev.index or 0, timing=True,
                 ifl_pool_segments=16)
    owned = {int(x): eng.open_log(table.ids[int(x)]).handle for x in gids}
    sendset = set(plan.send.tolist())
    rep = X.Replicator(X.EngineIO(eng), plan, dev, {k: v for k, v in owned.items() if k in sendset})
    d_epoch = torch.from_numpy(host).to(dev)
    areq = np.zeros(len(gids), X.DELTA_REQ)
    areq["log"] = [owned[int(x)] for x in gids]
    areq["src_off"] = offs[:-1]
    areq["len"] = per_log
    handles = np.array([owned[int(x)] for x in gids], np.uint32)
    n_rec = int(sum(main_records if table.ids[int(x)].is_main else sub_records for x in gids))
    o = [torch.empty(max(n_rec, 1), dtype=t, device=dev) for t in (torch.int32, torch.uint8, torch.int64)]
    ow = [torch.empty(16, dtype=t, device=dev) for t in
          (torch.int32, torch.int32, torch.int64, torch.int32, torch.int32, torch.uint8)]
    dec = _lib.Decoded()
    dec.off, dec.tag, dec.v0 = [t.data_ptr() for t in o]
    dec.w_idx, dec.w_rc, dec.w_v1, dec.w_var_off, dec.w_var_len, dec.w_sub = [t.data_ptr() for t in ow]
    dec.cap, dec.wcap, dec.out_kind = max(n_rec, 1), 16, _lib.CLG_MEM_DEVICE
    base = np.zeros(len(gids) + 1, np.uint64)
    bytes_owned = int(host.size)
    # every request slices at most one epoch of its log (the bench appends one per step)
    len_of = dict(zip(gids.tolist(), per_log.tolist()))
    payload_cap = int(sum(len_of[int(x)] for x in plan.req_gid)) + 64
    phase = {"append": 0.0, "decode": 0.0, "exchange": 0.0, "truncate": 0.0}
    ex_tot = X.ExchangeStats()

    areq_epoch = areq["epoch"]  # (a view: the per-step epoch goes in place; the engine writes every status)
    starts = np.zeros(len(gids), np.int64)  # (reused: a fresh array each step cost its page faults)
    areq_ptr, d_epoch_ptr = areq.ctypes.data, d_epoch.data_ptr()

    def step(e, timed):
        t0 = _t.perf_counter()
        areq_epoch.fill(e)
        _lib.check(_lib.lib.clg_upstream_delta_batch(eng.handle, areq_ptr, len(areq), d_epoch_ptr, _lib.CLG_MEM_DEVICE))
        t1 = _t.perf_counter()
        starts.fill(e)
        eng.decode_logs_device(handles, starts, dec, base)
        assert dec.n_rec == n_rec and dec.err_status == 0, (dec.n_rec, n_rec)
        t2 = _t.perf_counter()
        st = rep.exchange(e, payload_cap)
        t3 = _t.perf_counter()
        if e > 0:
            assert eng.truncate_all(e)
        t4 = _t.perf_counter()
        if timed:
            for k, v in zip(phase, (t1 - t0, t2 - t1, t3 - t2, t4 - t3)):
                phase[k] += v
            for f in ("sent_bytes", "recv_bytes", "applied", "applied_bytes", "skipped"):
                setattr(ex_tot, f, getattr(ex_tot, f) + getattr(st, f))

    warm = 2
    for e in range(warm):
        step(e, False)
    torch.cuda.synchronize()
    eng.kernel_stats_reset()
    dist.barrier()
    torch.cuda.synchronize()
    t0 = _t.perf_counter()
    K = args.config4_steps
    for e in range(warm, warm + K):
        step(e, True)
    torch.cuda.synchronize()
    dist.barrier()
    el = _t.perf_counter() - t0
    tt = torch.tensor([el], dtype=torch.float64, device="cpu" if rehearse else dev)
    dist.all_reduce(tt, op=dist.ReduceOp.MAX)
    el = float(tt.item())
    tot = torch.tensor([n_rec, bytes_owned, ex_tot.applied_bytes, ex_tot.sent_bytes], dtype=torch.float64,
                       device="cpu" if rehearse else dev)
    dist.all_reduce(tot, op=dist.ReduceOp.SUM)
    tot_rec, tot_bytes, tot_applied, tot_sent = [float(x) for x in tot.cpu()]
    st = eng.kernel_stats()
    kern = {k: dict(launches=v["launches"], avg_ms=round(v["ms"] / v["launches"], 5),
                    gbs=round(v["bytes"] / v["launches"] / (v["ms"] / v["launches"] * 1e-3) / 1e9, 1)
                    if v["ms"] > 0 else None) for k, v in st.items() if v["launches"]}
    c5 = config5(args, torch, dev, rank, world, dist, rehearse, eng, table, plan, rep, owned, areq, d_epoch,
                 warm + K)
    eng.close()
    if own_group:
        dist.destroy_process_group()
    ms = el * 1e3 / K
    return ({"workload": "config4: 5-stage DAG, p=128, full sharing (640 VertexIDs, 66176 logs: 1 main + 128 "
                        f"subpartition logs per producing vertex); per epoch {main_records} Order/Timestamp per main "
                        f"log, {sub_records} BufferBuilt per subpartition log; step = append + decode of owned logs "
                        "+ replication exchange (slice -> all-to-all -> processUpstreamDelta) + truncation",
            "n_gpus": world, "steps": K, "ms_per_step": round(ms, 4),
            "determinants_per_s": round(tot_rec / (el / K), 1), "log_gbs": round(tot_bytes / (el / K) / 1e9, 2),
            "logs_per_rank": {"owned": len(gids), "sent": int(len(plan.send)), "replicas": int(len(plan.wanted))},
            "exchange": {"sent_bytes_per_step_all_ranks": int(tot_sent / K),
                         "applied_bytes_per_step_all_ranks": int(tot_applied / K),
                         "applied_deltas_per_step_rank0": int(ex_tot.applied / K),
                         "replicated_gbs": round(tot_applied / el / 1e9, 2)},
            "phase_ms_rank0": {k: round(v * 1e3 / K, 3) for k, v in phase.items()},
            "kernels_rank0": kern,
            "transport": "gloo rehearsal" if rehearse else "RCCL (nccl backend)"}, c5)


def failed_vertices(graph, rng, k=16):
    """16 failed subtasks spread over the stages, including connected (adjacent-stage) pairs
    (BASELINE config 5: concurrent and connected failures)."""
    p = graph.vertices[0].parallelism
    n = len(graph.vertices) * p
    pairs = [(s * p + int(rng.integers(0, p)), (s + 1) * p + int(rng.integers(0, p))) for s in range(len(graph.vertices) - 1)]
    out = sorted({v for pr in pairs for v in pr})
    rest = [v for v in range(n) if v not in out]
    out += [int(x) for x in rng.choice(rest, size=k - len(out), replace=False)]
    return sorted(out)


def config5(args, torch, dev, rank, world, dist, rehearse, eng, table, plan, rep, owned, areq, d_epoch, e0):
    """BASELINE.json configs[4]: concurrent / connected failures of 16 subtasks of config 4's
    job, on the ranks that hold config 4's logs and replicas.  One step (epoch e):
      * (untimed) the owners append epoch e, so owners' copies are longer than the replicas'
        (copies of one log on several GPUs with different lengths);
      * merge: every rank's copies of the failed vertices' logs (getDeterminants(e - 1), the
        request's start epoch) are measured in one call, all-reduce(MAX) picks the longest
        (DeterminantResponseEvent.merge :128-148), the winners are gathered in one call and
        moved by one all-to-all to the rank hosting each replacement (dist.merge_responses);
      * replay-prep on each destination straight from the receive buffer in HBM
        (clg_replay_prepare_device): main logs decoded in one batch (LogReplayerImpl's
        sequence), subpartition logs turned into BufferBuilt size lists (ReplayingState
        :157-214);
      * (untimed) replication of epoch e, then checkpoint completion of e on every rank:
        job CAS + truncation of every owned log and replica (JobCausalLogImpl :230-246).
    Latency = merge + replay-prep + truncation, max over ranks; GB/s = winners' bytes / the
    merge + replay-prep time.  The first step is checked against the oracle's decode and
    BufferBuilt sizes of the merged bytes."""
    import time as _t
    from clonos_amd import _lib, dist as X, job as J
    from clonos_amd.replay import merged_responses, prepare_replay_raw, table_ids
    g = table.graph
    failed = failed_vertices(g, np.random.default_rng(0xC1050005))
    dest_of = {v: J.owner_rank(v, world) for v in failed}
    fg = table.gids_of(failed)
    copies = {}
    for gid in fg:
        h = owned.get(int(gid), -1)
        if h < 0:
            h = int(rep.replica_handle[gid])
        if h >= 0:
            copies[int(gid)] = h
    copies_arr = X.copy_arrays(copies)  # (once: the merge takes the arrays every step)
    mine = [v for v in failed if dest_of[v] == rank]
    subs_of = {v: [int(x) for x in fg if int(table.vertex[x]) == v and not table.ids[x].is_main] for v in mine}
    ids = table_ids(table)
    sub_tab = {v: ids[np.array(subs_of[v], np.int64)] for v in mine}  # the tasks' subpartition tables
    io = X.EngineIO(eng)
    ph = {"merge": 0.0, "replay_prep": 0.0, "truncate": 0.0}
    sub = {"responses": 0.0, "prepare": 0.0}  # replay_prep's parts: the merged events, clg_replay_prepare_device
    mt = {}  # merge's parts (rank 0): copy lengths, the winners' gather
    pt = {}  # prepare's parts (rank 0): Python build, output allocation, the C call, result arrays
    win_bytes, n_main_rec, n_sizes = 0, 0, 0
    sync = torch.cuda.synchronize
    steps = args.config5_steps
    for it in range(steps + 1):
        e = e0 + it
        areq["epoch"] = e
        areq["status"] = 0
        _lib.check(_lib.lib.clg_upstream_delta_batch(eng.handle, areq.ctypes.data, len(areq), d_epoch.data_ptr(),
                                                     _lib.CLG_MEM_DEVICE))
        eng.sync()
        dist.barrier()
        t0 = _t.perf_counter()
        mc = X.merge_responses(io, table, failed, copies_arr, {v: e - 1 for v in failed}, dest_of, dev, timing=mt)
        sync()
        t1 = _t.perf_counter()
        ra = None
        if mine:
            mcd = mc if mc.buf.is_cuda else X.MergedCopies(mc.buf.to(dev), gids=mc.gids, offs=mc.offs, lens=mc.lens)
            accs = merged_responses(mcd, table, mine)
            t1b = _t.perf_counter()
            ra = prepare_replay_raw(eng, [(v, accs[v], sub_tab[v]) for v in mine], device_input=True, timing=pt)
            sub["responses"] += t1b - t1
            sub["prepare"] += _t.perf_counter() - t1b
        t2 = _t.perf_counter()
        rep.exchange(e)
        eng.sync()
        dist.barrier()
        t3 = _t.perf_counter()
        assert eng.truncate_all(e)
        t4 = _t.perf_counter()
        if it == 0:  # correctness: the oracle's decodeNext / BufferBuilt sizes of the merged bytes
            sys.path.insert(0, os.path.join(ROOT, "tests"))
            sys.path.insert(0, os.path.join(ROOT, "oracle"))
            import _oracle as O  # the checker
            import response_ref as R  # the checker
            merged = mc.as_dict()
            j = 0
            for i, v in enumerate(mine):
                gm = [int(x) for x in fg if int(table.vertex[x]) == v and table.ids[x].is_main][0]
                st_, r, _, _ = O.decode(merged.get(gm, b""))
                sl = ra.main.span_slice(i)
                assert st_ == 0 and sl.stop - sl.start == len(r["tag"]) and (ra.main.v0[sl] == r["v0"]).all()
                for x in subs_of[v]:
                    b0 = int(ra.base[j])
                    got = ra.sizes[b0:b0 + int(ra.count[j])].tolist()
                    assert ra.status[j] == 0 and got == R.buffer_sizes(merged.get(x, b""))
                    j += 1
            eng.kernel_stats_reset()  # (the timed steps' kernels and host stages below)
            sub = {k: 0.0 for k in sub}
            mt.clear()
            pt.clear()
            continue
        ph["merge"] += t1 - t0
        ph["replay_prep"] += t2 - t1
        ph["truncate"] += t4 - t3
        win_bytes += int(mc.lens.sum())
        if ra is not None:
            n_main_rec += int(ra.main.n_rec)
            n_sizes += int(ra.count.sum())
    c5_stats = eng.kernel_stats()
    dev_t = "cpu" if rehearse else dev
    mx = torch.tensor([ph["merge"], ph["replay_prep"], ph["truncate"], ph["merge"] + ph["replay_prep"] + ph["truncate"]],
                      dtype=torch.float64, device=dev_t)
    dist.all_reduce(mx, op=dist.ReduceOp.MAX)
    tot = torch.tensor([win_bytes, n_main_rec, n_sizes], dtype=torch.float64, device=dev_t)
    dist.all_reduce(tot, op=dist.ReduceOp.SUM)
    m_ms, r_ms, t_ms, all_ms = [float(x) * 1e3 / steps for x in mx.cpu()]
    wb, nm, nsz = [float(x) / steps for x in tot.cpu()]
    return {"workload": "config5: 16 failed subtasks of config 4's job (connected pairs across all stage "
                        "boundaries + random), copies on every rank holding the log (owners one epoch longer); "
                        "step = cross-GPU merge (all-reduce MAX + all-to-all) + batched replay-prep from the "
                        "receive buffer in HBM + checkpoint-complete truncation of every log on every rank",
            "n_gpus": world, "steps": steps, "failed_vertices": failed,
            "latency_ms": round(all_ms, 4),
            "phase_ms_max_over_ranks": {"merge": round(m_ms, 4), "replay_prep": round(r_ms, 4),
                                        "truncate": round(t_ms, 4)},
            "replay_prep_parts_ms_rank0": {k: round(v * 1e3 / steps, 4) for k, v in sub.items()},
            "merge_parts_ms_rank0": {k: round(v * 1e3 / steps, 4) for k, v in mt.items()},
            "prepare_parts_ms_rank0": {k: round(v * 1e3 / steps, 4) for k, v in pt.items()},
            "winner_bytes_per_step": int(wb), "main_records_per_step": int(nm), "buffer_sizes_per_step": int(nsz),
            "replay_gbs": round(wb / ((m_ms + r_ms) * 1e-3) / 1e9, 3) if m_ms + r_ms > 0 else None,
            "kernels_rank0": {k: dict(launches=v["launches"], avg_ms=round(v["ms"] / v["launches"], 5))
                              for k, v in c5_stats.items() if v["launches"]},
            "transport": "gloo rehearsal" if rehearse else "RCCL (nccl backend)"}


def config1(args, torch, steps=20):
    """BASELINE.json configs[0]: WordCount + causal TimeService / processing-time window,
    parallelism 4, sharing depth 1, one epoch (synth.config1_job, modelled from the
    reference's producer call sites).  Latency of the two batched operations a recovery and
    a steady-state buffer flush need: every producer->consumer channel's delta of the epoch
    (depth 1: each consumer gets its direct producers' logs; the consumers are rewound
    between steps) and the batched decode of every log.  Host outputs: the sizes are KBs."""
    import time as _t
    from clonos_amd import Engine, _lib, synth
    rng = np.random.default_rng(synth.SEED_CONFIG1)
    graph, data = synth.config1_job(rng)
    eng = Engine(segment_bytes=16384, pool_segments=4096, sharing_depth=1, timing=False, ifl_pool_segments=16)
    logs = {lid: eng.open_log(lid) for lid in data}
    for lid, b in data.items():
        logs[lid].appendDeterminant(b, 0)
    reqs = []
    for prod, cons in (("source", "window"), ("window", "sink")):
        for p in graph.vertex_ids(prod):
            for c in graph.vertex_ids(cons):
                for lid in data:
                    if lid.vertex_id == p:
                        reqs.append((logs[lid], (p << 16 | c, 0xC1), 0))
    n_req = len(reqs)
    creq = (_lib.SliceReq * n_req)()
    cres = (_lib.SliceRes * n_req)()
    for k, (lg, ch, ep) in enumerate(reqs):
        creq[k].log, creq[k].consumer, creq[k].epoch = lg.handle, _lib.ChannelId(*ch), ep
    out = np.empty(sum(len(b) for b in data.values()) * 4 + 64, np.uint8)
    lids = list(data)
    handles = np.array([logs[l].handle for l in lids], np.uint32)
    zeros = np.zeros(n_req, np.int32)
    t_slice = t_dec = 0.0
    n_rec = 0
    for it in range(steps + 2):
        t0 = _t.perf_counter()
        if it:
            eng.seek_consumers_raw(creq, zeros, n_req)  # the consumers back at the epoch start
        got = eng.slice_batch_raw(creq, cres, n_req, out.ctypes.data, out.size, device=False)
        t1 = _t.perf_counter()
        dec = eng.decode_logs([logs[l] for l in lids], [0] * len(lids))
        t2 = _t.perf_counter()
        if it >= 2:
            t_slice += t1 - t0
            t_dec += t2 - t1
        n_rec = int(dec.n_rec)
    eng.close()
    log_bytes = sum(len(b) for b in data.values())
    res = {"workload": "config1: WordCount + causal TimeService/processing-time window, p=4, sharing depth 1, one "
                       "epoch (modelled from the reference's producer call sites); per step every channel's delta "
                       "(seek + batched slice) and the batched decode of every log, host outputs",
           "logs": len(data), "log_bytes": log_bytes, "determinants": n_rec, "slice_requests": n_req,
           "slice_bytes": int(got), "steps": steps,
           "slice_latency_ms": round(t_slice * 1e3 / steps, 4), "decode_latency_ms": round(t_dec * 1e3 / steps, 4)}
    if not args.no_cpu_baseline:  # the C++ oracle's decodeNext loop over the same logs, one thread
        sys.path.insert(0, os.path.join(ROOT, "tests"))
        import _oracle as O  # the checker, timed here as the CPU baseline
        host = np.frombuffer(b"".join(data[l] for l in lids), np.uint8)
        lens = np.array([len(data[l]) for l in lids], np.uint64)
        offs = np.zeros(len(lids), np.uint64)
        offs[1:] = np.cumsum(lens)[:-1]
        reps, t0 = 0, _t.perf_counter()
        while _t.perf_counter() - t0 < 1.0 or reps == 0:
            O.lib.orc_bench_decode(O.ptr(host), O.ptr(offs), O.ptr(lens), len(lids), 1)
            reps += 1
        dt = (_t.perf_counter() - t0) / reps
        res["cpu_baseline"] = {"value": round(dt * 1e3, 4), "unit": "ms per decode of every log", "cores": 1,
                               "kind": "port", "sample": f"oracle decode of the {len(lids)} logs x{reps}"}
    return res


def inflight_replay(args, torch, dev, n_sub=256, n_epochs=4, per_epoch=8, buf_bytes=32768, steps=5):
    """in-flight (data) log replay.  n_sub subpartition logs, each holding
    per_epoch network buffers (32 KiB, the default memory segment) per epoch in HBM; one step
    = getInFlightIterator(1, 1) + drain for every subpartition (a recovering downstream
    replays from epoch 1 after skipping one buffer), gathered into one device buffer by one
    kernel.  Algorithmic bytes: 2 x replayed bytes (read + packed write)."""
    import time as _t
    from clonos_amd import Engine, inflight as IF
    rng = np.random.default_rng(0xC105_0F40)
    seg = 16384
    segs = n_sub * n_epochs * per_epoch * ((buf_bytes + seg - 1) // seg)
    eng = Engine(segment_bytes=seg, pool_segments=64, ifl_segment_bytes=seg, ifl_pool_segments=segs + 64, timing=True)
    logs = [IF.InFlightLog(eng) for _ in range(n_sub)]
    pat = rng.integers(0, 256, buf_bytes + 4096, dtype=np.uint8).tobytes()
    for e in range(n_epochs):  # one batched log() call per epoch; ragged tail buffers
        items = []
        for i, f in enumerate(logs):
            for k in range(per_epoch):
                n = buf_bytes if k < per_epoch - 1 else 1 + (i * 977 + e * 131) % buf_bytes
                o = (i * 31 + k * 7 + e) % 4096
                items.append((f, e, pat[o:o + n]))
        IF.log_batch(eng, items)
    reqs = IF.make_requests([(f, 1, 1) for f in logs])
    st, cres, _, sizes, total, nbuf = IF.replay_batch_raw(eng, reqs, out=np.zeros(1, np.uint8))
    out = torch.empty(total, dtype=torch.uint8, device=dev)
    sizes = np.zeros(nbuf, np.uint32)  # caller-sized outputs: one engine call per step
    for _ in range(2):
        st, *_ = IF.replay_batch_raw(eng, reqs, out=out.data_ptr(), cap=total, sizes=sizes)
        assert st == 0
    torch.cuda.synchronize()
    eng.kernel_stats_reset()
    t0 = _t.perf_counter()
    for _ in range(steps):
        IF.replay_batch_raw(eng, reqs, out=out.data_ptr(), cap=total, sizes=sizes)
    torch.cuda.synchronize()
    el = (_t.perf_counter() - t0) / steps
    k = eng.kernel_stats().get("ifl_gather", {})
    kms = k["ms"] / k["launches"] if k.get("launches") else None
    # spot check against the logged bytes: the first replayed buffer of subpartition 0
    first = pat[(0 * 31 + 1 * 7 + 1) % 4096:][:buf_bytes]
    assert out[:buf_bytes].cpu().numpy().tobytes() == first
    eng.close()
    res = {"workload": f"in-flight log replay: {n_sub} subpartitions x {n_epochs} epochs x {per_epoch} buffers "
                       f"(32 KiB), replay from epoch 1 skipping 1", "replayed_bytes": total, "buffers": nbuf,
           "ms_per_step": round(el * 1e3, 4), "kernel_avg_ms": round(kms, 5) if kms else None,
           "kernel_gbs": round(2 * total / (kms * 1e-3) / 1e9, 1) if kms else None,
           "hbm_frac": round(2 * total / (kms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4) if kms else None}
    if not args.no_cpu_baseline:  # host memcpy of the same buffers (the Java drain copies nothing;
        bufs = [np.frombuffer(b, np.uint8) for (_, _, b) in items]  # this is the byte-move floor)
        t0 = _t.perf_counter()
        reps = 0
        while _t.perf_counter() - t0 < 2.0 or reps == 0:
            np.concatenate(bufs)
            reps += 1
        dt = (_t.perf_counter() - t0) / reps
        hc = host_cpu()
        res["cpu_baseline"] = {"value": round(sum(b.size for b in bufs) / dt / 1e9, 2), "unit": "GB/s", "cores": 1,
                               "kind": "port", "sample": f"memcpy gather of one epoch's {len(bufs)} buffers, x{reps} "
                                                         "(one thread: the Java drain is one thread per subpartition)",
                               **{k2: v for k2, v in hc.items() if k2 != "cores"}}
    return res


def config3(args, torch, dev, n_logs=256, n_epochs=10, per_epoch=40000, steps=5):
    """BASELINE.json configs[2]: mixed variable-length determinants (Order, BufferBuilt,
    TimerTrigger "PTS"/"87", Timestamp, RNG, Serializable String/Boolean/Integer,
    SourceCheckpoint, IgnoreCheckpoint), 256 subtask logs x 10 epochs (~0.9 GB) resident in
    HBM; one step = batched decode of every log from its first epoch.  Reported next to the
    headline line (decode only; no consumers are defined for this config)."""
    import time as _t
    from clonos_amd import CausalLogID, Engine, _lib, synth
    from clonos_amd import determinants as D
    rng = np.random.default_rng(synth.SEED_CONFIG3)
    gen = [synth.config3_epoch(per_epoch, rng, e) for e in range(n_epochs)]
    epochs = [g[0] for g in gen]
    per_log = sum(int(e.size) for e in epochs)
    seg = 16384
    total = per_log * n_logs
    n_det = n_logs * per_epoch * n_epochs
    # the long-record variant: one log's epoch carries a 40 KB TimerTrigger
    # name, another's a 9 KB Serializable stream (an int[] of 2250), each at a record boundary
    long_tt = D.encode(D.TimerTriggerDeterminant(7, 1, D.INTERNAL, b"T" * 40000))
    long_js = D.encode(D.SerializableDeterminant(D.jser_int_array(list(range(2250)))))
    def with_long(e, rec):
        k = int(gen[e][1][len(gen[e][1]) // 2])
        return np.concatenate([epochs[e][:k], np.frombuffer(rec, np.uint8), epochs[e][k:]])
    special = {(37, 4): with_long(4, long_tt), (181, 7): with_long(7, long_js)}  # (log, epoch) -> bytes

    def build_engine(variant, decode="auto", sidecar=True):
        old = os.environ.get("CLONOS_SIDECAR")
        if not sidecar:
            os.environ["CLONOS_SIDECAR"] = "0"  # (read when the engine opens)
        try:
            e_ = Engine(segment_bytes=seg, pool_segments=n_logs * ((per_log + seg - 1) // seg + n_epochs + 1) + 64,
                        timing=True, ifl_pool_segments=16, decode=decode)
        finally:
            if not sidecar:
                if old is None:
                    del os.environ["CLONOS_SIDECAR"]
                else:
                    os.environ["CLONOS_SIDECAR"] = old
        ls = []
        for v in range(n_logs):  # every log: the epoch sequence rotated, so layouts differ per log
            log = e_.open_log(CausalLogID.main(v))
            for e in range(n_epochs):
                b = special.get((v, (e + v) % n_epochs)) if variant == "long" else None
                log.processUpstreamDelta((b if b is not None else epochs[(e + v) % n_epochs]).tobytes(), 0, e)
            ls.append(log)
        e_.sync()
        return e_, ls

    def write_cost(e_):
        """The write path's kernel time for the whole log (every byte reaches HBM through
        k_scatter once; with the sidecar it also lists the Serializable candidates)."""
        st_ = e_.kernel_stats()
        ks = [st_.get(n, {"launches": 0, "ms": 0.0}) for n in ("upstream_scatter", "append_scatter")]
        return {"launches": sum(k["launches"] for k in ks), "ms_total": round(sum(k["ms"] for k in ks), 4)}
    eng, logs = build_engine("clean")
    writer = {"with_sidecar": write_cost(eng)}
    cap = n_det + 16  # (the long-record variant holds two records more)
    o = [torch.empty(cap, dtype=torch.int32, device=dev), torch.empty(cap, dtype=torch.uint8, device=dev),
         torch.empty(cap, dtype=torch.int64, device=dev)]
    wcap = n_det // 2 + 16
    ow = [torch.empty(wcap, dtype=t, device=dev) for t in
          (torch.int32, torch.int32, torch.int64, torch.int32, torch.int32, torch.uint8)]
    dec = _lib.Decoded()
    dec.off, dec.tag, dec.v0 = [t.data_ptr() for t in o]
    dec.w_idx, dec.w_rc, dec.w_v1, dec.w_var_off, dec.w_var_len, dec.w_sub = [t.data_ptr() for t in ow]
    dec.cap, dec.wcap, dec.out_kind = cap, wcap, _lib.CLG_MEM_DEVICE
    handles = np.array([l.handle for l in logs], np.uint32)
    starts = np.zeros(n_logs, np.int64)
    base = np.zeros(n_logs + 1, np.uint64)
    for _ in range(2):  # warm-up (the first batch also learns that the logs hold Serializable records)
        eng.decode_logs_device(handles, starts, dec, base)
    assert dec.n_rec == n_det and dec.err_status == 0
    torch.cuda.synchronize()
    t0 = _t.perf_counter()
    for _ in range(steps):  # one decode at a time (the host's planning and completion between them)
        eng.decode_logs_device(handles, starts, dec, base)
    torch.cuda.synchronize()
    el_sync = (_t.perf_counter() - t0) / steps
    # the step as config 2 runs it: two decodes in flight (CLG_DECODE_MAX_INFLIGHT), each with its
    # own outputs, so the GPU does not wait for the host between decodes
    dec2 = _lib.Decoded()
    o2 = [torch.empty_like(t) for t in o] + [torch.empty_like(t) for t in ow]
    dec2.off, dec2.tag, dec2.v0 = [t.data_ptr() for t in o2[:3]]
    dec2.w_idx, dec2.w_rc, dec2.w_v1, dec2.w_var_off, dec2.w_var_len, dec2.w_sub = [t.data_ptr() for t in o2[3:]]
    dec2.cap, dec2.wcap, dec2.out_kind = cap, wcap, _lib.CLG_MEM_DEVICE
    pairs, queued = [(dec, base), (dec2, np.zeros_like(base))], []

    def run_async(k):
        for i in range(k):
            if len(queued) == 2:
                eng.decode_wait()
                d_ = queued.pop(0)
                assert d_.n_rec == n_det and d_.err_status == 0
            d_, b_ = pairs[i % 2]
            eng.decode_logs_device_async(handles, starts, d_, b_)
            queued.append(d_)
        while queued:
            eng.decode_wait()
            d_ = queued.pop(0)
            assert d_.n_rec == n_det and d_.err_status == 0
    run_async(2)  # warm-up
    torch.cuda.synchronize()
    eng.kernel_stats_reset()
    t0 = _t.perf_counter()
    run_async(steps)
    torch.cuda.synchronize()
    el = (_t.perf_counter() - t0) / steps
    st = eng.kernel_stats()
    n_wide = int(dec.n_wide)
    # checkpoint-complete epoch truncation of every log (JobCausalLogImpl.notifyCheckpointComplete
    # fan-out, ThreadCausalLogImpl :398-435): metadata + segment release, reported as latency
    t0 = _t.perf_counter()
    applied = eng.truncate_all(n_epochs // 2)
    trunc_ms = (_t.perf_counter() - t0) * 1e3
    assert applied
    eng.close()
    algo = total + 13 * n_det + 25 * n_wide
    kern = {k: dict(launches=v["launches"], avg_ms=round(v["ms"] / v["launches"], 5))
            for k, v in st.items() if v["launches"]}

    def timed_decode(variant, decode, n_expect):
        e_, ls = build_engine(variant, decode)
        try:
            h = np.array([l.handle for l in ls], np.uint32)
            e_.decode_logs_device(h, starts, dec, base)  # warm-up (table hint)
            assert dec.n_rec == n_expect and dec.err_status == 0, (variant, decode, dec.n_rec, n_expect)
            torch.cuda.synchronize()
            e_.kernel_stats_reset()
            t0 = _t.perf_counter()
            for _ in range(steps):
                e_.decode_logs_device(h, starts, dec, base)
            torch.cuda.synchronize()
            ms = (_t.perf_counter() - t0) / steps * 1e3
            ks = e_.kernel_stats()
            paths = sorted(k for k in ks if k in ("decode_fallback", "decode_span_fallback"))
            kms = {k: round(v["ms"] / v["launches"], 4) for k, v in ks.items() if v["launches"] and v["ms"] > 0}
            kms["dp_spans"] = ks.get("robust_dp_spans", {}).get("launches", 0) // steps  # (robust: spans the DP took)
            return ms, paths, kms
        finally:
            e_.close()
    # the write path without the sidecar, for the cost it moves from the decode to the writer
    e_ns, _ = build_engine("clean", sidecar=False)
    writer["without_sidecar"] = write_cost(e_ns)
    e_ns.close()
    writer["per_call_latency_us"] = {k: round(v["ms_total"] * 1e3 / max(1, v["launches"]), 2) for k, v in writer.items()}

    def batched_write(sidecar):
        """The same 0.9 GB written as one device-input upstream batch per epoch (256 deltas
        each, clg_upstream_delta_batch from HBM): the writer's throughput, where the per-call
        figures above are one wave's latency per chunk."""
        from clonos_amd import dist as X
        old = os.environ.get("CLONOS_SIDECAR")
        if not sidecar:
            os.environ["CLONOS_SIDECAR"] = "0"
        try:
            e_ = Engine(segment_bytes=seg, pool_segments=n_logs * ((per_log + seg - 1) // seg + n_epochs + 1) + 64,
                        timing=True, ifl_pool_segments=16)
        finally:
            if not sidecar:
                if old is None:
                    del os.environ["CLONOS_SIDECAR"]
                else:
                    os.environ["CLONOS_SIDECAR"] = old
        try:
            ls = [e_.open_log(CausalLogID.main(v)) for v in range(n_logs)]
            blob = np.concatenate(epochs)
            eoff = np.concatenate([[0], np.cumsum([int(x.size) for x in epochs])]).astype(np.uint64)
            d_blob = torch.from_numpy(blob).to(dev)
            torch.cuda.synchronize()
            e_.kernel_stats_reset()
            t0 = _t.perf_counter()
            for e in range(n_epochs):
                req = np.zeros(n_logs, X.DELTA_REQ)
                req["log"] = [l.handle for l in ls]
                req["epoch"] = e
                k = (np.arange(n_logs) + e) % n_epochs  # (each log's epoch sequence rotated, as above)
                req["src_off"] = eoff[k]
                req["len"] = (eoff[k + 1] - eoff[k]).astype(np.uint32)
                e_.upstream_delta_batch(req.ctypes.data, n_logs, d_blob.data_ptr(), _lib.CLG_MEM_DEVICE)
            torch.cuda.synchronize()
            wall = (_t.perf_counter() - t0) * 1e3
            return dict(write_cost(e_), wall_ms=round(wall, 3), gbs=round(total / (wall * 1e-3) / 1e9, 2))
        finally:
            e_.close()
    writer["batched_with_sidecar"] = batched_write(True)
    writer["batched_without_sidecar"] = batched_write(False)
    writer["sidecar_ms_per_step"] = round(writer["batched_with_sidecar"]["ms_total"] -
                                          writer["batched_without_sidecar"]["ms_total"], 4)
    writer["note"] = ("k_scatter time to write the whole config-3 log (0.9 GB) with and without the Serializable "
                      "candidate lists (the decode work moved to the writer, paid once per byte written: one decode "
                      "step's worth): as 2 560 one-log calls (per-call latency: one wave per 16 KiB chunk measures "
                      "its candidates) and as 10 batched device-input calls of 256 deltas (throughput); "
                      "sidecar_ms_per_step from the batched figures")
    # the robust pipeline alone (the fallback's throughput) and the long-record batch
    rob_ms, _, rob_k = timed_decode("clean", "robust", n_det)
    # the long-record batch against the clean one through the same harness (a fresh engine each)
    clean_ms, _, clean_k = timed_decode("clean", "auto", n_det)
    long_ms, long_paths, long_k = timed_decode("long", "auto", n_det + 2)
    out = {"workload": f"config3: {n_logs} subtask logs x {n_epochs} epochs x {per_epoch} mixed determinants "
                       "(incl. Serializable, BufferBuilt), decode", "log_bytes": total, "determinants": n_det,
           "wide_records": n_wide, "ms_per_step": round(el * 1e3, 4), "determinants_per_s": round(n_det / el, 1),
           "ms_per_step_one_at_a_time": round(el_sync * 1e3, 4),
           "log_gbs": round(total / el / 1e9, 2), "algo_gbs": round(algo / el / 1e9, 1),
           "hbm_frac": round(algo / el / 1e9 / HBM_PEAK_GBS, 4), "kernels": kern, "writer": writer,
           "truncate_all": {"logs": n_logs, "checkpoint": n_epochs // 2, "latency_ms": round(trunc_ms, 4)},
           "robust_pipeline": {"ms_per_step": round(rob_ms, 4), "determinants_per_s": round(n_det / rob_ms * 1e3, 1),
                               "log_gbs": round(total / rob_ms / 1e6, 2), "kernels_ms": rob_k},
           "long_records": {"note": "the same batch with a 40 KB TimerTrigger name (log 37) and a 9 KB "
                                    "Serializable int[] stream (log 181) inserted at record boundaries",
                            "ms_per_step": round(long_ms, 4), "clean_ms_per_step": round(clean_ms, 4),
                            "vs_clean": round(long_ms / clean_ms, 4),
                            "pipeline_ms": long_k.get("decode_pipeline"), "clean_pipeline_ms": clean_k.get("decode_pipeline"),
                            "pipeline_vs_clean": round(long_k["decode_pipeline"] / clean_k["decode_pipeline"], 4)
                            if long_k.get("decode_pipeline") and clean_k.get("decode_pipeline") else None,
                            "fallbacks": long_paths}}
    if not args.no_cpu_baseline:  # the C++ oracle's decodeNext loop on host cores, whole workload once
        sys.path.insert(0, os.path.join(ROOT, "tests"))
        import _oracle as O  # the checker, timed here as the CPU baseline
        host = np.concatenate([epochs[(e + v) % n_epochs] for v in range(n_logs) for e in range(n_epochs)])
        lens = np.full(n_logs, per_log, np.uint64)
        offs = np.arange(n_logs, dtype=np.uint64) * np.uint64(per_log)
        hc = host_cpu()
        threads = args.cpu_threads or hc["cores"]
        reps, dt = 0, 0.0  # the whole config-3 decode, repeated for at least 2 s
        while dt < 2.0 or reps == 0:
            t0 = _t.perf_counter()
            n1 = O.lib.orc_bench_decode(O.ptr(host), O.ptr(offs), O.ptr(lens), n_logs, threads)
            dt += _t.perf_counter() - t0
            reps += 1
            assert n1 == n_det, (n1, n_det)
        # one core: one call over the first k logs (output buffers allocated once), k sized
        # for about 2 s from the multi-core rate
        per_log_1 = dt / reps / n_logs * threads
        k = int(min(n_logs, max(1, 2.0 / max(per_log_1, 1e-9))))
        t0 = _t.perf_counter()
        nk = O.lib.orc_bench_decode(O.ptr(host), O.ptr(offs), O.ptr(lens), k, 1)
        d1 = _t.perf_counter() - t0
        out["cpu_baseline"] = {"value": round(n_det * reps / dt, 1), "unit": "determinants/s", "cores": threads,
                               "kind": "port",
                               "sample": f"whole config-3 decode ({total} B) x{reps} in {dt:.2f}s on {threads} threads",
                               "cores_1": {"value": round(nk / d1, 1), "unit": "determinants/s",
                                           "sample": f"{k} logs decode in one call, one thread, {d1:.2f}s"},
                               **{k2: v for k2, v in hc.items() if k2 != "cores"}}
    return out


def host_cpu():
    """The host cores this process may use: its affinity mask, capped by a cgroup CPU quota
    when one is set (a GPU box shares its host between GPUs), and the CPU model."""
    try:
        affinity = len(os.sched_getaffinity(0))
    except AttributeError:
        affinity = os.cpu_count() or 1
    quota = None
    try:
        q, period = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            quota = max(1, int(int(q) / int(period)))
    except (OSError, ValueError):
        pass
    model = ""
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                model = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    usable = min(affinity, quota) if quota else affinity
    return {"cores": usable, "affinity": affinity, "cgroup_quota_cpus": quota, "cpu": model}


def cpu_baseline(bufs, log_bytes, cons, args):
    """The C++ oracle (sequential decodeNext loop + memcpy slicing) on host cores, same
    workload as the GPU step.  Threads: one log per std::thread."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import _oracle as O  # the checker, timed here as the CPU baseline
    host = np.concatenate(bufs)
    starts = np.zeros(len(bufs), np.uint64)
    starts[1:] = np.cumsum(np.array(log_bytes, np.uint64))[:-1]
    lens = np.array(log_bytes, np.uint64)
    src = np.array([int(starts[i]) + off for i, _, off in cons], np.uint64)
    ln = np.array([log_bytes[i] - off for i, _, off in cons], np.uint64)
    dst = np.zeros(len(cons), np.uint64)
    dst[1:] = np.cumsum(ln)[:-1]
    out = np.empty(int(ln.sum()), np.uint8)
    hc = host_cpu()
    threads = args.cpu_threads or hc["cores"]
    # repeat the full step until at least args.cpu_seconds of CPU wall time (bounded sample)
    reps, td, ts, nrec = 0, 0.0, 0.0, 0
    while td + ts < args.cpu_seconds or reps == 0:
        t0 = time.perf_counter()
        n1 = O.lib.orc_bench_decode(O.ptr(host), O.ptr(starts), O.ptr(lens), len(bufs), threads)
        t1 = time.perf_counter()
        O.lib.orc_bench_slice(O.ptr(host), O.ptr(src), O.ptr(ln), O.ptr(dst), len(cons), O.ptr(out), threads)
        t2 = time.perf_counter()
        assert n1 == len(bufs) * args.records
        nrec += n1
        td += t1 - t0
        ts += t2 - t1
        reps += 1
    # 1 core: the same work for the first k logs (decode + those logs' consumers' slices), one
    # call each on one thread (output buffers allocated once), k sized for about a quarter of
    # the multi-core sample's time from the multi-core rate
    per_log_1 = (td + ts) / reps / len(bufs) * threads
    k = int(min(len(bufs), max(1, args.cpu_seconds / 4 / max(per_log_1, 1e-9))))
    kc = [j for j, (i, _, _) in enumerate(cons) if i < k]
    src1, ln1 = np.ascontiguousarray(src[kc]), np.ascontiguousarray(ln[kc])
    dst1 = np.zeros(len(kc), np.uint64)
    dst1[1:] = np.cumsum(ln1)[:-1]
    t0 = time.perf_counter()
    n1 = O.lib.orc_bench_decode(O.ptr(host), O.ptr(starts), O.ptr(lens), k, 1)
    t1 = time.perf_counter()
    O.lib.orc_bench_slice(O.ptr(host), O.ptr(src1), O.ptr(ln1), O.ptr(dst1), len(kc), O.ptr(out), 1)
    t2 = time.perf_counter()
    return {"value": round(nrec / (td + ts), 1), "unit": "determinants/s", "cores": threads, "kind": "port",
            "sample": f"full config-2 step ({len(bufs)} logs x {args.records} records decode + {len(cons)} slices, "
                      f"{int(ln.sum())} B) x {reps}; decode {td:.2f}s slice {ts:.2f}s on {threads} threads",
            "cores_1": {"value": round(n1 / (t2 - t0), 1), "unit": "determinants/s",
                        "sample": f"{k} logs decode ({t1 - t0:.2f}s) + their {len(kc)} slices ({t2 - t1:.2f}s), "
                                  "one thread"},
            **{k2: v for k2, v in hc.items() if k2 != "cores"}}


if __name__ == "__main__":
    main()
