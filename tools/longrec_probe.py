"""Developer probe: which records make the fast decode fall back.  Config-3-shaped batch (64
logs x 4 epochs), one record of a given kind and size inserted at a record boundary in one
log; prints the decode paths taken, the time per decode and (CLONOS_FUSED_DEBUG) the abort
reason of the fast run on stderr.  JSON lines on stdout."""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402
from clonos_amd import CausalLogID, Engine, _lib, synth  # noqa: E402
from clonos_amd import determinants as D  # noqa: E402

os.environ["CLONOS_FUSED_DEBUG"] = "1"
FULL = os.environ.get("LONGREC_FULL") == "1"  # config 3's full shape (256 logs x 10 epochs)
N_LOGS, N_EP, PER = (256, 10, 40000) if FULL else (64, 4, 40000)
rng = np.random.default_rng(synth.SEED_CONFIG3)
gen = [synth.config3_epoch(PER, rng, e) for e in range(N_EP)]
epochs = [g[0] for g in gen]
dev = torch.device("cuda", 0)
n_det = N_LOGS * N_EP * PER
cap = max(n_det, N_LOGS * 400001) + 65536  # room for an inserted run of short records
o = [torch.empty(cap, dtype=t, device=dev) for t in (torch.int32, torch.uint8, torch.int64)]
ow = [torch.empty(n_det // 2 + 16, dtype=t, device=dev)
      for t in (torch.int32, torch.int32, torch.int64, torch.int32, torch.int32, torch.uint8)]
dec = _lib.Decoded()
dec.off, dec.tag, dec.v0 = [t.data_ptr() for t in o]
dec.w_idx, dec.w_rc, dec.w_v1, dec.w_var_off, dec.w_var_len, dec.w_sub = [t.data_ptr() for t in ow]
dec.cap, dec.wcap, dec.out_kind = cap, n_det // 2 + 16, _lib.CLG_MEM_DEVICE


def case(name, rec, log=37, ep=2, frac=0.5, n_ins=1):
    seg = 16384
    per_log = sum(int(e.size) for e in epochs) + (len(rec) if rec else 0)
    eng = Engine(segment_bytes=seg, pool_segments=N_LOGS * ((per_log + seg - 1) // seg + N_EP + 1) + 64, timing=True,
                 ifl_pool_segments=16)
    try:
        hs = []
        for v in range(N_LOGS):
            l = eng.open_log(CausalLogID.main(v))
            for e in range(N_EP):
                b = epochs[e]
                if rec is not None and v == log and e == ep:
                    k = int(gen[e][1][int(len(gen[e][1]) * frac)])
                    b = np.concatenate([b[:k], np.frombuffer(rec, np.uint8), b[k:]])
                l.processUpstreamDelta(b.tobytes(), 0, e)
            hs.append(l.handle)
        eng.sync()
        hs = np.array(hs, np.uint32)
        starts = np.zeros(N_LOGS, np.int64)
        base = np.zeros(N_LOGS + 1, np.uint64)
        print(f"--- {name}", file=sys.stderr, flush=True)
        eng.decode_logs_device(hs, starts, dec, base)
        ok = dec.err_status == 0 and dec.n_rec == n_det + (n_ins if rec else 0)
        torch.cuda.synchronize()
        eng.kernel_stats_reset()
        t0 = time.perf_counter()
        for _ in range(3):
            eng.decode_logs_device(hs, starts, dec, base)
        torch.cuda.synchronize()
        ms = (time.perf_counter() - t0) / 3 * 1e3
        ks = eng.kernel_stats()
        paths = sorted(k for k in ks if k in ("decode_fallback", "decode_span_fallback", "decode_chunk_repair"))
        kms = {k: round(v["ms"] / v["launches"], 4) for k, v in ks.items() if v["launches"] and v["ms"] > 0}
        print(json.dumps({"case": name, "rec_bytes": len(rec) if rec else 0, "ok": bool(ok), "ms": round(ms, 3),
                          "paths": paths, "kernels": kms}), flush=True)
    finally:
        eng.close()


def bench_layout(variant):
    """bench.py config3's build_engine: every log's epochs rotated; its long-record variant."""
    seg = 16384
    long_tt = D.encode(D.TimerTriggerDeterminant(7, 1, D.INTERNAL, b"T" * 40000))
    long_js = D.encode(D.SerializableDeterminant(D.jser_int_array(list(range(2250)))))

    def with_long(e, rec):
        k = int(gen[e][1][len(gen[e][1]) // 2])
        return np.concatenate([epochs[e][:k], np.frombuffer(rec, np.uint8), epochs[e][k:]])
    special = {(37, 4): with_long(4, long_tt), (181, 7): with_long(7, long_js)} if variant != "clean" else {}
    if variant == "timer":
        special.pop((181, 7))
    if variant == "jser":
        special.pop((37, 4))
    per_log = sum(int(e.size) for e in epochs)
    eng = Engine(segment_bytes=seg, pool_segments=N_LOGS * ((per_log + seg - 1) // seg + N_EP + 1) + 64, timing=True,
                 ifl_pool_segments=16)
    try:
        hs = []
        for v in range(N_LOGS):
            l = eng.open_log(CausalLogID.main(v))
            for e in range(N_EP):
                b = special.get((v, (e + v) % N_EP))
                l.processUpstreamDelta((b if b is not None else epochs[(e + v) % N_EP]).tobytes(), 0, e)
            hs.append(l.handle)
        eng.sync()
        hs = np.array(hs, np.uint32)
        starts = np.zeros(N_LOGS, np.int64)
        base = np.zeros(N_LOGS + 1, np.uint64)
        eng.decode_logs_device(hs, starts, dec, base)
        torch.cuda.synchronize()
        eng.kernel_stats_reset()
        for _ in range(3):
            eng.decode_logs_device(hs, starts, dec, base)
        torch.cuda.synchronize()
        ks = eng.kernel_stats()
        print(json.dumps({"layout": variant, "n_rec": int(dec.n_rec),
                          "stats": {k: (round(v["ms"] / v["launches"], 4) if v["ms"] else v["launches"])
                                    for k, v in ks.items() if v["launches"]}}), flush=True)
    finally:
        eng.close()


if FULL:
    for v in ("clean", "both", "timer", "jser", "clean"):
        bench_layout(v)
    case("clean", None)
    case("timer_40000", D.encode(D.TimerTriggerDeterminant(7, 1, D.INTERNAL, b"T" * 40000)), log=37, ep=4)
    case("jser_intarr_2250", D.encode(D.SerializableDeterminant(D.jser_int_array(list(range(2250))))), log=181, ep=7)
    # 64 KB runs of channel-0 Order records ("00 00") across chunk ends, both parities
    for frac in (0.3, 0.7):
        case(f"zero_run_64k_odd_{frac}", D.encode(D.TimestampDeterminant(5)) + D.encode(D.OrderDeterminant(0)) * 32768,
             log=37, ep=4, frac=frac, n_ins=32769)
        case(f"zero_run_64k_even_{frac}", D.encode(D.OrderDeterminant(0)) * 32768, log=37, ep=4, frac=frac, n_ins=32768)
    case("clean", None)
    sys.exit(0)
case("clean", None)
for n in (300, 2000, 7000, 9000, 40000):
    case(f"timer_{n}", D.encode(D.TimerTriggerDeterminant(7, 1, D.INTERNAL, b"T" * n)))
for n in (200, 1000, 2250):
    case(f"jser_intarr_{n}", D.encode(D.SerializableDeterminant(D.jser_int_array(list(range(n))))))
case("timer_40000_near_end", D.encode(D.TimerTriggerDeterminant(7, 1, D.INTERNAL, b"T" * 40000)), frac=0.999)


def order_case(name, lead):
    """64 logs of 400 000 Order records after `lead` (a 9-byte Timestamp puts every Order
    record at an odd offset; nothing: even)."""
    seg = 16384
    body = D.encode(D.OrderDeterminant(0)) * 400000  # channel 0: "00 00", a valid record at every offset
    eng = Engine(segment_bytes=seg, pool_segments=N_LOGS * ((len(body) + 64) // seg + 4) + 64, timing=True,
                 ifl_pool_segments=16)
    try:
        hs = []
        for v in range(N_LOGS):
            l = eng.open_log(CausalLogID.main(v))
            l.processUpstreamDelta(lead + body, 0, 0)
            hs.append(l.handle)
        eng.sync()
        hs = np.array(hs, np.uint32)
        starts = np.zeros(N_LOGS, np.int64)
        base = np.zeros(N_LOGS + 1, np.uint64)
        eng.decode_logs_device(hs, starts, dec, base)
        n = 400000 + (1 if lead else 0)
        ok = dec.err_status == 0 and dec.n_rec == N_LOGS * n
        torch.cuda.synchronize()
        eng.kernel_stats_reset()
        t0 = time.perf_counter()
        for _ in range(3):
            eng.decode_logs_device(hs, starts, dec, base)
        torch.cuda.synchronize()
        ms = (time.perf_counter() - t0) / 3 * 1e3
        ks = eng.kernel_stats()
        print(json.dumps({"case": name, "ok": bool(ok), "ms": round(ms, 3),
                          "count_ms": round(ks["decode_count"]["ms"] / ks["decode_count"]["launches"], 4),
                          "paths": sorted(k for k in ks if k in ("decode_fallback", "decode_span_fallback",
                                                                  "decode_chunk_repair"))}), flush=True)
    finally:
        eng.close()


order_case("order_even", b"")
order_case("order_odd", D.encode(D.TimestampDeterminant(5)))
