"""Developer probe: the config-2 decode alone (64 logs x 1 M records in 16 KiB segments), timed
by the engine's HIP events, for A/B builds (CLONOS_LIB).  Prints one JSON line."""
import json, os, sys
import numpy as np
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: F401  (the engine binds torch's HIP runtime)
from clonos_amd import CausalLogID, Engine, _lib, synth

n_logs, n_rec = int(os.environ.get("PROBE_LOGS", 64)), int(os.environ.get("PROBE_REC", 1_000_000))
rng = np.random.default_rng(synth.SEED_CONFIG2)
bufs = [synth.config2_log(n_rec, rng)[0] for _ in range(n_logs)]
seg = 16384
pool = sum(int(b.size) // seg + 2 for b in bufs) + 64
with Engine(segment_bytes=seg, pool_segments=pool, timing=True) as eng:
    logs = []
    for v, b in enumerate(bufs):
        lg = eng.open_log(CausalLogID.main(v))
        lg.processUpstreamDelta(b.tobytes(), 0, 1)
        logs.append(lg)
    n = n_logs * n_rec
    o = [torch.empty(n, dtype=t, device="cuda") for t in (torch.int32, torch.uint8, torch.int64)]
    w = [torch.empty(1024, dtype=t, device="cuda") for t in (torch.int32, torch.int32, torch.int64, torch.int32, torch.int32, torch.uint8)]
    d = _lib.Decoded()
    d.off, d.tag, d.v0 = [x.data_ptr() for x in o]
    d.w_idx, d.w_rc, d.w_v1, d.w_var_off, d.w_var_len, d.w_sub = [x.data_ptr() for x in w]
    d.cap, d.wcap, d.out_kind = n, 1024, _lib.CLG_MEM_DEVICE
    h = np.array([lg.handle for lg in logs], np.uint32)
    base = np.zeros(n_logs + 1, np.uint64)
    for k in range(8):
        if k == 3:
            eng.sync()
            eng.kernel_stats_reset()
        try:
            eng.decode_logs_device(h, np.ones(n_logs, np.int64), d, base)
        except Exception as e:  # (timing variants decode wrongly on purpose)
            pass
    eng.sync()
    st = eng.kernel_stats()
    print(json.dumps({k: round(v["ms"] / v["launches"], 4) for k, v in st.items() if v["launches"] and not k.startswith("host")}))
