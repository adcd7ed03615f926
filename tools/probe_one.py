"""Developer probe: time the one-pass decode kernel on config 2 under CLONOS_ONE_PROBE
settings (run each setting in its own process: the engine reads the env once)."""
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
from clonos_amd import CausalLogID, Engine, _lib, synth  # noqa: E402

n_logs = int(sys.argv[1]) if len(sys.argv) > 1 else 64
rng = np.random.default_rng(synth.SEED_CONFIG2)
bufs = [synth.config2_log(1_000_000, rng)[0] for _ in range(n_logs)]
seg = 16384
eng = Engine(segment_bytes=seg, pool_segments=sum(b.size // seg + 2 for b in bufs) + 64, timing=True)
logs = []
for v, b in enumerate(bufs):
    lg = eng.open_log(CausalLogID.main(v))
    lg.processUpstreamDelta(b.tobytes(), 0, 1)
    logs.append(lg)
eng.sync()
n = n_logs * 1_000_000
dev = torch.device("cuda", 0)
o = [torch.empty(n, dtype=t, device=dev) for t in (torch.int32, torch.uint8, torch.int64)]
ow = [torch.empty(1024, dtype=t, device=dev) for t in (torch.int32, torch.int32, torch.int64, torch.int32, torch.int32,
                                                          torch.uint8)]
dec = _lib.Decoded()
dec.off, dec.tag, dec.v0 = [t.data_ptr() for t in o]
dec.w_idx, dec.w_rc, dec.w_v1, dec.w_var_off, dec.w_var_len, dec.w_sub = [t.data_ptr() for t in ow]
dec.cap, dec.wcap, dec.out_kind = n, 1024, _lib.CLG_MEM_DEVICE
h = np.array([l.handle for l in logs], np.uint32)
st = np.ones(len(logs), np.int64)
base = np.zeros(len(logs) + 1, np.uint64)
for _ in range(3):
    try:
        eng.decode_logs_device(h, st, dec, base)
    except Exception as e:  # probes produce invalid output
        pass
eng.kernel_stats_reset()
for _ in range(5):
    try:
        eng.decode_logs_device(h, st, dec, base)
    except Exception:
        pass
print(json.dumps({"probe": os.environ.get("CLONOS_ONE_PROBE", "0"), "warm": os.environ.get("CLONOS_WARM", "96"),
                  "decode": os.environ.get("CLONOS_DECODE", "threepass"),
                  "kernels": {k: round(v["ms"] / v["launches"], 4) for k, v in eng.kernel_stats().items()
                              if v["launches"]}}), flush=True)
