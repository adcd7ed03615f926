"""Developer probe: where config 1's decode latency goes (44 logs, 73 KB): the Python wrapper
with host outputs, the native call with host outputs, and the native call into device
arrays; host-side stage timers (CLONOS_HOST_PROF) and kernel events.  JSON lines."""
import json
import os
import sys
import time

import numpy as np

os.environ.setdefault("CLONOS_HOST_PROF", "1")
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402
from clonos_amd import Engine, _lib, synth  # noqa: E402

rng = np.random.default_rng(synth.SEED_CONFIG1)
graph, data = synth.config1_job(rng)
eng = Engine(segment_bytes=16384, pool_segments=4096, sharing_depth=1, timing=True, ifl_pool_segments=16)
logs = {lid: eng.open_log(lid) for lid in data}
for lid, b in data.items():
    logs[lid].appendDeterminant(b, 0)
lids = list(data)
lg = [logs[l] for l in lids]
h = np.array([l.handle for l in lg], np.uint32)
ep = np.zeros(len(lg), np.int64)
total = sum(len(b) for b in data.values())
print(json.dumps({"span_bytes": [len(data[l]) for l in lids]}), flush=True)
dev = torch.device("cuda", 0)
cap, wcap = total // 2 + 64, total // 6 + 64
o = [torch.empty(cap, dtype=t, device=dev) for t in (torch.int32, torch.uint8, torch.int64)]
ow = [torch.empty(wcap, dtype=t, device=dev) for t in (torch.int32, torch.int32, torch.int64, torch.int32, torch.int32, torch.uint8)]
dd = _lib.Decoded()
dd.off, dd.tag, dd.v0 = [t.data_ptr() for t in o]
dd.w_idx, dd.w_rc, dd.w_v1, dd.w_var_off, dd.w_var_len, dd.w_sub = [t.data_ptr() for t in ow]
dd.cap, dd.wcap, dd.out_kind = cap, wcap, _lib.CLG_MEM_DEVICE
base = np.zeros(len(lg) + 1, np.uint64)
hd, _ = Engine._host_outputs(cap, wcap)


def timeit(name, fn, n=50):
    for _ in range(5):
        fn()
    eng.kernel_stats_reset()
    t0 = time.perf_counter()
    for _ in range(n):
        fn()
    ms = (time.perf_counter() - t0) / n * 1e3
    ks = {k: round(v["ms"] / v["launches"], 4) for k, v in eng.kernel_stats().items() if v["launches"]}
    print(json.dumps({"case": name, "ms": round(ms, 4), "stats": ks}), flush=True)


timeit("python_host", lambda: eng.decode_logs(lg, [0] * len(lg)))
timeit("native_host", lambda: _lib.lib.clg_decode_logs(eng._h, h.ctypes.data, ep.ctypes.data, len(lg),
                                                         _lib.C.byref(hd), base.ctypes.data))
timeit("native_device", lambda: _lib.lib.clg_decode_logs(eng._h, h.ctypes.data, ep.ctypes.data, len(lg),
                                                           _lib.C.byref(dd), base.ctypes.data))
