"""Latency of small batched decodes (a launch-bound case): 16 logs x ~4 KiB decoded into
host arrays, repeated, timing off.  Prints one JSON line."""
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from clonos_amd import CausalLogID, Engine, synth  # noqa: E402

rng = np.random.default_rng(3)
blobs = [synth.config2_log(750, rng)[0] for _ in range(16)]
with Engine(segment_bytes=16384, pool_segments=256, timing=False) as eng:
    logs = []
    for v, b in enumerate(blobs):
        lg = eng.open_log(CausalLogID.main(v))
        lg.processUpstreamDelta(b.tobytes(), 0, 1)
        logs.append(lg)
    for _ in range(20):
        eng.decode_logs(logs, [1] * len(logs))
    ts = []
    for _ in range(300):
        t = time.perf_counter()
        eng.decode_logs(logs, [1] * len(logs))
        ts.append((time.perf_counter() - t) * 1e6)
ts.sort()
print(json.dumps({"metric": "small batched decode latency (us)", "logs": 16, "bytes": int(sum(b.size for b in blobs)),
                  "p50": round(ts[len(ts) // 2], 1),
                  "p99": round(ts[int(len(ts) * 0.99)], 1)}))
