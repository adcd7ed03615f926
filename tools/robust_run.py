"""Developer driver: the robust pipeline alone on config-3 logs (synth.config3_epoch), decoded
`reps` times -- a short program for rocprofv3 kernel traces and counter passes of the robust
kernels.  Checks the first decode's record count.  usage: robust_run.py [n_logs] [reps]"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402,F401
from clonos_amd import CausalLogID, Engine, synth  # noqa: E402

n_logs = int(sys.argv[1]) if len(sys.argv) > 1 else 64
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 3
N_EP, PER = 10, 40000
rng = np.random.default_rng(synth.SEED_CONFIG3)
gen = [synth.config3_epoch(PER, rng, e) for e in range(N_EP)]
eng = Engine(segment_bytes=16384, pool_segments=n_logs * 240 + 64, timing=True, decode="robust", ifl_pool_segments=16)
logs = []
for v in range(n_logs):
    l = eng.open_log(CausalLogID.main(v))
    for e in range(N_EP):
        l.processUpstreamDelta(gen[(e + v) % N_EP][0].tobytes(), 0, e)
    logs.append(l)
want = n_logs * sum(len(g[1]) for g in gen)
for r in range(reps):
    dec = eng.decode_logs(logs, [0] * n_logs)
    assert os.environ.get("CLONOS_NOCHECK") or dec.n_rec == want, (dec.n_rec, want)
ks = eng.kernel_stats()
print({k: round(v["ms"] / max(1, v["launches"]), 4) for k, v in ks.items() if k.startswith("robust")})
eng.close()
