"""Developer diagnostics: per-tile phase cycles of the sidecar table kernel (k_decode_jser_side,
CLONOS_SCAN_PHASES stamps 6-7) on config 3 written as the bench writes it.  Not part of the
product or the tests."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
out = "gpurun_out/side_phases.bin"
os.makedirs("gpurun_out", exist_ok=True)
os.environ["CLONOS_SCAN_PHASES"] = out
from clonos_amd import CausalLogID, Engine, synth  # noqa: E402

nlogs = int(sys.argv[1]) if len(sys.argv) > 1 else 64
rng = np.random.default_rng(synth.SEED_CONFIG3)
epochs = [synth.config3_epoch(40000, rng, e)[0] for e in range(10)]
with Engine(segment_bytes=16384, pool_segments=nlogs * 240, timing=True) as eng:
    logs = []
    for v in range(nlogs):
        lg = eng.open_log(CausalLogID.main(v))
        for e in range(10):
            lg.processUpstreamDelta(epochs[(e + v) % 10].tobytes(), 0, e)
        logs.append(lg)
    eng.sync()
    for _ in range(3):
        dec = eng.decode_logs(logs, [0] * nlogs)
    print({k: round(v["ms"] / max(1, v["launches"]), 4) for k, v in eng.kernel_stats().items() if v["launches"]})
p = np.fromfile(out, np.uint64).reshape(-1, 8)
st, w = p[:, 6].astype(np.int64), p[:, 7]
ok = st > 0
print("tiles", len(p), "stamped", ok.sum())
m = (1 << 21) - 1
ph = np.stack([(w & m), (w >> 21) & m, (w >> 42) & m], 1)[ok].astype(np.int64)
for i, nm in enumerate(["desc+hdr", "entries", "rank+tables"]):
    print(nm, "p50", np.percentile(ph[:, i], 50), "p90", np.percentile(ph[:, i], 90), "max", ph[:, i].max())
gen = (w[ok] >> 59).astype(np.int64)
print("general items per tile: mean", gen.mean(), "max", gen.max(), "tiles with any", (gen > 0).sum())
s0 = st[ok]
print("span of starts (cycles)", s0.max() - s0.min(), "per-tile total p50", np.percentile(ph.sum(1), 50))
