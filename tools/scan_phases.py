"""Developer diagnostics: per-phase cycle breakdown of k_fast_scan (s_memtime stamps,
CLONOS_SCAN_PHASES) on the config-2 workload.  Not part of the product or the tests."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
out = "gpurun_out/scan_phases.bin"
os.environ["CLONOS_SCAN_PHASES"] = out
from clonos_amd import CausalLogID, Engine, synth  # noqa: E402

nlogs = int(sys.argv[1]) if len(sys.argv) > 1 else 16
rng = np.random.default_rng(synth.SEED_CONFIG2)
with Engine(segment_bytes=16384, pool_segments=nlogs * 400, timing=True) as eng:
    logs = []
    for i in range(nlogs):
        b, _ = synth.config2_log(1_000_000, rng)
        lg = eng.open_log(CausalLogID.main(i))
        lg.processUpstreamDelta(b.tobytes(), 0, 1)
        logs.append(lg)
    for _ in range(3):
        dec = eng.decode_logs(logs, [1] * nlogs)
    print("n_rec", dec.n_rec, {k: round(v["ms"] / max(1, v["launches"]), 4) for k, v in eng.kernel_stats().items() if v["launches"]})
p = np.fromfile(out, np.uint64).reshape(-1, 8).astype(np.int64)
ok = (p[:, 0] > 0) & (p[:, 6] > 0)
d = np.diff(p[ok][:, :7], axis=1)
names = ["stage", "magic", "bfs", "keep", "parse", "chain+store"]
tot = d.sum(axis=1)
print("tiles", ok.sum(), "cycles/tile mean %.0f p50 %.0f p99 %.0f" % (tot.mean(), np.median(tot), np.percentile(tot, 99)))
for i, n in enumerate(names):
    print(f"  {n:12s} mean {d[:, i].mean():9.0f}  p50 {np.median(d[:, i]):9.0f}  p99 {np.percentile(d[:, i], 99):9.0f}")
