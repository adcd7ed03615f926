"""Developer diagnostics: per-phase cycle breakdown of the decode count kernel
(s_memtime stamps, CLONOS_SCAN_PHASES) on the config-2 workload (argv[2] = c3: config 3).  Not part of the product
or the tests."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
out = "gpurun_out/scan_phases.bin"
os.makedirs("gpurun_out", exist_ok=True)
os.environ["CLONOS_SCAN_PHASES"] = out
from clonos_amd import CausalLogID, Engine, synth  # noqa: E402

nlogs = int(sys.argv[1]) if len(sys.argv) > 1 else 16
rng = np.random.default_rng(synth.SEED_CONFIG2)
with Engine(segment_bytes=16384, pool_segments=nlogs * 400, timing=True) as eng:
    logs = []
    c3 = len(sys.argv) > 2 and sys.argv[2].startswith("c3")
    if len(sys.argv) > 2 and sys.argv[2] == "c3n":  # config 3 without Serializable records
        synth.CONFIG3_MIX[:] = [(n, w) for n, w in synth.CONFIG3_MIX if not n.startswith("ser_")]
    for i in range(nlogs):
        b = np.concatenate([synth.config3_epoch(40000, rng, e)[0] for e in range(10)]) if c3 else \
            synth.config2_log(1_000_000, rng)[0]
        lg = eng.open_log(CausalLogID.main(i))
        lg.processUpstreamDelta(b.tobytes(), 0, 1)
        logs.append(lg)
    for _ in range(3):
        try:
            dec = eng.decode_logs(logs, [1] * nlogs)
            print("n_rec", dec.n_rec)
        except Exception as e:  # CLONOS_FUSED_NODEP: output is invalid by design
            print("decode:", str(e)[:120])
    print( {k: round(v["ms"] / max(1, v["launches"]), 4) for k, v in eng.kernel_stats().items() if v["launches"]})
p = np.fromfile(out, np.uint64).reshape(-1, 8).astype(np.int64)
ok = (p[:, 0] > 0) & (p[:, 4] > 0)
print("tiles", len(p), "complete", ok.sum())
q = p[ok][:, :5]
d = np.diff(q, axis=1)
names = ["entry+stage", "spec", "true", "counts"]  # phases of k_decode_count
tot = q[:, 4] - q[:, 0]
print("cycles/tile mean %.0f p50 %.0f p99 %.0f" % (tot.mean(), np.median(tot), np.percentile(tot, 99)))
for i, n in enumerate(names):
    print(f"  {n:10s} mean {d[:, i].mean():9.0f}  p50 {np.median(d[:, i]):9.0f}  p99 {np.percentile(d[:, i], 99):9.0f}  max {d[:, i].max():9.0f}")
t0 = q[:, 0].min()
span = q[:, 4].max() - t0
print("kernel span (cycles of s_memtime) %d" % span)
idx = np.nonzero(ok)[0]
for frac in (0.0, 0.1, 0.25, 0.5, 0.75, 0.9, 1.0):
    k = min(len(idx) - 1, int(frac * (len(idx) - 1)))
    print(f"  tile {idx[k]:6d} start {q[k,0]-t0:10d} end {q[k,4]-t0:10d}")

m = p[ok][:, 5]
m0, m1, it = m & 0xFFFFF, (m >> 20) & 0xFFFFF, (m >> 40) & 0xFF
for name, x in (("first-merge max steps", m0), ("re-merge max steps", m1), ("fix-up passes", it)):
    print(f"  {name:22s} mean {x.mean():7.2f} p50 {np.median(x):5.0f} p90 {np.percentile(x, 90):5.0f} p99 {np.percentile(x, 99):5.0f} max {x.max()}")

j6, j7 = p[:, 6], p[:, 7]
if (j7 > 0).any():  # k_decode_jser stamps (J runs): stage / scan + lengths
    sc, ln = j7[j7 > 0] & 0xFFFFFFFF, j7[j7 > 0] >> 32
    print(f"  jser stage mean {j6[j7 > 0].mean():9.0f}   scan mean {sc.mean():9.0f}   lengths+stores mean {ln.mean():9.0f} p99 {np.percentile(ln, 99):9.0f}")
