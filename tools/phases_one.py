"""Developer diagnostics: per-tile phase stamps of k_decode_one (CLONOS_SCAN_PHASES=<file>),
config 2 at 64 logs; prints per-phase cycle percentiles and the tile start-time spread."""
import os
import sys

import numpy as np

path = sys.argv[1] if len(sys.argv) > 1 else "/tmp/one_phases.bin"
if "--analyze" not in sys.argv:
    os.environ["CLONOS_SCAN_PHASES"] = path
    sys.argv = [sys.argv[0], "64"]
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    import runpy
    runpy.run_path(os.path.join(os.path.dirname(os.path.abspath(__file__)), "probe_one.py"), run_name="__main__")
a = np.fromfile(path, np.uint64).reshape(-1, 8).astype(np.int64)
names = ["stage", "spec", "canon", "entry_wait", "merge+count", "lookback", "emit"]
d = np.diff(a, axis=1)
for i, n in enumerate(names):
    x = d[:, i]
    print(f"{n:12s} mean {x.mean():9.0f} p50 {np.percentile(x, 50):9.0f} p90 {np.percentile(x, 90):9.0f} "
          f"p99 {np.percentile(x, 99):9.0f}")
tot = a[:, 7] - a[:, 0]
print(f"{'total':12s} mean {tot.mean():9.0f} p50 {np.percentile(tot, 50):9.0f} p99 {np.percentile(tot, 99):9.0f}")
t0 = a[:, 0] - a[:, 0].min()
print("kernel span cycles", a[:, 7].max() - a[:, 0].min(), "tiles", len(a))
for q in (0, 0.25, 0.5, 0.75, 1.0):
    i = int(q * (len(a) - 1))
    print(f"  tile {i:6d} start {t0[i]:10d} end {a[i, 7] - a[:, 0].min():10d}")
