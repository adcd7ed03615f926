"""Developer probe: per-phase cycles of the robust jser fill and emit (CLONOS_ROBUST_PHASES
s_memtime stamps, 16 per tile) on config-3 logs.  usage: robust_phases.py [n_logs]"""
import os
import subprocess
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
out = "gpurun_out/robust_phases.bin"
os.makedirs("gpurun_out", exist_ok=True)
env = dict(os.environ, CLONOS_ROBUST_PHASES=out)
n = sys.argv[1] if len(sys.argv) > 1 else "64"
subprocess.run([sys.executable, os.path.join(ROOT, "tools", "robust_run.py"), n, "1"], env=env, check=True)
p = np.fromfile(out, np.uint64).reshape(-1, 16).astype(np.int64)


def deltas(cols, names):
    ok = np.all(p[:, cols] > 0, axis=1)
    q = p[ok][:, cols]
    d = np.diff(q, axis=1)
    print(f"tiles {ok.sum()}:", {nm: round(float(d[:, i].mean()), 1) for i, nm in enumerate(names)},
          "total", round(float((q[:, -1] - q[:, 0]).mean()), 1), "span",
          int(q.max() - q.min()))


deltas([0, 1, 2, 3], ["stage", "count", "parse"])
deltas([8, 9, 10, 11, 12], ["stage", "tables", "phaseA", "phaseB"])
ok = p[:, 12] > 0
print("emit per tile: far records", round(float(p[ok, 13].mean()), 2), "max lane records", round(float(p[ok, 14].mean()), 1),
      "records", round(float((p[ok, 15] & 0xFFFFFFFF).mean()), 1), "rare", round(float((p[ok, 15] >> 32).mean()), 1))
ph = p[ok][:, 11] - p[ok][:, 10]
for q in (50, 90, 99):
    print("phaseA p%d" % q, int(np.percentile(ph, q)))
ok = p[:, 3] > 0
print("jser per tile: candidates", round(float(p[ok, 4].mean()), 1), "general", round(float(p[ok, 5].mean()), 2),
      "max lane", round(float(p[ok, 6].mean()), 2))
q = np.fromfile(out + ".scan", np.uint64).reshape(-1, 8).astype(np.int64)
ok = np.all(q[:, :7] > 0, axis=1)
d = np.diff(q[ok][:, :7], axis=1)
print(f"deferred scan tiles {ok.sum()}:", {nm: round(float(d[:, i].mean()), 1) for i, nm in
      enumerate(["stage", "tables", "bfs", "keep", "parse", "chain"])})
