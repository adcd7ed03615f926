"""Developer probe: per-tile phase stamps of the one-pass decode (CLONOS_ONE_PASS=2,
CLONOS_SCAN_PHASES=<file>; tools/one_pass_probe.py): s_memrealtime (100 MHz) at start, after the
canonical exit is published, after the entry wait, after the count, after the look-back, after
emit, at the end; word 7 = XCC id << 32."""
import sys
import numpy as np
a = np.fromfile(sys.argv[1], np.uint64).reshape(-1, 8)
a = a[a.shape[0] // 2:]  # (the second half: the one-pass stamps; the first holds count_tile's)
t0 = a[:, 0].astype(np.int64)
ok = t0 > 0
a = a[ok]
st = a[:, :7].astype(np.int64)
base = st[:, 0].min()
us = (st - base) / 100.0
d = np.diff(us, axis=1)
names = ["stage+spec+canon", "entry wait", "count", "look-back", "emit", "recheck+end"]
print("tiles", len(a), "kernel span us", round(us.max(), 1))
for k, n in enumerate(names):
    print(f"{n:18s} mean {d[:, k].mean():7.2f} us  p50 {np.percentile(d[:, k], 50):7.2f}  p90 {np.percentile(d[:, k], 90):7.2f}  max {d[:, k].max():8.2f}")
xcc = (a[:, 7] >> 32).astype(np.int64) & 7
print("tiles per xcc", np.bincount(xcc, minlength=8))
# start time vs tile index: how far out of order
order = np.argsort(us[:, 0], kind="stable")
print("start time of tile t minus tile t-1 (us): mean", round(np.diff(us[:, 0]).mean(), 3), "p10/p90",
      np.percentile(np.diff(us[:, 0]), [10, 50, 90]).round(2))
print("block lifetime us: mean", round((us[:, 6] - us[:, 0]).mean(), 1))
