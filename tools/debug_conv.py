"""Developer diagnostics: decode a config-2 log with CLONOS_DEBUG_DUMP and summarise the
convergence points / tile summaries (not part of the product or the tests)."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ["CLONOS_DEBUG_DUMP"] = "gpurun_out/conv_dump.bin"
from clonos_amd import Engine, synth  # noqa: E402

from clonos_amd import CausalLogID  # noqa: E402

rng = np.random.default_rng(synth.SEED_CONFIG2)
n = int(sys.argv[1]) if len(sys.argv) > 1 else 300_000
nlogs = int(sys.argv[2]) if len(sys.argv) > 2 else 1
bufs = [synth.config2_log(n, rng) for _ in range(nlogs)]
buf, offs = bufs[0]
with Engine(timing=True, pool_segments=1 << 16) as eng:
    logs = []
    for i, (b, o) in enumerate(bufs):
        lg = eng.open_log(CausalLogID.main(i))
        lg.processUpstreamDelta(b.tobytes(), 0, 1)
        logs.append(lg)
    dec = eng.decode_logs(logs, [1] * nlogs)
    st = eng.kernel_stats()
print("n_rec", dec.n_rec, "expected", n * nlogs)
for k, v in st.items():
    print(k, v)
raw = open("gpurun_out/conv_dump.bin", "rb").read()
nt, ns = np.frombuffer(raw[:8], np.uint32)
o = 8
conv = np.frombuffer(raw[o:o + nt * 64 * 4], np.uint32).reshape(nt, 64)
o += nt * 64 * 4
sums = np.frombuffer(raw[o:o + nt * 24], np.uint8).reshape(nt, 24)
o += nt * 24
flags = np.frombuffer(raw[o:o + ns * 4], np.uint32)
unknown = (conv == 0xFFFFFFFF)
print("tiles", nt, "spans", ns, "flags", flags.tolist()[:8])
print("unknown points: %.3f" % unknown.mean(), "per region index:", unknown.mean(axis=0)[:8])
f = sums[:, 8]
x = sums[:, 9]
print("f hist", np.bincount(f, minlength=3)[:5], "x hist", np.bincount(x, minlength=3)[:5], "x==255", (x == 255).sum())
o += nt * 32  # tile descriptors
pw = np.frombuffer(raw[o:o + nt * 64 * 4], np.uint32).reshape(nt, 64)
pops = pw & 0xFFFF
live = (pw >> 16) & 0x7FFF
far = pw >> 31
print("far-collision returns", far.sum(), "unknown with live==0", ((conv == 0xFFFFFFFF) & (live == 0)).sum(),
      "unknown total", (conv == 0xFFFFFFFF).sum(), "pops>=2047", (pops >= 2047).sum())
uk = np.argwhere(conv == 0xFFFFFFFF)[:8]
print("unknown samples (tile, lane, pops, live):", [(int(a), int(b), int(pops[a, b]), int(live[a, b])) for a, b in uk])
print("pops per region: mean %.1f p50 %d p99 %d max %d; per-tile max mean %.1f" % (
    pops.mean(), np.median(pops), np.percentile(pops, 99), pops.max(), pops.max(axis=1).mean()))
starts = set(offs.tolist())
# how many known conv points are true record starts (tile aligned coords: tile k covers [k*16384, ...) for host spans aligned at 0)
good = bad = 0
for t in range(min(nt, 50 if nlogs == 1 else 0)):
    for l in range(64):
        c = int(conv[t, l])
        if c == 0xFFFFFFFF:
            continue
        if (t * 16384 + c) in starts:
            good += 1
        else:
            bad += 1
print("points on true path:", good, "off path:", bad)
conv_off = conv.astype(np.int64) - np.arange(64)[None, :] * 256
kn = ~unknown
print("distance of point past region start: mean %.1f max %d" % (conv_off[kn].mean(), conv_off[kn].max()))
