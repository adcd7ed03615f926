"""Developer probe: which tiles of a config-3 batch the robust pipeline's convergence-point
tier (decode_fast.hip) cannot chain, so that their spans go to the DP tier.  Decodes 8
config-3 logs robustly with CLONOS_DEBUG_DUMP and prints, per flagged span, the first tile
whose chain breaks (its span offset: the records there come from the same generator).  JSON lines."""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
out_dir = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/robust_probe"
os.makedirs(out_dir, exist_ok=True)
dump = os.path.join(out_dir, "dump.bin")
os.environ["CLONOS_DEBUG_DUMP"] = dump
import torch  # noqa: E402,F401
from clonos_amd import CausalLogID, Engine, synth  # noqa: E402
from clonos_amd import determinants as D  # noqa: E402

N_LOGS, N_EP, PER = 8, 10, 40000
rng = np.random.default_rng(synth.SEED_CONFIG3)
gen = [synth.config3_epoch(PER, rng, e) for e in range(N_EP)]
seg = 16384
eng = Engine(segment_bytes=seg, pool_segments=N_LOGS * 400 + 64, timing=True, decode="robust", ifl_pool_segments=16)
logs, blobs = [], []
for v in range(N_LOGS):
    l = eng.open_log(CausalLogID.main(v))
    parts = []
    for e in range(N_EP):
        b = gen[(e + v) % N_EP][0]
        l.processUpstreamDelta(b.tobytes(), 0, e)
        parts.append(b.tobytes())
    logs.append(l)
    blobs.append(b"".join(parts))
dec = eng.decode_logs(logs, [0] * N_LOGS)
eng.close()
raw = open(dump, "rb").read()
nt, ns = np.frombuffer(raw[:8], np.uint32)
o = 8
o += nt * 64 * 4  # convergence points
sums = np.frombuffer(raw[o:o + nt * 24], np.dtype([("cnt", "<u4"), ("wcnt", "<u4"), ("f", "u1"), ("x", "u1"),
                                                   ("pad", "u1", 2), ("pad2", "<u4"), ("valid", "<u8")]))
o += nt * 24
flags = np.frombuffer(raw[o:o + ns * 4], np.uint32)
o += ns * 4
tiles = np.frombuffer(raw[o:o + nt * 32], np.dtype([("abase", "<u8"), ("delta", "<u4"), ("len", "<u4"), ("span", "<u4"),
                                                   ("pad", "<u4"), ("span_off", "<u8")]))
print(json.dumps({"tiles": int(nt), "spans": int(ns), "flagged": int((flags != 0).sum())}), flush=True)


for s in np.nonzero(flags)[0].tolist():
    ti = np.nonzero(tiles["span"] == s)[0]
    bad = None
    for i, t in enumerate(ti):
        sm = sums[t]
        why = []
        if sm["x"] == 0xFF:
            why.append("x_fail")
        if sm["f"] == 0xFF:
            why.append("f_fail")
        if i == 0 and sm["f"] != 0:
            why.append("first_f_not_0")
        if i > 0 and sums[ti[i - 1]]["x"] != sm["f"]:
            why.append(f"prev_x_{int(sums[ti[i - 1]]['x'])}_ne_f_{int(sm['f'])}")
        if why:
            bad = (i, int(t), why, int(tiles[t]["span_off"]))
            break
    print(json.dumps({"span": s, "flag": int(flags[s]), "tiles": len(ti), "first_break": bad}), flush=True)
