"""Developer probe: the count / emit kernels on config-4-shaped batches -- only the 65 536
small subpartition spans, only the 640 main-log spans, both -- to see where the count pass of
a config-4 decode spends its time.  Prints JSON lines."""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402,F401
from clonos_amd import CausalLogID, Engine, _lib, synth  # noqa: E402

rng = np.random.default_rng(4)
n_sub, n_main = 65536, 640
subs = [synth.build(np.zeros(64, np.int64), [synth.KINDS["buffer_built"]], {0: [rng.integers(1, 32769, 64)]})[0]
        for _ in range(1)]
sub_b = subs[0].tobytes()
main_b = synth.config2_log(4096, rng)[0].tobytes()
eng = Engine(segment_bytes=16384, pool_segments=n_sub * 2 + n_main * 8 + 64, timing=True, ifl_pool_segments=16)
hs, kinds = [], []
for v in range(n_main):
    l = eng.open_log(CausalLogID.main(v))
    l.processUpstreamDelta(main_b, 0, 0)
    l.processUpstreamDelta(main_b, 0, 1)
    hs.append(l.handle); kinds.append(1)
for v in range(n_sub):
    l = eng.open_log(CausalLogID.sub(v % 640, 1, 2, v // 640))
    l.processUpstreamDelta(sub_b, 0, 0)
    l.processUpstreamDelta(sub_b, 0, 1)
    hs.append(l.handle); kinds.append(0)
eng.sync()
hs, kinds = np.array(hs, np.uint32), np.array(kinds)
cap = n_main * 4096 + n_sub * 64 + 16
dev = torch.device("cuda", 0)
o = [torch.empty(cap, dtype=t, device=dev) for t in (torch.int32, torch.uint8, torch.int64)]
ow = [torch.empty(16, dtype=t, device=dev) for t in (torch.int32, torch.int32, torch.int64, torch.int32, torch.int32, torch.uint8)]
dec = _lib.Decoded()
dec.off, dec.tag, dec.v0 = [t.data_ptr() for t in o]
dec.w_idx, dec.w_rc, dec.w_v1, dec.w_var_off, dec.w_var_len, dec.w_sub = [t.data_ptr() for t in ow]
dec.cap, dec.wcap, dec.out_kind = cap, 16, _lib.CLG_MEM_DEVICE
for name, sel in (("subs", kinds == 0), ("mains", kinds == 1), ("both", kinds >= 0)):
    h = np.ascontiguousarray(hs[sel])
    st = np.ones(len(h), np.int64)
    base = np.zeros(len(h) + 1, np.uint64)
    eng.decode_logs_device(h, st, dec, base)
    eng.kernel_stats_reset()
    for _ in range(5):
        eng.decode_logs_device(h, st, dec, base)
    k = eng.kernel_stats()
    print(json.dumps({"batch": name, "spans": int(len(h)), "n_rec": int(dec.n_rec),
                      **{n: round(v["ms"] / v["launches"], 4) for n, v in k.items() if v["launches"]}}), flush=True)
