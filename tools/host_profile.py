"""Developer diagnostics: wall-clock split of one bench step (decode call, consumer
seeks, slice call) on the config-2 workload.  Not part of the product or the tests."""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from clonos_amd import CausalLogID, Engine, _lib, synth  # noqa: E402

nlogs = int(sys.argv[1]) if len(sys.argv) > 1 else 64
rng = np.random.default_rng(synth.SEED_CONFIG2)
bufs = [synth.config2_log(1_000_000, rng) for _ in range(nlogs)]
eng = Engine(segment_bytes=16384, pool_segments=nlogs * 360, timing=False, async_slice=True)
logs = []
for i, (b, _) in enumerate(bufs):
    lg = eng.open_log(CausalLogID.main(i))
    lg.processUpstreamDelta(b.tobytes(), 0, 1)
    logs.append(lg)
cons = [(i, (c + 1, i), int(o[int(rng.integers(0, len(o)))])) for i, (_, o) in enumerate(bufs) for c in range(8)]
total = sum(b.size - off for (b, _), (i, _, off) in zip([bufs[i] for i, _, _ in cons], cons))
n_det = nlogs * 1_000_000
dev = torch.device("cuda", 0)
o_off = torch.empty(n_det, dtype=torch.int32, device=dev)
o_tag = torch.empty(n_det, dtype=torch.uint8, device=dev)
o_v0 = torch.empty(n_det, dtype=torch.int64, device=dev)
o_w = [torch.empty(1024, dtype=t, device=dev) for t in (torch.int32, torch.int32, torch.int64, torch.int32, torch.int32, torch.uint8)]
o_slice = torch.empty(total + 64, dtype=torch.uint8, device=dev)
dec = _lib.Decoded()
dec.off, dec.tag, dec.v0 = o_off.data_ptr(), o_tag.data_ptr(), o_v0.data_ptr()
dec.w_idx, dec.w_rc, dec.w_v1, dec.w_var_off, dec.w_var_len, dec.w_sub = [t.data_ptr() for t in o_w]
dec.cap, dec.wcap, dec.out_kind = n_det, 1024, _lib.CLG_MEM_DEVICE
handles = np.array([l.handle for l in logs], np.uint32)
starts = np.ones(nlogs, np.int64)
base = np.zeros(nlogs + 1, np.uint64)
creq = (_lib.SliceReq * len(cons))()
cres = (_lib.SliceRes * len(cons))()
for k, (i, ch, _) in enumerate(cons):
    creq[k].log = logs[i].handle
    creq[k].consumer = _lib.ChannelId(ch[0], ch[1])
    creq[k].epoch = 1
seek_offs = np.array([off for _, _, off in cons], np.int32)
T = {"decode_call": [], "seek_call": [], "slice_call(async)": [], "step": []}
for it in range(12):
    t0 = time.perf_counter()
    eng.decode_logs_device(handles, starts, dec, base)
    t1 = time.perf_counter()
    eng.seek_consumers_raw(creq, seek_offs, len(cons))
    t2 = time.perf_counter()
    eng.slice_batch_raw(creq, cres, len(cons), o_slice.data_ptr(), o_slice.numel(), device=True)
    t3 = time.perf_counter()
    if it >= 2:
        T["decode_call"].append(t1 - t0); T["seek_call"].append(t2 - t1); T["slice_call(async)"].append(t3 - t2)
        T["step"].append(t3 - t0)
torch.cuda.synchronize()
print({k: round(1e3 * float(np.mean(v)), 3) for k, v in T.items()}, "ms")
eng.close()
