"""Config 3 decode timing (BASELINE.json configs[2]): mixed variable-length determinants incl.
Serializable and BufferBuilt, 256 subtask logs x 10 epochs (~1 GB) resident in HBM; one
step = batched decode of every log from its first epoch.  Developer tool; prints JSON."""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

ap = argparse.ArgumentParser()
ap.add_argument("--logs", type=int, default=256)
ap.add_argument("--epochs", type=int, default=10)
ap.add_argument("--records", type=int, default=40000, help="records per log per epoch")
ap.add_argument("--steps", type=int, default=5)
ap.add_argument("--decode", default="auto")
args = ap.parse_args()

import torch  # noqa: E402
from clonos_amd import CausalLogID, Engine, _lib, synth  # noqa: E402

rng = np.random.default_rng(synth.SEED_CONFIG3 if hasattr(synth, "SEED_CONFIG3") else 0xC1050003)
t0 = time.time()
epochs = [synth.config3_epoch(args.records, rng, e)[0] for e in range(args.epochs)]
gen_s = time.time() - t0
per_log = sum(int(e.size) for e in epochs)
seg = 16384
eng = Engine(segment_bytes=seg, pool_segments=args.logs * ((per_log + seg - 1) // seg + args.epochs + 1) + 64,
             timing=True, decode=args.decode)
logs = []
for v in range(args.logs):
    log = eng.open_log(CausalLogID.main(v))
    # every log is the same epoch sequence rotated, so that logs differ in layout
    for e in range(args.epochs):
        log.processUpstreamDelta(epochs[(e + v) % args.epochs].tobytes(), 0, e)
    logs.append(log)
eng.sync()
total = per_log * args.logs
n_det = args.logs * args.records * args.epochs
dev = torch.device("cuda", 0)
o_off = torch.empty(n_det, dtype=torch.int32, device=dev)
o_tag = torch.empty(n_det, dtype=torch.uint8, device=dev)
o_v0 = torch.empty(n_det, dtype=torch.int64, device=dev)
wcap = n_det // 2 + 16
o_w = [torch.empty(wcap, dtype=t, device=dev) for t in (torch.int32, torch.int32, torch.int64, torch.int32, torch.int32, torch.uint8)]
dec = _lib.Decoded()
dec.off, dec.tag, dec.v0 = o_off.data_ptr(), o_tag.data_ptr(), o_v0.data_ptr()
dec.w_idx, dec.w_rc, dec.w_v1, dec.w_var_off, dec.w_var_len, dec.w_sub = [t.data_ptr() for t in o_w]
dec.cap, dec.wcap, dec.out_kind = n_det, wcap, _lib.CLG_MEM_DEVICE
handles = np.array([l.handle for l in logs], np.uint32)
starts = np.zeros(len(logs), np.int64)
base = np.zeros(len(logs) + 1, np.uint64)
eng.decode_logs_device(handles, starts, dec, base)
assert dec.n_rec == n_det and dec.err_status == 0, (dec.n_rec, n_det, dec.err_status)
torch.cuda.synchronize()
eng.kernel_stats_reset()
t0 = time.perf_counter()
for _ in range(args.steps):
    eng.decode_logs_device(handles, starts, dec, base)
torch.cuda.synchronize()
el = (time.perf_counter() - t0) / args.steps
st = eng.kernel_stats()
algo = total + 13 * n_det + 25 * int(dec.n_wide)
print(json.dumps({"config": "config3", "log_bytes": total, "n_det": n_det, "n_wide": int(dec.n_wide),
                  "ms_per_step": el * 1e3, "det_per_s": n_det / el, "algo_gbs": algo / el / 1e9, "gen_s": gen_s,
                  "kernels": {k: dict(launches=v["launches"], avg_ms=v["ms"] / max(1, v["launches"]))
                              for k, v in st.items()}}))
