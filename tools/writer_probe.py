import os, sys, json, time
sys.path.insert(0, ".")
import numpy as np, torch
from clonos_amd import CausalLogID, Engine, _lib, synth
from clonos_amd import dist as X
n_logs, n_epochs, per_epoch, seg = 256, 10, 40000, 16384
rng = np.random.default_rng(synth.SEED_CONFIG3)
epochs = [synth.config3_epoch(per_epoch, rng, e)[0] for e in range(n_epochs)]
per_log = sum(int(e.size) for e in epochs)
total = per_log * n_logs
blob = np.concatenate(epochs)
eoff = np.concatenate([[0], np.cumsum([int(x.size) for x in epochs])]).astype(np.uint64)
d_blob = torch.from_numpy(blob).cuda()
out = {}
for sc in (1, 0):
    if not sc: os.environ["CLONOS_SIDECAR"] = "0"
    e_ = Engine(segment_bytes=seg, pool_segments=n_logs * ((per_log + seg - 1) // seg + n_epochs + 1) + 64, timing=True, ifl_pool_segments=16)
    os.environ.pop("CLONOS_SIDECAR", None)
    ls = [e_.open_log(CausalLogID.main(v)) for v in range(n_logs)]
    torch.cuda.synchronize(); e_.kernel_stats_reset()
    for e in range(n_epochs):
        req = np.zeros(n_logs, X.DELTA_REQ)
        req["log"] = [l.handle for l in ls]; req["epoch"] = e
        k = (np.arange(n_logs) + e) % n_epochs
        req["src_off"] = eoff[k]; req["len"] = (eoff[k + 1] - eoff[k]).astype(np.uint32)
        e_.upstream_delta_batch(req.ctypes.data, n_logs, d_blob.data_ptr(), _lib.CLG_MEM_DEVICE)
    torch.cuda.synchronize()
    st = e_.kernel_stats().get("upstream_scatter", {"ms": 0, "launches": 0})
    out["sidecar" if sc else "none"] = round(st["ms"], 4)
    e_.close()
print(os.environ.get("CLONOS_LIB", "default"), json.dumps(out))
