"""Developer probe (not part of the product or the tests): the write path's kernel time for the
whole config-3 log (256 logs x 10 epochs, 0.9 GB) written as 10 batched device-input upstream
calls, with the Serializable candidate lists (the sidecar) and without (CLONOS_SIDECAR=0).
Each variant is written twice on fresh engines and the second write is reported (the first
warms the GPU).  Run it against builds of the library (CLONOS_LIB) to split the sidecar's cost,
e.g. one whose lists hold positions only (sidecar)."""
import json
import os
import sys

sys.path.insert(0, ".")
import numpy as np  # noqa: E402
import torch  # noqa: E402
from clonos_amd import CausalLogID, Engine, _lib, synth  # noqa: E402
from clonos_amd import dist as X  # noqa: E402

n_logs, n_epochs, per_epoch, seg = 256, 10, 40000, 16384
rng = np.random.default_rng(synth.SEED_CONFIG3)
epochs = [synth.config3_epoch(per_epoch, rng, e)[0] for e in range(n_epochs)]
per_log = sum(int(e.size) for e in epochs)
blob = np.concatenate(epochs)
eoff = np.concatenate([[0], np.cumsum([int(x.size) for x in epochs])]).astype(np.uint64)
d_blob = torch.from_numpy(blob).cuda()


def write_once(sidecar):
    if not sidecar:
        os.environ["CLONOS_SIDECAR"] = "0"
    e_ = Engine(segment_bytes=seg, pool_segments=n_logs * ((per_log + seg - 1) // seg + n_epochs + 1) + 64,
                timing=True, ifl_pool_segments=16)
    os.environ.pop("CLONOS_SIDECAR", None)
    try:
        ls = [e_.open_log(CausalLogID.main(v)) for v in range(n_logs)]
        torch.cuda.synchronize()
        e_.kernel_stats_reset()
        for e in range(n_epochs):
            req = np.zeros(n_logs, X.DELTA_REQ)
            req["log"] = [lg.handle for lg in ls]
            req["epoch"] = e
            k = (np.arange(n_logs) + e) % n_epochs
            req["src_off"] = eoff[k]
            req["len"] = (eoff[k + 1] - eoff[k]).astype(np.uint32)
            e_.upstream_delta_batch(req.ctypes.data, n_logs, d_blob.data_ptr(), _lib.CLG_MEM_DEVICE)
        torch.cuda.synchronize()
        return round(e_.kernel_stats().get("upstream_scatter", {"ms": 0.0})["ms"], 4)
    finally:
        e_.close()


out = {}
for sc in (1, 0):
    write_once(sc)  # warm-up
    out["sidecar" if sc else "none"] = write_once(sc)
print(os.environ.get("CLONOS_LIB", "default"), json.dumps(out))
