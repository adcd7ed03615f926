"""Developer diagnostics: the config-2 bench shard through the fused decode, with the
first aborting tile's lane state dumped (CLONOS_FUSED_DEBUG=1) and the raw bytes of that
tile written to gpurun_out/ for offline replay."""
import os, sys, numpy as np
sys.path.insert(0, '/root/repo')
from clonos_amd import Engine, synth, CausalLogID
seed = int(sys.argv[1]) if len(sys.argv) > 1 else 77
e = Engine(segment_bytes=16384, pool_segments=(1 << 31) // 16384, timing=True)
rng = np.random.default_rng(seed)
logs, bufs = [], []
for v in range(64):
    log = e.open_log(CausalLogID.main(v))
    b, _ = synth.config2_log(1000000, rng)
    log.processUpstreamDelta(b.tobytes(), 0, 1)
    logs.append(log); bufs.append(b)
for rep in range(3):
    e.kernel_stats_reset()
    dec = e.decode_logs(logs, [1] * 64)
    print(rep, dec.n_rec, "fallback" if "decode_fallback" in e.kernel_stats() else "fused", flush=True)
os.makedirs("gpurun_out", exist_ok=True)
np.save("gpurun_out/dbg_log3.npy", bufs[3])
