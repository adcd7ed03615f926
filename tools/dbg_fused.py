"""Developer diagnostics for the fused decode: which inputs take the fused path.
Run with CLONOS_FUSED_DEBUG=1 to print the abort reason and tile."""
import sys, numpy as np
sys.path.insert(0, '/root/repo'); sys.path.insert(0, '/root/repo/tests')
from clonos_amd import Engine, synth, CausalLogID
for seg in (256, 16384):
    for nlogs, nrec in [(1, 200000), (2, 200000), (16, 20000), (16, 200000), (64, 100000), (64, 1000000)]:
        e = Engine(segment_bytes=seg, pool_segments=(1 << 31) // seg, timing=True)
        rng = np.random.default_rng(77)
        logs = []
        for v in range(nlogs):
            log = e.open_log(CausalLogID.main(v))
            b, _ = synth.config2_log(nrec, rng)
            log.processUpstreamDelta(b.tobytes(), 0, 1)
            logs.append(log)
        e.kernel_stats_reset()
        dec = e.decode_logs(logs, [1] * nlogs)
        st = e.kernel_stats()
        print(seg, nlogs, nrec, dec.n_rec, "fallback" if "decode_fallback" in st else "fused", flush=True)
        e.close()
