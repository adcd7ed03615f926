"""Developer probe: test_decode_logs_segment_sizes[48] outside pytest, with the span-level
difference against the oracle (first differing record) and the decode paths taken."""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import torch  # noqa: E402,F401
import _oracle as O  # noqa: E402  (checker)
from clonos_amd import CausalLogID, Engine, synth  # noqa: E402

os.environ["CLONOS_FUSED_DEBUG"] = "1"
for seg in (48,):
    rng = np.random.default_rng(seg)
    with Engine(segment_bytes=seg, pool_segments=(1 << 22) // seg + 64, timing=True) as eng:
        logs = []
        for v in range(5):
            log = eng.open_log(CausalLogID.main(v))
            b, _ = synth.config2_log(int(rng.integers(1000, 60000)), rng)
            log.processUpstreamDelta(b.tobytes(), 0, 0)
            for _ in range(int(rng.integers(0, 400))):
                log.appendDeterminant(synth.random_determinant(rng), 1)
            logs.append(log)
        start = [int(rng.integers(0, 2)) for _ in logs]
        expect = [log.getDeterminants(e) for log, e in zip(logs, start)]
        eng.kernel_stats_reset()
        dec = eng.decode_logs(logs, start)
        ks = eng.kernel_stats()
        out = {"seg": seg, "paths": {k: v["launches"] for k, v in ks.items() if "fallback" in k or "repair" in k}}
        spans = []
        for s, b in enumerate(expect):
            st, r, _, _ = O.decode(b)
            sl = dec.span_slice(s)
            got = dec.off[sl]
            n = min(len(got), len(r["off"]))
            diff = np.nonzero(got[:n] != r["off"][:n])[0]
            d0 = int(diff[0]) if len(diff) else None
            spans.append({"span": s, "bytes": len(b), "want": int(len(r["off"])), "got": int(len(got)),
                          "first_diff": d0, "at_off": int(r["off"][d0]) if d0 is not None else None,
                          "want_offs": r["off"][max(0, d0 - 6):d0 + 12].tolist() if d0 is not None else None,
                          "got_offs": got[max(0, d0 - 6):d0 + 12].tolist() if d0 is not None else None,
                          "want_tags": r["tag"][max(0, d0 - 6):d0 + 12].tolist() if d0 is not None else None})
        out["spans"] = spans
        print(json.dumps(out), flush=True)
