"""Developer check: does the fast decode keep long TimerTrigger / SourceCheckpoint /
Serializable records (> 126 bytes, code 0 in the count pass's step-code map, measured from
HBM by the true walk) on the fused path?  Prints the kernel launch counts per batch
(`decode_fallback` present = the batch fell back to the robust pipeline).
usage (GPU box): [CLONOS_LIB=ab/libX.so] python3 tools/dbg_lm.py"""
import os
import sys

sys.path.insert(0, os.getcwd())
import numpy as np

from clonos_amd import Engine, synth
from clonos_amd import determinants as D


def long_batch(rng, n_min, n_max):
    parts = []
    for i in range(400):
        parts.append(synth.config3_epoch(int(rng.integers(5, 60)), rng)[0].tobytes())
        k = i % 4
        n = int(rng.integers(n_min, n_max))
        if k == 0:
            parts.append(D.encode(D.TimerTriggerDeterminant(i, 7 * i, D.INTERNAL, b"A" * n)))
        elif k == 1:
            parts.append(D.encode(D.SourceCheckpointDeterminant(i, i, 3 * i, D.CHECKPOINT, b"r" * n)))
        elif k == 2:
            parts.append(D.encode(D.SerializableDeterminant(D.jser_string("s" * n))))
    return b"".join(parts)


e = Engine(segment_bytes=16384, pool_segments=(1 << 26) // 16384, timing=True)
rng = np.random.default_rng(21)
for name, lo, hi in (("short", 10, 100), ("short", 10, 100), ("long", 100, 320), ("long", 100, 320)):
    e.kernel_stats_reset()
    e.decode_host(long_batch(rng, lo, hi))
    print(name, {k: v["launches"] for k, v in e.kernel_stats().items()}, flush=True)
e.close()
