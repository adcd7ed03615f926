"""GPU: the fast decode in parts (clg_config.decode_parts) -- the count pass of part k + 1
beside the scan and emit of part k on a second stream -- gives exactly the one-part result:
every SoA word, the span ranges, the per-span fallback, bit-exact against the oracle.

Parts split at multiples of the 1024-tile scan block and need 2048 tiles (16 MiB) each, so
the batches here are 40-60 MB.  SimpleDeterminantEncoder.decodeNext (:78-342)."""
import numpy as np
import pytest

from clonos_amd import CausalLogID, Engine
from clonos_amd import determinants as D
from clonos_amd import synth
from test_gpu_decode import assert_span_equal

pytestmark = pytest.mark.gpu

FIELDS = ("off", "tag", "v0", "w_idx", "w_rc", "w_v1", "w_var_off", "w_var_len", "w_sub", "span_rec_base")


def _decode(bufs, parts, start_epoch=0):
    with Engine(segment_bytes=16384, pool_segments=sum(len(b) for b in bufs) // 16384 + 8 * len(bufs) + 64,
                timing=True, decode_parts=parts) as eng:
        logs = []
        for v, b in enumerate(bufs):
            log = eng.open_log(CausalLogID.main(v))
            log.processUpstreamDelta(b, 0, start_epoch)
            logs.append(log)
        eng.sync()
        out = []
        for _ in range(2):  # the first batch may learn the Serializable table hint
            eng.kernel_stats_reset()
            out.append(eng.decode_logs(logs, [start_epoch] * len(logs)))
        return out[-1], eng.kernel_stats()


def _same(a, b):
    for f in FIELDS:
        np.testing.assert_array_equal(getattr(a, f), getattr(b, f), err_msg=f)


@pytest.mark.parametrize("parts", [2, 3, 4])
def test_parts_config2(parts):
    rng = np.random.default_rng(0xC1050002 + parts)
    bufs = [synth.config2_log(int(rng.integers(1_000_000, 1_400_000)), rng)[0].tobytes() for _ in range(12)]
    one, st1 = _decode(bufs, 1)
    many, stp = _decode(bufs, parts)
    tiles = sum(-(-len(b) // 8192) for b in bufs)  # (segments hold two whole tiles)
    assert "decode_parts" not in st1 and stp["decode_parts"]["launches"] == min(parts, tiles // 2048)
    _same(one, many)
    for s in (0, 5, 11):
        assert_span_equal(many, s, bufs[s])


def test_parts_config3_tables():
    """Serializable records: each part builds its own tables (k_decode_jser over the part's
    tiles, the general walker over the part's candidates) before its count."""
    rng = np.random.default_rng(0xC1050003)
    bufs = [b"".join(synth.config3_epoch(60000, rng, e)[0].tobytes() for e in range(7)) for _ in range(12)]
    one, _ = _decode(bufs, 1)
    many, stp = _decode(bufs, 3)
    assert stp["decode_parts"]["launches"] == 3 and "decode_fallback" not in stp
    _same(one, many)
    for s in (0, 11):
        assert_span_equal(many, s, bufs[s])


def test_parts_span_fallback():
    """A span the fast pass cannot settle (a 16-byte aligned odd Order chain) in the middle
    part: the per-span fallback re-runs scan + emit over the whole batch after the parted
    count; the result equals the one-part decode and the oracle."""
    rng = np.random.default_rng(5)
    bufs = [synth.config2_log(1_000_000, rng)[0].tobytes() for _ in range(9)]
    bufs[4] = D.encode(D.TimestampDeterminant(5)) + D.encode(D.OrderDeterminant(0)) * 400_000
    one, st1 = _decode(bufs, 1)
    many, stp = _decode(bufs, 3)
    assert "decode_span_fallback" in stp and "decode_fallback" not in stp
    _same(one, many)
    assert_span_equal(many, 4, bufs[4])
