"""GPU: small whole spans decoded a lane each (decode_fused.hip tiny_tiles) -- a batch of many
small logs, as config 4's 65 536 subpartition logs of 320 bytes -- bit-exact against the
oracle, including runs that hold a record of a field-length tag (the wave path takes them),
invalid tags and records past the span end (the per-span fallback reports them exactly as the
robust pipeline).  SimpleDeterminantEncoder.decodeNext (:78-342)."""
import numpy as np
import pytest

from clonos_amd import CausalLogID, ClonosError, Engine
from clonos_amd import determinants as D
from test_gpu_decode import assert_span_equal

pytestmark = pytest.mark.gpu


def _fixed_log(rng, nbytes):
    """Order / Timestamp / RNG / BufferBuilt / IgnoreCheckpoint records up to ~nbytes."""
    out = b""
    while len(out) < nbytes:
        k = int(rng.integers(0, 5))
        d = [lambda: D.OrderDeterminant(int(rng.integers(-128, 128))),
             lambda: D.TimestampDeterminant(int(rng.integers(0, 1 << 62))),
             lambda: D.RNGDeterminant(int(rng.integers(-(1 << 31), 1 << 31))),
             lambda: D.BufferBuiltDeterminant(int(rng.integers(0, 1 << 31))),
             lambda: D.IgnoreCheckpointDeterminant(int(rng.integers(0, 100)), int(rng.integers(0, 1 << 40)))][k]()
        out += D.encode(d)
    return out


def _logs_decode(bufs, decode="three_pass"):
    with Engine(segment_bytes=16384, pool_segments=len(bufs) + 64, timing=True, decode=decode) as eng:
        logs = []
        for v, b in enumerate(bufs):
            log = eng.open_log(CausalLogID.sub(v, 1, 2, v % 100))
            if b:
                log.processUpstreamDelta(b, 0, 0)
            logs.append(log)
        eng.sync()
        dec = eng.decode_logs(logs, [0] * len(logs))
        return dec, eng.kernel_stats()


@pytest.mark.parametrize("seed", range(3))
def test_many_small_logs(seed):
    rng = np.random.default_rng(100 + seed)
    bufs = [_fixed_log(rng, int(rng.integers(1, 1100))) for _ in range(700)]
    bufs[5] = b""  # an empty log
    if seed == 1:  # a field-length record here and there: those runs take the wave path
        for i in range(3, 700, 97):
            bufs[i] += D.encode(D.TimerTriggerDeterminant(1, 2, 3)) + D.encode(
                D.SourceCheckpointDeterminant(4, 5, 6, D.CHECKPOINT, b"ref"))
    dec, st = _logs_decode(bufs)
    assert "decode_fallback" not in st and "decode_span_fallback" not in st
    for s, b in enumerate(bufs):
        assert_span_equal(dec, s, b)


@pytest.mark.parametrize("kind", ["tag", "truncated"])
def test_small_log_errors_equal_robust(kind):
    """An invalid tag / a record past the end in one small log among many: the first error
    (status, span, offset, tag) and the records before it equal the robust pipeline's."""
    rng = np.random.default_rng(7)
    bufs = [_fixed_log(rng, int(rng.integers(50, 900))) for _ in range(300)]
    if kind == "tag":  # a record boundary, then tag 9
        bufs[123] = _fixed_log(rng, 60) + b"\x09" + _fixed_log(rng, 200)
    else:  # a Timestamp's tag and its first four bytes at the end
        bufs[123] += D.encode(D.TimestampDeterminant(9))[:5]
    errs = []
    for mode in ("auto", "robust"):
        with pytest.raises(ClonosError) as ei:
            _logs_decode(bufs, mode)
        x = ei.value
        errs.append((x.status, x.err_span, x.err_off, x.err_tag, x.n_rec))
    assert errs[0] == errs[1] and errs[0][1] == 123


def test_full_runs_of_small_spans():
    """More small spans than 64 per count block (262 144 spans of 300 bytes): the lane path
    takes full runs of 64 tiles; every span's records are counted and placed exactly."""
    from clonos_amd import synth
    rng = np.random.default_rng(11)
    n_spans, per = 262144, 60
    kd = synth.KINDS["buffer_built"]
    blob, _ = synth.build(np.zeros(n_spans * per, np.int64), [kd], {0: [rng.integers(0, 1 << 31, n_spans * per)]})
    L = per * 5
    spans = [(i * L, L) for i in range(n_spans)]
    with Engine(segment_bytes=16384, pool_segments=64, timing=True, decode="three_pass") as eng:
        dec = eng.decode_host(blob, spans)
        st = eng.kernel_stats()
    assert "decode_fallback" not in st and "decode_span_fallback" not in st
    assert dec.n_rec == n_spans * per
    np.testing.assert_array_equal(np.diff(dec.span_rec_base.astype(np.int64)), per)
    b = blob.tobytes()
    for s in rng.integers(0, n_spans, 40):
        assert_span_equal(dec, int(s), b[s * L:(s + 1) * L])
