"""GPU: records longer than a fast-decode tile (8 KiB) stay on the fast path.

A TimerTrigger name of 40 KB or a Serializable stream of 9 KB anywhere in a batch used to
send the whole batch to the robust pipeline.  Each case is decoded bit-exact against the
oracle and must not fall back (16 KiB segments; a record may cross segments, tiles and
the count pass's chunk boundaries).  SimpleDeterminantEncoder.java:228-242 (TimerTrigger
name), :273-287 (SourceCheckpoint reference), :333-341 (Serializable stream)."""
import numpy as np
import pytest

from clonos_amd import Engine
from clonos_amd import determinants as D
from clonos_amd import synth
from test_gpu_decode import assert_span_equal

pytestmark = pytest.mark.gpu


def fell_back(eng) -> bool:
    return "decode_fallback" in eng.kernel_stats()


@pytest.fixture
def leng():
    e = Engine(segment_bytes=16384, pool_segments=1 << 14, timing=True)
    yield e
    e.close()


def _long(kind: str, n: int, i: int = 0) -> bytes:
    if kind == "timer":
        return D.encode(D.TimerTriggerDeterminant(i, 7 * i, D.INTERNAL, bytes([65 + i % 26]) * n))
    if kind == "checkpoint":
        return D.encode(D.SourceCheckpointDeterminant(i, i, 3 * i, D.CHECKPOINT, b"r" * n))
    if kind == "string":
        return D.encode(D.SerializableDeterminant(D.jser_string("s" * n)))
    if kind == "intarray":
        return D.encode(D.SerializableDeterminant(D.jser_int_array(list(range(n // 4)))))
    raise ValueError(kind)


@pytest.mark.parametrize("kind,n", [("timer", 40000), ("checkpoint", 20000), ("string", 9000),
                                    ("intarray", 9000), ("timer", 9000), ("string", 30000)])
def test_long_record_stays_fast(leng, kind, n):
    rng = np.random.default_rng(n)
    for pos in range(3):  # the long record at different offsets (tile / chunk phases)
        head = synth.config3_epoch(3000 + 1777 * pos, rng)[0].tobytes()
        tail = synth.config3_epoch(5000, rng)[0].tobytes()
        buf = head + _long(kind, n, pos) + tail
        for _ in range(2):  # the first batch may learn the Serializable table hint
            leng.kernel_stats_reset()
            dec = leng.decode_host(buf)
            assert_span_equal(dec, 0, buf)
        assert not fell_back(leng), (kind, n, pos)


def test_config3_batch_with_long_records(leng):
    """The verdict's case: a config-3 batch (many spans) with one 40 KB TimerTrigger name
    and one 9 KB Serializable stream, bit-exact and on the fast path."""
    rng = np.random.default_rng(0xC1050003)
    spans = []
    for i in range(12):
        b, offs = synth.config3_epoch(20000, rng)
        b = b.tobytes()
        if i == 3:
            k = int(offs[len(offs) // 2])
            b = b[:k] + _long("timer", 40000, 3) + b[k:]
        if i == 7:
            k = int(offs[len(offs) // 3])
            b = b[:k] + _long("intarray", 9000) + b[k:]
        spans.append(b)
    blob, sp = b"", []
    for b in spans:
        sp.append((len(blob), len(b)))
        blob += b
    for _ in range(2):
        leng.kernel_stats_reset()
        dec = leng.decode_host(blob, sp)
        for s, b in enumerate(spans):
            assert_span_equal(dec, s, b)
    assert not fell_back(leng)
