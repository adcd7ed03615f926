"""GPU: batched encode (clg_encode_batch, encode.hip) == SimpleDeterminantEncoder.encodeTo
(SimpleDeterminantEncoder.java:56-75, writers :124-323) record by record.

Every check compares the GPU with the CPU oracle (orc_encode, oracle/clonos_oracle.cpp,
pinned by the hand KATs in test_oracle_kat.py and cross-checked against the Python
restatement pyref.encode_one): (1) determinant objects turned into the SoA layout by hand;
(2) the oracle's decode of the mixed config-3 stream, re-encoded (== the original bytes as
well); (3) logs with long payloads (blocks that do not fit the LDS stage).
"""
import numpy as np
import pytest

import _oracle as O
from clonos_amd import ClonosError, Engine
from clonos_amd import _lib
from clonos_amd import determinants as D
from clonos_amd import synth

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def eng():
    e = Engine(segment_bytes=16384, pool_segments=64, timing=True)
    yield e
    e.close()


def soa_of(dets):
    """Hand-built SoA (no decoder involved): tag, v0, side rows, payload pool."""
    tag, v0, side, var = [], [], [], bytearray()
    for i, d in enumerate(dets):
        if isinstance(d, D.OrderDeterminant):
            tag.append(0), v0.append(d.channel)
        elif isinstance(d, D.TimestampDeterminant):
            tag.append(1), v0.append(d.timestamp)
        elif isinstance(d, D.RNGDeterminant):
            tag.append(2), v0.append(d.number)
        elif isinstance(d, D.BufferBuiltDeterminant):
            tag.append(7), v0.append(d.number_of_bytes)
        elif isinstance(d, D.IgnoreCheckpointDeterminant):
            tag.append(6), v0.append(d.checkpoint_id)
            side.append((i, d.record_count, 0, 0, 0, 0))
        elif isinstance(d, D.TimerTriggerDeterminant):
            tag.append(4), v0.append(d.timestamp)
            name = d.name or b""
            side.append((i, d.record_count, 0, len(var), len(name) if d.callback_type == D.INTERNAL else 0,
                         d.callback_type))
            var += name if d.callback_type == D.INTERNAL else b""
        elif isinstance(d, D.SourceCheckpointDeterminant):
            tag.append(5), v0.append(d.checkpoint_id)
            ref = d.storage_reference
            side.append((i, d.record_count, d.checkpoint_timestamp, len(var), len(ref or b""),
                         d.checkpoint_type | (0x80 if ref is not None else 0)))
            var += ref or b""
        else:
            tag.append(3), v0.append(len(d.stream))
            side.append((i, 0, 0, len(var), len(d.stream), 0))
            var += d.stream
    cols = list(zip(*side)) if side else [[]] * 6
    wrap = lambda xs, bits, t: np.array([x & ((1 << bits) - 1) for x in xs], np.uint64).astype(t)  # noqa: E731
    return (np.array(tag, np.uint8), wrap(v0, 64, np.int64), np.array(cols[0], np.uint32), wrap(cols[1], 32, np.int32),
            wrap(cols[2], 64, np.int64), np.array(cols[3], np.uint32), np.array(cols[4], np.uint32),
            np.array(cols[5], np.uint8), bytes(var))


@pytest.mark.parametrize("seed", range(4))
def test_encode_matches_encoder(eng, seed):
    rng = np.random.default_rng(seed)
    dets = [synth.random_determinant(rng) for _ in range(int(rng.integers(1, 5000)))]
    soa = soa_of(dets)
    want = O.encode_soa(*soa)
    got = eng.encode_batch(*soa)
    assert got == want


def test_encode_roundtrip_config3(eng):
    rng = np.random.default_rng(33)
    buf = synth.config3_epoch(100_000, rng)[0].tobytes()
    st, r, _, _ = O.decode(buf)
    assert st == 0
    soa = (r["tag"], r["v0"], r["w_idx"], r["w_rc"], r["w_v1"], r["w_var_off"], r["w_var_len"], r["w_sub"], buf)
    want = O.encode_soa(*soa)
    assert want == buf
    assert eng.encode_batch(*soa) == want
    dec = eng.decode_host(buf)  # the GPU decode's SoA re-encodes to the same bytes
    assert eng.encode_decoded(dec, buf) == want
    assert eng.kernel_stats()["encode_write"]["launches"] >= 1


def test_encode_long_payloads(eng):
    """Streams and names far larger than a block's LDS stage: direct stores."""
    rng = np.random.default_rng(34)
    parts = []
    for _ in range(30):
        parts.append(D.encode(D.SerializableDeterminant(D.jser_int_array(
            rng.integers(-2**31, 2**31, int(rng.integers(2000, 9000))).tolist()))))
        parts.append(D.encode(D.TimerTriggerDeterminant(1, 2, D.INTERNAL, b"n" * int(rng.integers(0, 40000)))))
        parts.append(synth.random_log(int(rng.integers(1, 3000)), rng))
    buf = b"".join(parts)
    st, r, _, _ = O.decode(buf)
    assert st == 0
    soa = (r["tag"], r["v0"], r["w_idx"], r["w_rc"], r["w_v1"], r["w_var_off"], r["w_var_len"], r["w_sub"], buf)
    want = O.encode_soa(*soa)
    assert want == buf
    assert eng.encode_batch(*soa) == want


def test_encode_errors(eng):
    tag = np.array([0, 1, 9, 2], np.uint8)
    with pytest.raises(ClonosError) as ei:
        eng.encode_batch(tag, np.zeros(4, np.int64))
    assert ei.value.status == _lib.CLG_E_INVALID_ARG and ei.value.bad_index == 2
    # a wide record whose side row names another record
    tag = np.array([0, 6, 0], np.uint8)
    with pytest.raises(ClonosError) as ei:
        eng.encode_batch(tag, np.zeros(3, np.int64), np.array([2], np.uint32), np.zeros(1, np.int32),
                         np.zeros(1, np.int64), np.zeros(1, np.uint32), np.zeros(1, np.uint32), np.zeros(1, np.uint8))
    assert ei.value.bad_index == 1
    assert eng.encode_batch(np.zeros(0, np.uint8), np.zeros(0, np.int64)) == b""
