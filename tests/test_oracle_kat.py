"""CPU: pin the oracle against known-answer vectors and the reference's own tests.

Sources of truth (no golden vectors exist in the reference for this path):
  * byte layouts derived by hand from SimpleDeterminantEncoder.java:124-323;
  * Java Object Serialization spec streams (String, Boolean) -- parity unpinned;
  * NettyTests.java:144-186 (composite slice + discardReadComponents) -- the only
    reference test on the log's buffer semantics;
  * QueueTest.java:60-72 (Order replay channels 1,2,2).
Then the C++ oracle is cross-checked against the independent Python restatement.
"""
import numpy as np
import pytest

import _oracle as O
from _oracle import pyref
from clonos_amd import determinants as D
from clonos_amd import synth

KAT_ENCODE = [
    (D.OrderDeterminant(3), "0003"),
    (D.TimestampDeterminant(0x0102030405060708), "01" "0102030405060708"),
    (D.RNGDeterminant(-1), "02" "ffffffff"),
    (D.BufferBuiltDeterminant(32768), "07" "00008000"),
    (D.TimerTriggerDeterminant(7, 1, D.INTERNAL, b"PTS"), "04" "00000007" "0000000000000001" "06" "00000003" "505453"),
    (D.TimerTriggerDeterminant(7, 1, D.WATERMARK), "04" "00000007" "0000000000000001" "00"),
    (D.SourceCheckpointDeterminant(0, 1, 2, D.CHECKPOINT, b""),
     "05" "00000000" "0000000000000001" "0000000000000002" "00" "01" "00000000"),
    (D.SourceCheckpointDeterminant(0, 1, 2, D.SAVEPOINT, None), "05" "00000000" "0000000000000001" "0000000000000002" "01" "00"),
    (D.IgnoreCheckpointDeterminant(5, 9), "06" "00000005" "0000000000000009"),
    (D.SerializableDeterminant(D.jser_string("abc")), "03" "aced0005" "740003" "616263"),
]

BOOLEAN_TRUE = bytes.fromhex("aced0005737200116a6176612e6c616e672e426f6f6c65616ecd207280d59cfaee0200015a000576616c7565787001")


@pytest.mark.parametrize("det,hexs", KAT_ENCODE)
def test_encode_kat(det, hexs):
    assert D.encode(det).hex() == hexs
    # both oracle encoders reproduce the hand-derived bytes from the decoded fields
    raw = bytes.fromhex(hexs)
    st, r, _, _ = O.decode(raw)
    assert st == 0 and len(r["tag"]) == 1
    assert O.encode_soa(r["tag"], r["v0"], r["w_idx"], r["w_rc"], r["w_v1"], r["w_var_off"], r["w_var_len"],
                        r["w_sub"], raw) == raw
    d = pyref.decode_all(raw)[0]
    assert pyref.encode_one(d["tag"], d["v0"], d["rc"], d["v1"], d["sub"],
                            raw[d["var_off"]:d["var_off"] + d["var_len"]]) == raw


def test_record_sizes_match_reference():
    # getEncodedSizeInBytes overrides (Order 2, Timestamp 9, RNG 5, BufferBuilt 5, Ignore 13,
    # TimerTrigger 14 / 18+name, SourceCheckpoint 23 / 27+ref, Serializable 1+stream)
    assert D.encoded_size(D.OrderDeterminant(0)) == 2
    assert D.encoded_size(D.TimestampDeterminant(0)) == 9
    assert D.encoded_size(D.RNGDeterminant(0)) == 5
    assert D.encoded_size(D.BufferBuiltDeterminant(0)) == 5
    assert D.encoded_size(D.IgnoreCheckpointDeterminant(0, 0)) == 13
    assert D.encoded_size(D.TimerTriggerDeterminant(0, 0, D.IDLE)) == 14
    assert D.encoded_size(D.TimerTriggerDeterminant(0, 0, D.INTERNAL, b"PTS")) == 21
    assert D.encoded_size(D.TimerTriggerDeterminant(0, 0, D.INTERNAL, b"87")) == 20
    assert D.encoded_size(D.SourceCheckpointDeterminant(0, 0, 0, D.CHECKPOINT, b"")) == 27
    assert D.encoded_size(D.SourceCheckpointDeterminant(0, 0, 0, D.CHECKPOINT, None)) == 23


def test_jser_spec_vectors():
    assert D.jser_boolean(True) == BOOLEAN_TRUE
    for stream, n in [(D.jser_string("abc"), 10), (BOOLEAN_TRUE, 47), (D.jser_integer(1), 81), (D.jser_null(), 5)]:
        assert len(stream) == n
        assert O.jser_len(stream + b"\x07\x00\x00\x00\x01") == n  # trailing record must not be consumed
        assert pyref.jser_len(stream + b"\x00\x01") == n
    assert O.jser_len(b"\xac\xed\x00\x04\x70") < 0
    assert O.jser_len(BOOLEAN_TRUE[:-1]) < 0  # truncated stream


def test_queuetest_order_channels():
    # QueueTest.java:60-72 replays channels 1,2,2 through LogReplayer.replayNextChannel
    log = b"".join(D.encode(D.OrderDeterminant(c)) for c in (1, 2, 2))
    st, r, _, _ = O.decode(log)
    assert st == 0 and r["tag"].tolist() == [0, 0, 0] and r["v0"].tolist() == [1, 2, 2]


def test_nettytests_composite_semantics():
    # NettyTests.CompositeFromCompositeComponentsTest :144-186: 5 components of 11 bytes
    log = O.OracleLog(11)
    for _ in range(5):
        assert log.append(0, b"Hello world") == 0
    assert log.state()["capacity"] == 55
    st, b = log.read_phys(16, 41 - 16)
    assert st == 0 and b == b" worldHello worldHello wo"
    # readerIndex(12); discardReadComponents(); capacity == 44  (via a checkpoint whose
    # epoch starts at physical offset 12)
    log2 = O.OracleLog(11)
    log2.append(0, b"Hello world" + b"H")
    log2.append(1, b"ello world" + b"Hello world" * 3)
    assert log2.state()["epochs"] == [(0, 0), (1, 12)]
    assert log2.checkpoint_complete(1) == 0
    s = log2.state()
    assert s["capacity"] == 44 and s["n_components"] == 4 and s["epochs"] == [(1, 1)] and s["writer"] == 44
    p = pyref.ThreadLog(11)
    p.append(0, b"Hello world" + b"H")
    p.append(1, b"ello world" + b"Hello world" * 3)
    p.checkpoint_complete(1)
    assert p.state() == s


def test_discard_all_case():
    # readerIndex == writerIndex == capacity: every component dropped, indexes reset
    log = O.OracleLog(16)
    log.append(0, bytes(range(32)))
    assert log.checkpoint_complete(1) == 0
    assert log.state() == dict(writer=0, capacity=0, n_components=0, epochs=[(1, 0)])
    log.append(1, b"\x00\x05")
    assert log.state()["capacity"] == 16


@pytest.mark.parametrize("seed", range(6))
def test_oracle_decode_matches_pyref(seed):
    rng = np.random.default_rng(seed)
    buf = synth.random_log(300, rng)
    st, r, _, _ = O.decode(buf)
    assert st == 0
    ref = pyref.decode_all(buf)
    assert len(ref) == len(r["tag"])
    assert r["off"].tolist() == [x["off"] for x in ref]
    assert r["tag"].tolist() == [x["tag"] for x in ref]
    assert r["v0"].tolist() == [x["v0"] for x in ref]
    wide = [(i, x) for i, x in enumerate(ref) if x["wide"]]
    assert r["w_idx"].tolist() == [i for i, _ in wide]
    assert r["w_rc"].tolist() == [x["rc"] for _, x in wide]
    assert r["w_v1"].tolist() == [x["v1"] for _, x in wide]
    assert r["w_var_off"].tolist() == [x["var_off"] for _, x in wide]
    assert r["w_var_len"].tolist() == [x["var_len"] for _, x in wide]
    assert r["w_sub"].tolist() == [x["sub"] for _, x in wide]


ERROR_CASES = [
    (b"\x08", -2, 0),                                   # unknown tag
    (b"\x00\x01\xff", -2, 2),                           # negative tag byte
    (b"\x01\x00\x00", -3, 0),                           # truncated timestamp
    (b"\x00\x01\x04" + b"\x00" * 12 + b"\x07", -4, 2),  # TimerTrigger ordinal 7
    (b"\x04" + b"\x00" * 12 + b"\x06" + b"\xff\xff\xff\xff", -5, 0),  # negative name length
    (b"\x05" + b"\x00" * 20 + b"\x02\x00", -4, 0),      # CheckpointType ordinal 2 (after reads)
    (b"\x05" + b"\x00" * 20 + b"\x02\x01\x00\x00", -3, 0),  # truncated ref length beats bad enum
    (b"\x03\xac\xed\x00\x05\x74\x00\x09ab", -6, 0),     # truncated java string
    (b"\x03\x00", -6, 0),                               # missing magic
]


@pytest.mark.parametrize("buf,status,off", ERROR_CASES)
def test_oracle_error_semantics(buf, status, off):
    st, r, eo, et = O.decode(buf)
    assert (st, eo) == (status, off)
    with pytest.raises(pyref.DecodeError) as ex:
        pyref.decode_all(buf)
    assert (ex.value.status, ex.value.off) == (status, off)


@pytest.mark.parametrize("seed", range(8))
def test_oracle_log_matches_pyref(seed):
    """Random ThreadCausalLog op sequences: C++ oracle == Python restatement."""
    rng = np.random.default_rng(100 + seed)
    comp = int(rng.choice([16, 32, 48]))
    a, b = O.OracleLog(comp), pyref.ThreadLog(comp)
    epoch = 0
    last_cp = 0  # JobCausalLogImpl's CAS (:231-238) only lets newer checkpoints through
    chans = [(1, 1), (2, 2), (3, 3)]
    for step in range(400):
        op = rng.integers(0, 11)
        if op == 10:
            # upstream delta: dedup overlap, extension, or a gap (components are added
            # before the reader index throws, ThreadCausalLogImpl.java:136-143)
            rec = b"".join(D.encode(synth.random_determinant(rng, allow_serializable=False))
                           for _ in range(int(rng.integers(1, 4))))
            cur = dict(a.state()["epochs"])
            have = a.get_determinants(epoch)[1] if epoch in cur else b""
            off = len(have) - int(rng.integers(0, min(len(have), 6) + 1)) + int(rng.integers(-1, 2)) * 3
            off = max(off, 0)
            st = a.upstream(rec, off, epoch)
            try:
                b.upstream(rec, off, epoch)
                st2 = 0
            except pyref.LogError as ex:
                st2 = ex.status
            assert st == st2
        elif op <= 4:
            rec = D.encode(synth.random_determinant(rng, allow_serializable=False))
            assert a.append(epoch, rec) == 0
            b.append(epoch, rec)
        elif op == 5:
            ch = chans[int(rng.integers(0, 3))]
            e = epoch - int(rng.integers(0, 2))
            st, v = a.has_delta(ch, e)
            try:
                v2, st2 = b.has_delta(ch, e), 0
            except pyref.LogError as ex:
                v2, st2 = False, ex.status
            assert (st, v) == (st2, v2)
            if st == 0 and v:
                assert a.offset(ch) == (0, b.offset(ch))
                st, d = a.get_delta(ch, e)
                try:
                    d2, st2 = b.get_delta(ch, e), 0
                except pyref.LogError as ex:
                    d2, st2 = b"", ex.status
                assert (st, d) == (st2, d2)
        elif op == 6:
            epoch += 1
        elif op == 7 and epoch - 1 > last_cp:
            cp = epoch - int(rng.integers(0, 2))
            last_cp = cp
            st = a.checkpoint_complete(cp)
            try:
                b.checkpoint_complete(cp)
                st2 = 0
            except pyref.LogError as ex:
                st2 = ex.status
            assert st == st2
        elif op == 8:
            e = epoch - int(rng.integers(0, 3))
            st, d = a.get_determinants(e)
            try:
                d2, st2 = b.get_determinants(e), 0
            except pyref.LogError as ex:
                d2, st2 = b"", ex.status
            assert (st, d) == (st2, d2)
        else:
            assert a.log_length() == b.log_length()
        assert a.state() == b.state()


@pytest.mark.parametrize("seed", range(3))
def test_oracle_encode_matches_pyref(seed):
    """orc_encode (C++) == pyref.encode_one (Python) on random records of every tag, and
    both invert the decoder (encode(decode(x)) == x)."""
    rng = np.random.default_rng(500 + seed)
    buf = synth.random_log(3000, rng)
    st, r, _, _ = O.decode(buf)
    assert st == 0
    soa = (r["tag"], r["v0"], r["w_idx"], r["w_rc"], r["w_v1"], r["w_var_off"], r["w_var_len"], r["w_sub"], buf)
    assert O.encode_soa(*soa) == buf
    py = b"".join(pyref.encode_one(d["tag"], d["v0"], d["rc"], d["v1"], d["sub"],
                                   buf[d["var_off"]:d["var_off"] + d["var_len"]]) for d in pyref.decode_all(buf))
    assert py == buf
