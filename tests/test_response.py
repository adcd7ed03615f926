"""CPU: DeterminantResponseEvent wire format + merge (DeterminantResponseEvent.java:93-148).

The oracle (oracle/response_ref.py) is pinned by hand-derived known answers below: Java
int arithmetic of CausalLogID.hashCode, DataOutputView byte layouts, and java.util.HashMap
iteration order (JDK 8).  No reference test covers this event, so these KATs are derived
from the reference's source, not from reference outputs.  The product functions
(clg_response_*) are host logic in libclonos_engine.so and are checked against the oracle
on seeded random event sequences.
"""
import os
import struct
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import response_ref as R  # noqa: E402  (checker)

from clonos_amd import CausalLogID  # noqa: E402
from clonos_amd import _lib  # noqa: E402
from clonos_amd.replay import DeterminantResponseEvent, accumulate, causal_log_id_hash  # noqa: E402


# ---------------------------------------------------------------- oracle KATs
def test_hash_kat():
    # 17*31 + 5 = 532; 532*31 + 1 = 16493  (CausalLogID.java:151-156)
    assert R.LogId.main(5).java_hash() == 16493
    # subpartition: continue with lower/upper folded to ints and the index
    h = 31 * (31 * 17 + 7) + 0
    h = 31 * h + (0x00000001 ^ 0x00000002)          # lower = 0x00000002_00000001
    h = 31 * h + 0                                    # upper = 0
    h = 31 * h + 3
    assert R.LogId.subpartition(7, 0x0000000200000001, 0, 3).java_hash() == h
    # Java int overflow wraps: vertex -1, huge upper
    x = R.LogId.subpartition(-1, -1, -(1 << 63), -128).java_hash()
    assert -(1 << 31) <= x < (1 << 31)


def test_wire_kat():
    r = R.Response(True, 3, 0x0102030405060708)
    r.dets.put(R.LogId.main(3), b"\x00\x01")
    want = bytes.fromhex("01" "0003" "0102030405060708" "01" "0003" "01" "00000002" "0001")
    assert r.write() == want
    s = R.Response(False, -2, -1)
    s.dets.put(R.LogId.subpartition(-2, 1, 2, 5), b"")
    want = bytes.fromhex("00" "fffe" "ffffffffffffffff" "01" "fffe" "00" "0000000000000001" "0000000000000002"
                         "05" "00000000")
    assert s.write() == want


def test_hashmap_order_kat():
    """Iteration order = bucket order, bins in insertion order, 16 -> 32 buckets at the 13th key."""
    m = R.JavaHashMap()
    ids = [R.LogId.main(v) for v in range(12)]
    for k in ids:
        m.put(k, b"")
    assert m.cap == 16
    # main(v) hash = 31*(31*17+v)+1 = 16338 + 31 v; spread is a no-op below 2^16
    order = sorted(range(12), key=lambda v: ((16338 + 31 * v) & 15, v))
    assert [k.vertex for k, _ in m.items()] == order
    m.put(R.LogId.main(12), b"")
    assert m.cap == 32
    order = sorted(range(13), key=lambda v: ((16338 + 31 * v) & 31, v))
    assert [k.vertex for k, _ in m.items()] == order


def test_merge_semantics_kat():
    a = R.Response(False, 1)
    b = R.Response(False, 1)
    b.dets.put(R.LogId.main(1), b"xx")
    a.merge(b)  # neither found: nothing happens (:130-131)
    assert a.dets.size == 0 and not a.found
    b.found = True
    a.merge(b)
    assert a.found and a.dets.get(R.LogId.main(1)) == b"xx"
    c = R.Response(True, 1)
    c.dets.put(R.LogId.main(1), b"yy")  # tie -> v2 (:140-145)
    a.merge(c)
    assert a.dets.get(R.LogId.main(1)) == b"yy"
    d = R.Response(True, 1)
    d.dets.put(R.LogId.main(1), b"z")  # shorter loses
    a.merge(d)
    assert a.dets.get(R.LogId.main(1)) == b"yy"


def test_count_byte_is_signed():
    r = R.Response(True, 9)
    for i in range(130):
        r.dets.put(R.LogId.subpartition(9, 1, 1, i - 128), b"\x07\x00\x00\x00\x01")
    w = r.write()
    assert w[11] == 130
    back, used = R.Response.read(w)
    assert back.dets.size == 0 and used == 12


# ---------------------------------------------------------------- product vs oracle
def _rand_id(rng, vertices):
    v = int(rng.choice(vertices))
    if rng.random() < 0.3:
        return R.LogId.main(v)
    return R.LogId.subpartition(v, int(rng.integers(-2**63, 2**63 - 1)) if rng.random() < 0.3 else 77,
                                int(rng.integers(0, 3)), int(rng.integers(-128, 128)))


def _to_cl(k: R.LogId) -> CausalLogID:
    return CausalLogID.main(k.vertex) if k.is_main else CausalLogID.sub(k.vertex, k.lower, k.upper, k.sub)


def _product_from(resp: R.Response) -> DeterminantResponseEvent:
    p = DeterminantResponseEvent(resp.found, resp.vertex, resp.corr)
    for k, v in resp.dets.items():  # iteration order == an insertion order giving the same map
        p.put(_to_cl(k), v)
    return p


@pytest.mark.parametrize("seed", range(6))
def test_put_write_read_match_oracle(seed):
    rng = np.random.default_rng(seed)
    vertices = rng.integers(-300, 300, size=8)
    o = R.Response(bool(rng.integers(0, 2)), int(rng.integers(-2**15, 2**15)), int(rng.integers(-2**63, 2**63 - 1)))
    p = DeterminantResponseEvent(o.found, o.vertex, o.corr, capacity=4)
    for _ in range(int(rng.integers(0, 120))):
        k = _rand_id(rng, vertices)
        v = rng.integers(0, 256, size=int(rng.integers(0, 40)), dtype=np.uint8).tobytes()
        o.dets.put(k, v)
        p.put(_to_cl(k), v)
    w = o.write()
    assert p.write() == w
    assert causal_log_id_hash(CausalLogID.main(5)) == 16493
    back, used = DeterminantResponseEvent.read(w)
    assert used == len(w)
    ob, _ = R.Response.read(w)
    assert back.write() == ob.write() == w
    assert list(back.getDeterminants().items()) == [(_to_cl(k), v) for k, v in ob.dets.items()]


@pytest.mark.parametrize("seed", range(6))
def test_merge_sequences_match_oracle(seed):
    rng = np.random.default_rng(100 + seed)
    vertices = rng.integers(0, 40, size=5)
    events = []
    for _ in range(int(rng.integers(1, 7))):
        e = R.Response(bool(rng.random() < 0.8), 3, int(rng.integers(0, 1000)))
        for _ in range(int(rng.integers(0, 25))):
            e.dets.put(_rand_id(rng, vertices), rng.integers(0, 256, size=int(rng.integers(0, 30)),
                                                               dtype=np.uint8).tobytes())
        events.append(e.write())
    want = R.accumulate(3, events)
    got = accumulate(3, [DeterminantResponseEvent.read(w)[0] for w in events])
    assert got.isFound() == want.found
    assert got.write() == want.write()


def test_collisions_trigger_small_table_resize():
    """9 ids in one bucket of a 16-bucket table: treeifyBin resizes instead (cap < 64)."""
    ids, seen = [], {}
    for s in range(-128, 128):
        for lo in range(0, 64):
            k = R.LogId.subpartition(1, lo, 0, s)
            h = k.java_hash() & 0xFFFFFFFF
            b = (h ^ (h >> 16)) & 15
            seen.setdefault(b, []).append(k)
    bucket = max(seen.values(), key=len)[:9]
    o = R.Response(True, 1)
    p = DeterminantResponseEvent(True, 1)
    for k in bucket:
        o.dets.put(k, b"\x07\x00\x00\x00\x05")
        p.put(_to_cl(k), b"\x07\x00\x00\x00\x05")
    assert o.dets.cap == 32
    assert p._c.table_cap == 32
    assert p.write() == o.write()


def test_read_errors():
    r = R.Response(True, 3)
    r.dets.put(R.LogId.main(3), b"\x00\x01\x00\x02")
    w = r.write()
    for cut in (0, 5, 11, 13, 16, len(w) - 1):
        with pytest.raises(_lib.ClonosError) as ei:
            DeterminantResponseEvent.read(w[:cut])
        assert ei.value.status == _lib.CLG_E_TRUNCATED
    bad = bytearray(w)
    bad[15:19] = struct.pack(">i", -1)
    with pytest.raises(_lib.ClonosError) as ei:
        DeterminantResponseEvent.read(bytes(bad))
    assert ei.value.status == _lib.CLG_E_NEG_LEN


def test_buffer_sizes_oracle():
    ok = b"".join(b"\x07" + struct.pack(">i", n) for n in (1, 32768, -5))
    assert R.buffer_sizes(ok) == [1, 32768, -5]
    with pytest.raises(ValueError) as ei:
        R.buffer_sizes(ok + b"\x00\x01" + ok)
    assert ei.value.args[0] == (R.E_NOT_BUFFER_BUILT, 15, 0)


@pytest.mark.parametrize("seed", range(8))
def test_put_batch_matches_oracle(seed):
    """clg_response_put_batch (one sort instead of a scan per put) against the oracle's puts one
    by one: pre-existing entries, keys put twice inside a batch, batches that cross the resize
    thresholds and a bucket of 9 colliding ids (the small-table treeify resize) -- the same
    wire bytes, hence the same iteration order, and the same table capacity."""
    from clonos_amd.replay import log_id_array
    rng = np.random.default_rng(500 + seed)
    vertices = rng.integers(-50, 50, size=6)
    keys = [_rand_id(rng, vertices) for _ in range(int(rng.integers(20, 200)))]
    if seed % 2:  # a bucket of colliding ids as well (test_collisions_trigger_small_table_resize)
        seen = {}
        for s in range(-128, 128):
            for lo in range(0, 64):
                k = R.LogId.subpartition(1, lo, 0, s)
                h = k.java_hash() & 0xFFFFFFFF
                seen.setdefault((h ^ (h >> 16)) & 15, []).append(k)
        keys += max(seen.values(), key=len)[:9]
    keys += [keys[int(i)] for i in rng.integers(0, len(keys), 10)]  # puts of keys already there
    vals = [rng.integers(0, 256, size=int(rng.integers(0, 30)), dtype=np.uint8).tobytes() for _ in keys]
    o = R.Response(True, 7, 1)
    p = DeterminantResponseEvent(True, 7, 1, capacity=len(keys) + 1)
    pre = int(rng.integers(0, len(keys) // 2))
    for k, v in zip(keys[:pre], vals[:pre]):  # some entries there already
        o.dets.put(k, v)
        p.put(_to_cl(k), v)
    for k, v in zip(keys[pre:], vals[pre:]):
        o.dets.put(k, v)
    bufs = [np.frombuffer(v, np.uint8) if v else np.zeros(1, np.uint8) for v in vals[pre:]]
    at = pre
    while at < len(keys):  # the rest in batches of 8 .. 60 puts
        m = min(len(keys) - at, int(rng.integers(8, 61)))
        ids = log_id_array([_to_cl(k) for k in keys[at:at + m]])
        ptrs = np.array([b.ctypes.data for b in bufs[at - pre:at - pre + m]], np.uint64)
        lens = np.array([len(v) for v in vals[at:at + m]], np.uint64)
        p.put_device_batch(ids, ptrs, lens, bufs)
        at += m
    assert p.write() == o.write()
    assert p._c.table_cap == o.dets.cap
