"""CPU: the Serializable record length pinned on JDK-written streams.

tests/golden/jser_reference.json holds the 199 distinct Java serialization streams the
reference's test resources carry behind a TypeSerializerSerializationUtil length prefix
(made by tests/golden/make_jser_reference.py).  Each prefix states where one stream ends,
independently of any walker here, so it pins:
  * the C++ oracle (oracle/clonos_oracle.cpp JWalker) and pyref (oracle/pyref.py);
  * the device walker itself (clonos_amd/csrc/jser_device.h), compiled for the host from
    the very source the kernels instantiate (tests/jser_walker_host.cpp), with and
    without its spill arena.
Beyond the fixture, seeded mutations of those streams and synthetic shapes (deep nesting,
long or cyclic class hierarchies, many handles) hold the three walkers to one another.
The GPU side of the same fixture is tests/test_gpu_jser.py.
"""
import ctypes as C
import json
import os
import random
import struct
import subprocess

import pytest

import _oracle as O
from _oracle import pyref

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
FIX = json.load(open(os.path.join(ROOT, "tests", "golden", "jser_reference.json")))
STREAMS = [bytes.fromhex(x["hex"]) for x in FIX]


@pytest.fixture(scope="module")
def walker(tmp_path_factory):
    so = str(tmp_path_factory.mktemp("jwalk") / "libjwalk.so")
    hipcc = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
    subprocess.run([hipcc, "-x", "hip", "--offload-host-only", "-O2", "-std=c++17", "-fPIC", "-shared",
                    "-I", os.path.join(ROOT, "include"), "-o", so, os.path.join(ROOT, "tests", "jser_walker_host.cpp")],
                   check=True)
    lib = C.CDLL(so)
    lib.walker_stream_len.restype = C.c_int64
    lib.walker_stream_len.argtypes = [C.c_char_p, C.c_uint64, C.c_uint64, C.POINTER(C.c_uint64)]
    lib.flat_record_len.restype = C.c_uint32
    lib.flat_record_len.argtypes = [C.c_char_p, C.c_uint32]

    def run(b: bytes, arena: int = 1 << 22):
        used = C.c_uint64()
        r = lib.walker_stream_len(b, len(b), arena, C.byref(used))
        return r, used.value
    run.flat = lambda rec: lib.flat_record_len(rec, len(rec))
    lib.walker_backward_reads.restype = C.c_uint64
    run.backward_reads = lib.walker_backward_reads
    return run


def test_fixture_shape():
    assert len(FIX) == 199
    assert all(x["len"] == len(bytes.fromhex(x["hex"])) for x in FIX)
    assert len(set(x["hex"] for x in FIX)) == len(FIX)


@pytest.mark.parametrize("i", range(len(FIX)), ids=[f"{i}:{os.path.basename(x['src'])}" for i, x in enumerate(FIX)])
def test_reference_stream_lengths(i, walker):
    s, n = STREAMS[i], FIX[i]["len"]
    tail = bytes([0x70, 0x00, 0x78, 0xAC, 0xED])  # the stream ends where the prefix says, whatever follows
    assert O.jser_len(s) == n
    assert O.jser_len(s + tail) == n
    assert pyref.jser_len(s + tail) == n
    assert walker(s + tail)[0] == n
    # one byte short is not a stream
    assert O.jser_len(s[:-1]) < 0 and pyref.jser_len(s[:-1]) is None and walker(s[:-1])[0] == -1


def test_reference_streams_need_the_spill_tier(walker):
    """23 of the streams outgrow the private tier (> 16 class descriptors or > 64
    handles): without arena space they report kJsSpill (-2, the engine grows the arena),
    never "invalid"; with it they measure exactly."""
    spilled = 0
    for s, x in zip(STREAMS, FIX):
        r0, _ = walker(s, 0)
        r, used = walker(s)
        assert r == x["len"]
        assert r0 in (x["len"], -2)
        if r0 == -2:
            spilled += 1
            assert used > 0
    assert spilled == 23


def _agree(walker, b: bytes):
    o = O.jser_len(b)
    p = pyref.jser_len(b)
    w, _ = walker(b)
    o = o if o >= 0 else -1
    p = p if p is not None else -1
    assert o == p == w, (b.hex(), o, p, w)
    return o


def test_mutations_agree(walker):
    """Seeded byte flips, truncations, insertions and splices of the reference streams:
    oracle, pyref and the device walker give the same length or all reject."""
    rng = random.Random(0xC105_0A5)
    n_valid = 0
    for k in range(3000):
        s = bytearray(rng.choice(STREAMS))
        op = k % 4
        if op == 0:
            for _ in range(rng.randint(1, 3)):
                s[rng.randrange(4, len(s))] = rng.randrange(256)
        elif op == 1:
            s = s[:rng.randrange(4, len(s) + 1)]
        elif op == 2:
            q = rng.randrange(4, len(s))
            s[q:q] = bytes([rng.choice([0x70, 0x71, 0x73, 0x74, 0x75, 0x77, 0x78, 0x79, 0x7E, rng.randrange(256)])])
        else:
            t = rng.choice(STREAMS)
            q = rng.randrange(4, len(s))
            s = s[:q] + t[rng.randrange(4, len(t)):]
        n_valid += _agree(walker, bytes(s)) > 0
    assert n_valid > 100  # the mix keeps some streams valid (tails after the object end)


MAGIC = b"\xac\xed\x00\x05"


def _utf(s: bytes) -> bytes:
    return struct.pack(">H", len(s)) + s


def _objarr_nest(depth: int) -> bytes:
    """depth nested Object[1] arrays (the innermost holds null): depth + 1 object() levels."""
    desc = b"\x72" + _utf(b"[Ljava.lang.Object;") + b"\x90\xceX\x9f\x10s)l" + b"\x02\x00\x00\x78\x70"
    out = b"\x75" + desc + struct.pack(">i", 1)
    for _ in range(depth - 1):
        out += b"\x75\x71" + struct.pack(">i", 0x7E0000) + struct.pack(">i", 1)
    return MAGIC + out + b"\x70"


def test_nesting_depth_limit(walker):
    for d in (1, 100, 510, 511, 512, 513, 600):
        n = _agree(walker, _objarr_nest(d))
        assert (n > 0) == (d + 1 <= 512), d


def _chain(n_classes: int, cyclic: bool = False) -> bytes:
    """TC_OBJECT of a class with n_classes - 1 serializable superclasses (one int field each)."""
    out = MAGIC + b"\x73"
    for i in range(n_classes):
        out += b"\x72" + _utf(b"C%d" % i) + bytes(8) + b"\x02" + b"\x00\x01" + b"I" + _utf(b"v") + b"\x78"
    if cyclic:
        out += b"\x71" + struct.pack(">i", 0x7E0000)  # the last class's super: the first class
    else:
        out += b"\x70"
    return out + bytes(4 * n_classes)


def test_class_hierarchy_limit_and_cycles(walker):
    for k in (1, 16, 17, 100, 256):
        assert _agree(walker, _chain(k)) == len(_chain(k))
    assert _agree(walker, _chain(257)) == -1
    assert _agree(walker, _chain(3, cyclic=True)) == -1


def test_many_handles_and_descriptors(walker):
    """An Object[] of 5000 distinct strings and 300 distinct classes: far past the private
    tier (64 handles, 16 descriptors)."""
    body = b""
    for i in range(300):
        body += b"\x73\x72" + _utf(b"K%d" % i) + bytes(8) + b"\x02\x00\x01J" + _utf(b"x") + b"\x78\x70" + bytes(8)
    for i in range(5000):
        body += b"\x74" + _utf(b"s%d" % i)
    desc = b"\x72" + _utf(b"[Ljava.lang.Object;") + bytes(8) + b"\x02\x00\x00\x78\x70"
    s = MAGIC + b"\x75" + desc + struct.pack(">i", 5300) + body
    assert _agree(walker, s) == len(s)
    r0, _ = walker(s, 0)
    assert r0 == -2
    r1, used = walker(s, 1 << 12)  # too small an arena: spill, not invalid
    assert r1 == -2
    r2, used = walker(s, 1 << 20)
    assert r2 == len(s) and used > 4 * 5300


def test_flat_parser_agrees_with_the_oracle(walker):
    """The inline flat-object parser (jser_flat.h) that both the decode and the write path's
    sidecar trust for lengths: on every reference stream, the flat shapes the synthetic
    configs write, and seeded mutations, a length it gives is the oracle's record length
    (1 + the stream's), and a stream it cannot finish inside the bytes gives 0 (the walker
    decides)."""
    from clonos_amd import determinants as D
    rng = random.Random(0xF1A7)
    shapes = [D.jser_boolean(True), D.jser_boolean(False), D.jser_integer(-7), D.jser_integer(2 ** 31 - 1),
              D.jser_long(-(2 ** 62)), D.jser_long(12345)]
    base = list(STREAMS) + shapes
    streams = list(base)
    for k in range(3000):
        s = bytearray(rng.choice(base))
        op = k % 3
        if op == 0:
            s[rng.randrange(4, len(s))] = rng.randrange(256)
        elif op == 1:
            s = s[:rng.randrange(4, len(s) + 1)]
        streams.append(bytes(s))
    n_flat = 0
    for s in streams:
        rec = b"\x03" + s + bytes([0x70, 0x00, 0x78, 0xAC, 0xED])  # (a tail: the stream ends where it ends)
        L = walker.flat(rec)
        if L:
            n_flat += 1
            assert O.jser_len(rec[1:]) == L - 1, (s.hex(), L)
            assert walker.flat(rec[:L]) == L  # the bytes up to its end suffice
            assert walker.flat(rec[:L - 1]) == 0  # one short: not finished inside the bytes
    for s in shapes:
        assert walker.flat(b"\x03" + s) == 1 + len(s)
    assert n_flat > 100


def test_modified_utf8_as_jdk8_reads_it(walker):
    """readUTF / readLongUTF (JDK 8 BlockDataInputStream.readUTFBody): units 0xxxxxxx,
    110xxxxx 10xxxxxx, 1110xxxx 10xxxxxx 10xxxxxx, none cut by the length, else
    UTFDataFormatException -- in a TC_STRING, a TC_LONGSTRING, a class name and a field name.
    Oracle, pyref and the device walker agree; the inline flat parser gives no length for a
    malformed name (the walker decides)."""
    good = [b"abc", b"", b"\xc0\x80", b"\xc3\xa9t\xc3\xa9", b"\xe2\x82\xac", b"\x00\x7f", b"\xef\xbf\xbf"]
    bad = [b"\x80", b"a\xbf", b"\xc3", b"\xc3a", b"\xe2\x82", b"\xe2\x82a", b"\xe2a\xac", b"\xf0\x9f\x98\x80",
           b"\xff", b"ab\xf8", b"\xed\xa0"]
    for body, ok in [(x, True) for x in good] + [(x, False) for x in bad]:
        s1 = MAGIC + b"\x74" + _utf(body)                                    # TC_STRING
        s2 = MAGIC + b"\x7c" + struct.pack(">Q", len(body)) + body           # TC_LONGSTRING
        name = b"C" + body
        s3 = MAGIC + b"\x73\x72" + _utf(name) + bytes(8) + b"\x02\x00\x01I" + _utf(b"v") + b"\x78\x70" + bytes(4)
        s4 = MAGIC + b"\x73\x72" + _utf(b"K") + bytes(8) + b"\x02\x00\x01I" + _utf(b"f" + body) + b"\x78\x70" + bytes(4)
        for s in (s1, s2, s3, s4):
            n = _agree(walker, s)
            assert (n == len(s)) == ok, (body, s.hex(), n)
        for s in (s3, s4):
            L = walker.flat(b"\x03" + s)
            assert L == (1 + len(s) if ok else 0), (body, s.hex(), L)


def test_walker_reads_forwards_only(walker):
    """The device readers (ZStreamBytes, the robust pipeline's span reader) keep a cursor over
    the span's tiles that only moves forwards, so the walker must ask for offsets in
    non-decreasing order; a class name once was checked before its first two bytes were read
    back (an out-of-bounds read on the GPU).  Every stream this module walks, counted."""
    test_modified_utf8_as_jdk8_reads_it(walker)
    test_mutations_agree(walker)
    for s in STREAMS:
        walker(s)
    assert walker.backward_reads() == 0
