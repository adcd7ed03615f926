"""pyref.py -- second, independent CPU restatement (TEST INFRASTRUCTURE ONLY).

Pure-Python loops, small cases only.  Used by tests to cross-check the C++ oracle
(oracle/clonos_oracle.cpp) and to regenerate tests/golden fixtures.  Never imported by
clonos_amd.

Restates (R/ = /root/reference/flink-runtime/src/main/java/org/apache/flink/runtime/causal/):
  R/determinant/SimpleDeterminantEncoder.java:78-342   decodeNext
  R/log/thread/ThreadCausalLogImpl.java:51-527          log state machine
  Netty 4.1.24 CompositeByteBuf.discardReadComponents   (pinned by NettyTests.java:144-186)
  Java Object Serialization spec section 6.4 grammar    (parity unpinned)
"""
from __future__ import annotations

import struct
import sys
from typing import Dict, List, Optional, Tuple

OK, E_CORRUPT_TAG, E_TRUNCATED, E_BAD_ENUM, E_NEG_LEN, E_BAD_SERIAL = 0, -2, -3, -4, -5, -6
E_CONSUMER_BACKWARDS, E_NO_CONSUMER, E_GAP, E_STATE = -7, -8, -9, -12


class DecodeError(Exception):
    def __init__(self, status, off, tag):
        super().__init__(f"decode error {status} at {off} tag {tag}")
        self.status, self.off, self.tag = status, off, tag


# --------------------------------------------------------------------------------------
# Java serialization stream length (recursive descent; independent of the C++ walker)
# --------------------------------------------------------------------------------------
MAX_DEPTH = 512  # open obj() calls: the JVM's StackOverflowError, which the reference does not catch


def _mutf(b):
    """Modified UTF-8 as JDK 8's ObjectInputStream reads it (readUTFBody / readUTFSpan): units
    0xxxxxxx, 110xxxxx 10xxxxxx, 1110xxxx 10xxxxxx 10xxxxxx, none cut by the length; else
    UTFDataFormatException."""
    i, n = 0, len(b)
    while i < n:
        b1 = b[i]
        if b1 < 0x80:
            i += 1
            continue
        k = 2 if b1 >> 5 == 6 else 3 if b1 >> 4 == 14 else 0
        if not k or n - i < k or any(b[i + j] & 0xC0 != 0x80 for j in range(1, k)):
            raise ValueError("utf")
        i += k
    return b
MAX_CHAIN = 256  # classes in one object's hierarchy (longer: a cyclic superclass chain)


class _J:
    def __init__(self, b: bytes):
        self.b, self.p = b, 0
        self.handles: List[object] = []
        self.depth = 0

    def take(self, n):
        if self.p + n > len(self.b):
            raise ValueError("eof")
        v = self.b[self.p:self.p + n]
        self.p += n
        return v

    def u8(self):
        return self.take(1)[0]

    def peek(self):
        if self.p >= len(self.b):
            raise ValueError("eof")
        return self.b[self.p]

    def u16(self):
        return struct.unpack(">H", self.take(2))[0]

    def s32(self):
        return struct.unpack(">i", self.take(4))[0]

    def utf(self):  # readUTF: modified UTF-8 (JDK 8 BlockDataInputStream.readUTFBody)
        return _mutf(self.take(self.u16()))

    def class_desc(self):
        tc = self.u8()
        if tc == 0x70:
            return None
        if tc == 0x71:
            h = self.s32() - 0x7E0000
            d = self.handles[h] if 0 <= h < len(self.handles) else None
            if not isinstance(d, dict):
                raise ValueError("bad desc ref")
            return d
        if tc == 0x72:
            name = self.utf()
            self.take(8)
            # the handle is assigned before classDescInfo, but the descriptor is usable only
            # once complete (JDK 8 initialises ObjectStreamClass at the end of readNonProxyDesc)
            slot = {"name": b"", "flags": 0, "fields": [], "super": None}
            self.handles.append(slot)
            d = {"name": name, "flags": 0, "fields": [], "super": None}
            d["flags"] = self.u8()
            for _ in range(self.u16()):
                t = chr(self.u8())
                self.utf()
                if t in "L[":
                    if self.peek() not in (0x74, 0x7C, 0x71):
                        raise ValueError("className1")
                    self.obj()
                elif t not in "BCDFIJSZ":
                    raise ValueError("typecode")
                d["fields"].append(t)
            self.annotation()
            d["super"] = self.class_desc()
            slot.update(d)
            return slot
        if tc == 0x7D:
            slot = {"name": b"", "flags": 0, "fields": [], "super": None}
            self.handles.append(slot)
            d = {"name": b"<proxy>", "flags": 2, "fields": [], "super": None}
            n = self.s32()
            if n < 0:
                raise ValueError("proxy")
            for _ in range(n):
                self.utf()
            self.annotation()
            d["super"] = self.class_desc()
            slot.update(d)
            return slot
        raise ValueError("classDesc tc")

    def annotation(self):
        while True:
            tc = self.peek()
            if tc == 0x78:
                self.p += 1
                return
            if tc == 0x77:
                self.p += 1
                self.take(self.u8())
            elif tc == 0x7A:
                self.p += 1
                n = self.s32()
                if n < 0:
                    raise ValueError("blockdatalong")
                self.take(n)
            else:
                self.obj()

    def values(self, d):
        sizes = {"B": 1, "Z": 1, "C": 2, "S": 2, "I": 4, "F": 4, "J": 8, "D": 8}
        for t in d["fields"]:
            if t in sizes:
                self.take(sizes[t])
            else:
                self.obj()

    def obj(self):
        self.depth += 1
        try:
            if self.depth > MAX_DEPTH:
                raise ValueError("depth")
            self._obj()
        finally:
            self.depth -= 1

    def _obj(self):
        tc = self.u8()
        while tc == 0x79:
            self.handles = []
            tc = self.u8()
        if tc == 0x70:
            return
        if tc == 0x71:
            h = self.s32() - 0x7E0000
            if not 0 <= h < len(self.handles):
                raise ValueError("ref")
            return
        if tc == 0x74:
            self.handles.append("s")
            self.utf()
            return
        if tc == 0x7C:
            self.handles.append("s")
            _mutf(self.take(struct.unpack(">Q", self.take(8))[0]))  # readLongUTF
            return
        if tc in (0x72, 0x7D):
            self.p -= 1
            self.class_desc()
            return
        if tc == 0x76:
            self.class_desc()
            self.handles.append("c")
            return
        if tc == 0x7E:
            self.class_desc()
            self.handles.append("e")
            if self.peek() not in (0x74, 0x7C, 0x71):
                raise ValueError("enum name")
            self.obj()
            return
        if tc == 0x75:
            d = self.class_desc()
            if d is None:
                raise ValueError("array desc")
            self.handles.append("a")
            n = self.s32()
            if n < 0:
                raise ValueError("array size")
            name = d["name"]
            es = {"B": 1, "Z": 1, "C": 2, "S": 2, "I": 4, "F": 4, "J": 8, "D": 8}.get(chr(name[1]) if len(name) > 1 else "")
            if len(name) < 2 or name[0:1] != b"[":
                raise ValueError("array name")
            if es:
                self.take(es * n)
            elif chr(name[1]) in "L[":
                for _ in range(n):
                    self.obj()
            else:
                raise ValueError("array comp")
            return
        if tc == 0x73:
            d = self.class_desc()
            if d is None:
                raise ValueError("object desc")
            self.handles.append("o")
            chain = []
            c = d
            while c is not None:
                chain.append(c)
                if len(chain) > MAX_CHAIN:
                    raise ValueError("hierarchy")
                c = c["super"]
            if d["flags"] & 0x04:
                if not d["flags"] & 0x08:
                    raise ValueError("externalizable v1")
                self.annotation()
                return
            for c in reversed(chain):
                if not c["flags"] & 0x02:
                    raise ValueError("not serializable")
                self.values(c)
                if c["flags"] & 0x01:
                    self.annotation()
            return
        raise ValueError("object tc")


def jser_len(b: bytes) -> Optional[int]:
    if len(b) < 4 or b[:4] != b"\xac\xed\x00\x05":
        return None
    j = _J(b)
    j.p = 4
    lim = sys.getrecursionlimit()
    sys.setrecursionlimit(max(lim, 8 * MAX_DEPTH + 1000))  # a few Python frames per obj()
    try:
        j.obj()
    except (ValueError, IndexError, struct.error):
        return None
    finally:
        sys.setrecursionlimit(lim)
    return j.p


# --------------------------------------------------------------------------------------
# decodeNext loop
# --------------------------------------------------------------------------------------
def decode_one(b: bytes, pos: int):
    """Returns (record dict, next pos) or raises DecodeError."""
    avail = len(b) - pos
    tag = struct.unpack_from(">b", b, pos)[0]

    def trunc():
        raise DecodeError(E_TRUNCATED, pos, tag)

    rec = dict(off=pos, tag=tag & 0xFF, wide=False, rc=0, v1=0, var_off=0, var_len=0, sub=0)
    if tag == 0:
        if avail < 2:
            trunc()
        rec["v0"] = struct.unpack_from(">b", b, pos + 1)[0]
        return rec, pos + 2
    if tag == 1:
        if avail < 9:
            trunc()
        rec["v0"] = struct.unpack_from(">q", b, pos + 1)[0]
        return rec, pos + 9
    if tag in (2, 7):
        if avail < 5:
            trunc()
        rec["v0"] = struct.unpack_from(">i", b, pos + 1)[0]
        return rec, pos + 5
    if tag == 6:
        if avail < 13:
            trunc()
        rec.update(wide=True, rc=struct.unpack_from(">i", b, pos + 1)[0], v0=struct.unpack_from(">q", b, pos + 5)[0])
        return rec, pos + 13
    if tag == 4:
        if avail < 14:
            trunc()
        rc, ts, ordv = struct.unpack_from(">iqb", b, pos + 1)
        if not 0 <= ordv <= 6:
            raise DecodeError(E_BAD_ENUM, pos, tag)
        rec.update(wide=True, rc=rc, v0=ts, sub=ordv)
        if ordv == 6:
            if avail < 18:
                trunc()
            nl = struct.unpack_from(">i", b, pos + 14)[0]
            if nl < 0:
                raise DecodeError(E_NEG_LEN, pos, tag)
            if avail < 18 + nl:
                trunc()
            rec.update(var_off=pos + 18, var_len=nl)
            return rec, pos + 18 + nl
        return rec, pos + 14
    if tag == 5:
        if avail < 23:
            trunc()
        rc, cp, ts, ordv, has = struct.unpack_from(">iqqbB", b, pos + 1)
        end = pos + 23
        rec.update(wide=True, rc=rc, v0=cp, v1=ts)
        if has != 0:
            if avail < 27:
                trunc()
            rl = struct.unpack_from(">i", b, pos + 23)[0]
            if rl < 0:
                raise DecodeError(E_NEG_LEN, pos, tag)
            if avail < 27 + rl:
                trunc()
            rec.update(var_off=pos + 27, var_len=rl)
            end = pos + 27 + rl
        if not 0 <= ordv <= 1:
            raise DecodeError(E_BAD_ENUM, pos, tag)
        rec["sub"] = ordv | (0x80 if has else 0)
        return rec, end
    if tag == 3:
        n = jser_len(b[pos + 1:])
        if n is None:
            raise DecodeError(E_BAD_SERIAL, pos, tag)
        rec.update(wide=True, v0=n, var_off=pos + 1, var_len=n)
        return rec, pos + 1 + n
    raise DecodeError(E_CORRUPT_TAG, pos, tag)


def encode_one(tag: int, v0: int, rc: int = 0, v1: int = 0, sub: int = 0, var: bytes = b"") -> bytes:
    """SimpleDeterminantEncoder.encodeTo (:56-75) with the per-type writers: Order :124-127,
    Timestamp :145-148, RNG :167-170, BufferBuilt :189-192, TimerTrigger :202-213,
    SourceCheckpoint :244-257, IgnoreCheckpoint :289-293, Serializable :316-323 (the
    stream bytes are given).  Fields are in the decode's record layout (decode_one)."""
    w = lambda fmt, *a: struct.pack(">" + fmt, *a)  # noqa: E731  (Netty ByteBuf: big-endian)
    m32 = lambda x: ((x + (1 << 31)) % (1 << 32)) - (1 << 31)  # noqa: E731  (int cast)
    m64 = lambda x: ((x + (1 << 63)) % (1 << 64)) - (1 << 63)  # noqa: E731  (long cast)
    if tag == 0:
        return w("bb", 0, ((v0 + 128) % 256) - 128)
    if tag == 1:
        return w("bq", 1, m64(v0))
    if tag in (2, 7):
        return w("bi", tag, m32(v0))
    if tag == 6:
        return w("biq", 6, m32(rc), m64(v0))
    if tag == 4:
        head = w("biqb", 4, m32(rc), m64(v0), sub)
        return head + (w("i", len(var)) + var if sub == 6 else b"")
    if tag == 5:
        has = 1 if sub & 0x80 else 0
        head = w("biqqbB", 5, m32(rc), m64(v0), m64(v1), sub & 0x7F, has)
        return head + (w("i", len(var)) + var if has else b"")
    if tag == 3:
        return b"\x03" + bytes(var)
    raise ValueError(f"unknown tag {tag}")


def decode_all(b: bytes) -> List[dict]:
    out, pos = [], 0
    while pos < len(b):
        r, pos = decode_one(b, pos)
        out.append(r)
    return out


# --------------------------------------------------------------------------------------
# ThreadCausalLogImpl over a Netty CompositeByteBuf of fixed-size components
# --------------------------------------------------------------------------------------
class _Epoch:
    __slots__ = ("id", "offset")

    def __init__(self, i, o):
        self.id, self.offset = i, o


class LogError(Exception):
    def __init__(self, status):
        super().__init__(status)
        self.status = status


class ThreadLog:
    def __init__(self, component: int, depth: int = -1):
        self.C, self.depth = component, depth
        self.comps: List[bytearray] = [bytearray(component)]
        self.writer = 0
        self.epochs: Dict[int, _Epoch] = {}
        self.consumers: Dict[object, list] = {}  # ch -> [epoch object, offset]

    @property
    def capacity(self):
        return len(self.comps) * self.C

    def _ensure(self, n):
        while self.capacity - self.writer < n:
            self.comps.append(bytearray(self.C))

    def _write(self, data: bytes):
        for i, x in enumerate(data):
            p = self.writer + i
            self.comps[p // self.C][p % self.C] = x
        self.writer += len(data)

    def _read(self, phys, n) -> bytes:
        return bytes(self.comps[(phys + i) // self.C][(phys + i) % self.C] for i in range(n))

    def _cia(self, e):
        if e not in self.epochs:
            self.epochs[e] = _Epoch(e, self.writer)
        return self.epochs[e]

    def _send(self, epoch, phys):
        nxt = self.epochs.get(epoch + 1)
        return (nxt.offset if nxt is not None else self.writer) - phys

    def append(self, epoch, data: bytes):
        if self.depth == 0:
            return
        self._cia(epoch)
        self._ensure(len(data))
        self._write(data)

    def upstream(self, delta: bytes, off_from_epoch: int, epoch: int):
        n = len(delta)
        if n == 0:
            return
        es = self._cia(epoch)
        cur = self.writer - es.offset
        num_new = off_from_epoch + n - cur
        if num_new > 0:
            self._ensure(num_new)  # :136-137: components are added before readerIndex throws
            if num_new > n:
                raise LogError(E_GAP)
            self._write(delta[n - num_new:])

    def has_delta(self, ch, epoch) -> bool:
        if self.depth == 0:
            return False
        es = self.epochs.get(epoch)
        if es is None:
            return False
        c = self.consumers.setdefault(ch, [es, 0])
        if c[0].id != epoch:
            if c[0].id > epoch:
                raise LogError(E_CONSUMER_BACKWARDS)
            c[0], c[1] = es, 0
        return self._send(epoch, c[0].offset + c[1]) != 0

    def offset(self, ch) -> int:
        if ch not in self.consumers:
            raise LogError(E_NO_CONSUMER)
        return self.consumers[ch][1]

    def get_delta(self, ch, epoch) -> bytes:
        if ch not in self.consumers:
            raise LogError(E_NO_CONSUMER)
        c = self.consumers[ch]
        phys = c[0].offset + c[1]
        n = self._send(epoch, phys)
        if n < 0 or phys < 0 or phys + n > self.capacity:
            raise LogError(E_STATE)
        out = self._read(phys, n)
        c[1] += n
        return out

    def get_determinants(self, start_epoch) -> bytes:
        if self.depth == 0:
            return b""
        if start_epoch in self.epochs:
            s = self.epochs[start_epoch].offset
        elif self.epochs:
            s = self.epochs[min(self.epochs)].offset
        else:
            s = 0
        if s < 0 or self.writer - s < 0 or self.writer > self.capacity:
            raise LogError(E_STATE)
        return self._read(s, self.writer - s)

    def log_length(self) -> int:
        if not self.epochs:
            return self.writer
        return self.writer - self.epochs[min(self.epochs)].offset

    def checkpoint_complete(self, cp):
        following = self._cia(cp)
        for e in [e for e in self.epochs if e < cp]:
            del self.epochs[e]
        R = following.offset
        if R < 0 or R > self.writer:
            raise LogError(E_STATE)
        move = 0
        if R != 0:
            if R == self.writer == self.capacity:
                move = R
                self.comps = []
            else:
                k = R // self.C
                self.comps = self.comps[k:]
                move = k * self.C
        for e in self.epochs.values():
            e.offset -= move
        self.writer -= move

    def state(self):
        return dict(writer=self.writer, capacity=self.capacity, n_components=len(self.comps),
                    epochs=sorted((k, v.offset) for k, v in self.epochs.items()))
