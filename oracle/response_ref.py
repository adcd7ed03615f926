"""response_ref.py -- CPU restatement of the replay-prep wire path (TEST INFRASTRUCTURE ONLY).

Checker for clg_response_* / clg_replay_prep_responses in libclonos_engine.so.  Pure
Python, small cases only; only tests/ and tests/golden/make_golden.py import it.

Restates (R/ = /root/reference/flink-runtime/src/main/java/org/apache/flink/runtime/causal/):
  R/log/job/CausalLogID.java:128-186            equals, hashCode, write, read
  R/DeterminantResponseEvent.java:93-148        write, read, merge (longest wins, ties -> v2)
  R/recovery/WaitingDeterminantsState.java:57,102  accumulator = (found=true, vertex), merge each
  R/recovery/ReplayingState.java:63-66,108-130  main log by CausalLogID(vertex); one recovery
                                                buffer per subpartition (EMPTY when absent)
  R/recovery/ReplayingState.java:157-181        subpartition buffers may hold BufferBuilt only
Third-party semantics restated (absent from /root/reference):
  JDK 8 java.util.HashMap iteration order for the map inside the event (table of 2^k
  buckets, default capacity 16, load factor 0.75, index = (h ^ (h >>> 16)) & (cap - 1),
  bins append at the tail and keep their order across resizes, a bin reaching 9 nodes in
  a table smaller than 64 doubles the table: HashMap.putVal / treeifyBin / resize).
  Tree bins (9+ nodes in one bucket of a table >= 64) order new nodes by identity hash
  codes, which no restatement can reproduce: PARITY UNPINNED there (never produced by the
  tests; the product reports the same map content in bucket order).
  DataOutputView: big-endian writeShort / writeLong / writeInt, writeBoolean = 1 byte,
  writeByte(size) keeps the low 8 bits; DataInputView.readByte is signed, so a map of
  128..255 entries (or a multiple of 256) reads back as no entries (the for loop at
  :115 runs `numDeterminantDeltas` times).
"""
from __future__ import annotations

import struct
from dataclasses import dataclass, field
import os
import sys
from typing import Dict, List, Optional, Tuple

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

E_TRUNCATED, E_CORRUPT_TAG, E_NOT_BUFFER_BUILT = -3, -2, -15


def _i16(v: int) -> int:
    v &= 0xFFFF
    return v - 0x10000 if v & 0x8000 else v


def _i32(v: int) -> int:
    v &= 0xFFFFFFFF
    return v - 0x100000000 if v & 0x80000000 else v


def _i64(v: int) -> int:
    v &= 0xFFFFFFFFFFFFFFFF
    return v - (1 << 64) if v >> 63 else v


@dataclass(frozen=True)
class LogId:
    """CausalLogID (CausalLogID.java:38-198).  Non-main fields are ignored by equality
    for main-thread ids (:138-143), so they are normalised to 0 here."""
    vertex: int
    is_main: bool = True
    lower: int = 0
    upper: int = 0
    sub: int = 0

    @staticmethod
    def main(v: int) -> "LogId":
        return LogId(_i16(v), True)

    @staticmethod
    def subpartition(v: int, lower: int, upper: int, sub: int) -> "LogId":
        return LogId(_i16(v), False, _i64(lower), _i64(upper), ((sub + 128) & 0xFF) - 128)

    def java_hash(self) -> int:  # :151-163 (Java int arithmetic)
        h = 17
        h = _i32(31 * h + self.vertex)
        h = _i32(31 * h + (1 if self.is_main else 0))
        if self.is_main:
            return h
        lo, up = self.lower & 0xFFFFFFFFFFFFFFFF, self.upper & 0xFFFFFFFFFFFFFFFF
        h = _i32(31 * h + _i32(lo ^ (lo >> 32)))
        h = _i32(31 * h + _i32(up ^ (up >> 32)))
        h = _i32(31 * h + self.sub)
        return h

    def write(self) -> bytes:  # :165-174
        if self.is_main:
            return struct.pack(">hB", self.vertex, 1)
        return struct.pack(">hBqqb", self.vertex, 0, self.lower, self.upper, self.sub)

    @staticmethod
    def read(b: bytes, p: int) -> Tuple["LogId", int]:  # :176-186
        if p + 3 > len(b):
            raise EOFError
        v, m = struct.unpack_from(">hB", b, p)
        p += 3
        if m != 0:  # readBoolean: any nonzero byte is true
            return LogId(v, True), p
        if p + 17 > len(b):
            raise EOFError
        lo, up, s = struct.unpack_from(">qqb", b, p)
        return LogId(v, False, lo, up, s), p + 17


class JavaHashMap:
    """Insertion-history-faithful model of java.util.HashMap's iteration order."""

    def __init__(self):
        self.cap = 16
        self.bins: Dict[int, List[Tuple[LogId, bytes]]] = {}
        self.size = 0

    @staticmethod
    def _spread(h: int) -> int:
        h &= 0xFFFFFFFF
        return h ^ (h >> 16)

    def _resize(self):
        old = self.items()
        self.cap *= 2
        self.bins = {}
        for k, v in old:  # iteration order; each new bin keeps its relative order
            self.bins.setdefault(self._spread(k.java_hash()) & (self.cap - 1), []).append((k, v))

    def get(self, k: LogId) -> Optional[bytes]:
        for kk, v in self.bins.get(self._spread(k.java_hash()) & (self.cap - 1), []):
            if kk == k:
                return v
        return None

    def put(self, k: LogId, v: bytes, remap=None) -> None:
        """put (remap None) or merge(k, v, remap) -- HashMap.putVal / HashMap.merge."""
        i = self._spread(k.java_hash()) & (self.cap - 1)
        b = self.bins.setdefault(i, [])
        for j, (kk, old) in enumerate(b):
            if kk == k:
                b[j] = (kk, v if remap is None else remap(old, v))
                return
        b.append((k, v))
        if len(b) >= 9 and self.cap < 64:  # treeifyBin on a small table resizes instead
            self._resize()
        self.size += 1
        if self.size > self.cap * 3 // 4:
            self._resize()

    def items(self) -> List[Tuple[LogId, bytes]]:
        out = []
        for i in sorted(self.bins):
            out.extend(self.bins[i])
        return out


@dataclass
class Response:
    """DeterminantResponseEvent (DeterminantResponseEvent.java:36-148)."""
    found: bool
    vertex: int
    corr: int = 0
    dets: JavaHashMap = field(default_factory=JavaHashMap)

    def write(self) -> bytes:  # :93-107
        out = [struct.pack(">?hqb", self.found, self.vertex, self.corr, ((self.dets.size + 128) & 0xFF) - 128)]
        for k, v in self.dets.items():
            out += [k.write(), struct.pack(">i", len(v)), v]
        return b"".join(out)

    @staticmethod
    def read(b: bytes) -> Tuple["Response", int]:  # :109-125
        if len(b) < 12:
            raise EOFError
        found, v, corr, n = struct.unpack_from(">BhqB", b, 0)
        n = n - 256 if n > 127 else n
        r = Response(found != 0, v, corr)
        p = 12
        for _ in range(max(n, 0)):
            k, p = LogId.read(b, p)
            if p + 4 > len(b):
                raise EOFError
            ln = struct.unpack_from(">i", b, p)[0]
            p += 4
            if ln < 0 or p + ln > len(b):  # new byte[negative] / readFully past the end
                raise EOFError
            r.dets.put(k, bytes(b[p:p + ln]))
            p += ln
        return r, p

    def merge(self, other: "Response") -> None:  # :128-148
        if not self.found and not other.found:
            return
        if not self.found:
            self.found = True
        for k, v in other.dets.items():
            self.dets.put(k, v, remap=lambda v1, v2: v1 if len(v1) > len(v2) else v2)


def accumulate(vertex: int, events: List[bytes]) -> Response:
    """WaitingDeterminantsState: accumulator (true, vertex) (:57) merged with each response
    in arrival order (:102)."""
    acc = Response(True, vertex)
    for ev in events:
        r, _ = Response.read(ev)
        acc.merge(r)
    return acc


def replay_spans(acc: Response, vertex: int, subparts: List[LogId]) -> List[bytes]:
    """ReplayingState: the main log (:63-66; absent -> no replay, like a null log) then one
    recovery buffer per subpartition of the task's table (:108-130; absent -> EMPTY)."""
    spans = [acc.dets.get(LogId.main(vertex)) or b""]
    for s in subparts:
        spans.append(acc.dets.get(s) or b"")
    return spans


def buffer_sizes(buf: bytes) -> List[int]:
    """SubpartitionRecoveryThread.run (:161-188): decodeNext in a loop (its exceptions come
    first), then anything but a BufferBuilt determinant raises (:172-177).  Raises
    ValueError((status, offset, signed tag), sizes_before)."""
    import pyref  # the independent decodeNext restatement
    out, p = [], 0
    while p < len(buf):
        try:
            rec, nxt = pyref.decode_one(buf, p)
        except pyref.DecodeError as e:
            raise ValueError((e.status, e.off, e.tag), out)
        if rec["tag"] != 7:
            raise ValueError((E_NOT_BUFFER_BUILT, p, rec["tag"]), out)
        out.append(rec["v0"])
        p = nxt
    return out
