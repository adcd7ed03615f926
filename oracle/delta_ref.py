"""delta_ref.py -- CPU restatement of the piggybacked causal-log delta wire format
(TEST INFRASTRUCTURE ONLY; imported by tests/ only).

Restates (R/ = /root/reference/flink-runtime/src/main/java/org/apache/flink/runtime/causal/):
  R/log/job/serde/AbstractDeltaSerializerDeserializer.java:89-163  header [size i32][epoch i64],
      processCausalLogDelta / processThreadDelta, serializeThreadDelta [ofe i32][len i32]
  R/log/job/serde/FlatDeltaSerializerDeserializer.java:57-120      per-log [CausalLogID] records
  R/log/job/serde/GroupingDeltaSerializerDeserializer.java:66-165  vertex / partition grouping
over log models with the ThreadCausalLog interface (has_delta, offset, get_delta), e.g.
tests/_oracle.OracleLog (the C++ ThreadCausalLogImpl restatement).  Logs are given in the
strategy's iteration order as (log, CausalLogID tuple (vertex, is_main, lower, upper, sub),
send) -- `send` is the Grouping strategy's post-hasDelta subpartition filter.
"""
from __future__ import annotations

import struct
from typing import List, Tuple

FLAT, HIERARCHICAL = 0, 1


def _delta(log, ch, epoch):
    st, off = log.offset(ch)
    assert st == 0
    st, d = log.get_delta(ch, epoch)
    assert st == 0
    return off, d


def serialize(strategy: int, entries, ch, epoch: int) -> bytes:
    hdr, deltas = bytearray(struct.pack(">iq", 0, epoch)), []
    if strategy == FLAT:  # Flat.serializeDataStrategy :57-90
        for log, cid, send in entries:
            st, has = log.has_delta(ch, epoch)
            assert st == 0
            if not (has and send):
                continue
            v, main, lo, hi, sub = cid
            hdr += struct.pack(">hB", v, 1 if main else 0)
            if not main:
                hdr += struct.pack(">qqb", lo, hi, sub)
            off, d = _delta(log, ch, epoch)
            hdr += struct.pack(">ii", off, len(d))
            deltas.append(d)
    else:  # Grouping.serializeVertex / serializePartitions / serializePartition :91-165
        i = 0
        while i < len(entries):
            v = entries[i][1][0]
            vstart, updates = len(hdr), 0
            hdr += struct.pack(">h", v)
            has = False
            if entries[i][1][1]:
                log = entries[i][0]
                st, has = log.has_delta(ch, epoch)
                assert st == 0
                i += 1
            hdr += bytes([1 if has else 0])
            if has:
                off, d = _delta(log, ch, epoch)
                hdr += struct.pack(">ii", off, len(d))
                deltas.append(d)
                updates += 1
            np_at, parts = len(hdr), 0
            hdr += b"\0"
            while i < len(entries) and entries[i][1][0] == v and not entries[i][1][1]:
                lo, hi = entries[i][1][2], entries[i][1][3]
                pstart = len(hdr)
                hdr += struct.pack(">qq", lo, hi)
                ns_at, subs = len(hdr), 0
                hdr += b"\0"
                while i < len(entries) and entries[i][1][0] == v and not entries[i][1][1] and \
                        entries[i][1][2:4] == (lo, hi):
                    log, cid, send = entries[i]
                    st, hs = log.has_delta(ch, epoch)
                    assert st == 0
                    if hs and send:
                        hdr += struct.pack(">b", cid[4])
                        off, d = _delta(log, ch, epoch)
                        hdr += struct.pack(">ii", off, len(d))
                        deltas.append(d)
                        subs += 1
                    i += 1
                if subs == 0:
                    del hdr[pstart:]
                else:
                    hdr[ns_at] = subs
                    parts += 1
            hdr[np_at] = parts
            updates += parts
            if updates == 0:
                del hdr[vstart:]
    struct.pack_into(">i", hdr, 0, len(hdr))
    return bytes(hdr) + b"".join(deltas)


def parse(strategy: int, msg: bytes) -> Tuple[int, List[Tuple[tuple, int, bytes]]]:
    """processCausalLogDelta: (epoch, [(CausalLogID tuple, offsetFromEpoch, delta bytes)])."""
    hsize, epoch = struct.unpack_from(">iq", msg, 0)
    p, at, out = 12, hsize, []

    def thread(cid):
        nonlocal p, at
        off, n = struct.unpack_from(">ii", msg, p)
        p += 8
        out.append((cid, off, msg[at:at + n]))
        at += n

    while p < hsize:
        v, main = struct.unpack_from(">hB", msg, p)
        p += 3
        if strategy == FLAT:
            if main:
                thread((v, True, 0, 0, 0))
            else:
                lo, hi, sub = struct.unpack_from(">qqb", msg, p)
                p += 17
                thread((v, False, lo, hi, sub))
        else:
            if main:
                thread((v, True, 0, 0, 0))
            npart = struct.unpack_from(">b", msg, p)[0]
            p += 1
            for _ in range(npart):
                lo, hi, ns = struct.unpack_from(">qqb", msg, p)
                p += 17
                for _ in range(ns):
                    sub = struct.unpack_from(">b", msg, p)[0]
                    p += 1
                    thread((v, False, lo, hi, sub))
    return epoch, out
