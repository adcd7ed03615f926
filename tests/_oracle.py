"""ctypes wrapper of the C++ CPU oracle (oracle/liboracle.so).  Test infrastructure only."""
from __future__ import annotations

import ctypes as C
import os
import subprocess
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORACLE_DIR = os.path.join(ROOT, "oracle")
LIB = os.path.join(ORACLE_DIR, "liboracle.so")
sys.path.insert(0, ORACLE_DIR)
import pyref  # noqa: E402  (independent Python restatement)


def _build():
    src = os.path.join(ORACLE_DIR, "clonos_oracle.cpp")
    if not os.path.exists(LIB) or os.path.getmtime(LIB) < os.path.getmtime(src):
        subprocess.run(["make", "-C", ORACLE_DIR, "-s", "liboracle.so"], check=True)


_build()
lib = C.CDLL(LIB)
P = C.c_void_p
lib.orc_jser_len.restype = C.c_int64
lib.orc_jser_len.argtypes = [C.c_char_p, C.c_size_t]
lib.orc_decode_span.restype = C.c_int
lib.orc_decode_span.argtypes = [P, C.c_size_t] + [P] * 9 + [C.c_size_t, C.c_size_t, C.POINTER(C.c_size_t),
                                                          C.POINTER(C.c_size_t), C.POINTER(C.c_int64),
                                                          C.POINTER(C.c_int32)]
lib.orc_log_new.restype = P
lib.orc_log_new.argtypes = [C.c_uint32, C.c_int32]
lib.orc_log_free.argtypes = [P]
for n, a in {
    "orc_log_append": [P, C.c_int64, C.c_char_p, C.c_uint32],
    "orc_log_upstream": [P, C.c_char_p, C.c_uint32, C.c_int32, C.c_int64],
    "orc_log_has_delta": [P, C.c_uint64, C.c_uint64, C.c_int64, C.POINTER(C.c_int)],
    "orc_log_offset": [P, C.c_uint64, C.c_uint64, C.POINTER(C.c_int32)],
    "orc_log_get_delta": [P, C.c_uint64, C.c_uint64, C.c_int64, P, C.c_uint32, C.POINTER(C.c_uint32)],
    "orc_log_get_determinants": [P, C.c_int64, P, C.c_uint32, C.POINTER(C.c_uint32)],
    "orc_log_length": [P, C.POINTER(C.c_int32)],
    "orc_log_checkpoint_complete": [P, C.c_int64],
    "orc_log_unregister": [P, C.c_uint64, C.c_uint64],
    "orc_log_state": [P, C.POINTER(C.c_int32), C.POINTER(C.c_int32), C.POINTER(C.c_int32), P, P, C.c_int32,
                      C.POINTER(C.c_int32)],
    "orc_log_consumer": [P, C.c_uint64, C.c_uint64, C.POINTER(C.c_int), C.POINTER(C.c_int64),
                         C.POINTER(C.c_int32)],
    "orc_log_read_phys": [P, C.c_int32, C.c_uint32, P],
}.items():
    getattr(lib, n).restype = C.c_int
    getattr(lib, n).argtypes = a
class OrcDet(C.Structure):
    _fields_ = [("tag", C.c_uint8), ("v0", C.c_int64), ("record_count", C.c_int32), ("v1", C.c_int64),
                ("sub", C.c_uint8), ("var", C.c_void_p), ("var_len", C.c_uint32)]


lib.orc_encode.restype = C.c_int64
lib.orc_encode.argtypes = [C.POINTER(OrcDet), C.c_void_p, C.c_size_t]
lib.orc_bench_decode.restype = C.c_int64
lib.orc_bench_decode.argtypes = [P, P, P, C.c_uint32, C.c_uint32]
lib.orc_bench_slice.restype = C.c_int64
lib.orc_bench_slice.argtypes = [P, P, P, P, C.c_uint32, P, C.c_uint32]


def ptr(a: np.ndarray) -> int:
    return a.ctypes.data if a.size else 0


def encode_soa(tag, v0, w_idx=(), w_rc=(), w_v1=(), w_var_off=(), w_var_len=(), w_sub=(), var: bytes = b"") -> bytes:
    """orc_encode (SimpleDeterminantEncoder.encodeTo) record by record over the decode's SoA
    layout: side row k belongs to record w_idx[k]; payloads are var[w_var_off, +w_var_len)."""
    side = {int(w_idx[k]): k for k in range(len(w_idx))}
    vb = np.frombuffer(bytes(var) or b"\0", np.uint8)
    base = vb.ctypes.data
    out = bytearray()
    buf = np.zeros(64, np.uint8)
    d = OrcDet()
    for i in range(len(tag)):
        d.tag, d.v0 = int(tag[i]), int(v0[i])
        k = side.get(i)
        d.record_count = int(w_rc[k]) if k is not None else 0
        d.v1 = int(w_v1[k]) if k is not None else 0
        d.sub = int(w_sub[k]) if k is not None else 0
        vl = int(w_var_len[k]) if k is not None else 0
        d.var, d.var_len = (base + int(w_var_off[k])) if vl else None, vl
        if buf.size < 64 + vl:
            buf = np.zeros(64 + vl, np.uint8)
        n = lib.orc_encode(C.byref(d), buf.ctypes.data, buf.size)
        if n < 0:
            raise ValueError(f"orc_encode status {n} at record {i}")
        out += buf[:n].tobytes()
    return bytes(out)


def jser_len(b: bytes) -> int:
    return lib.orc_jser_len(b, len(b))


def decode(buf: bytes):
    """Returns (status, records dict of numpy arrays, err_off, err_tag)."""
    arr = np.frombuffer(bytes(buf) or b"\0", np.uint8)
    n = len(buf)
    cap = n // 2 + 1
    off = np.zeros(cap, np.uint32)
    tag = np.zeros(cap, np.uint8)
    v0 = np.zeros(cap, np.int64)
    w_idx = np.zeros(cap, np.uint32)
    w_rc = np.zeros(cap, np.int32)
    w_v1 = np.zeros(cap, np.int64)
    w_vo = np.zeros(cap, np.uint32)
    w_vl = np.zeros(cap, np.uint32)
    w_sub = np.zeros(cap, np.uint8)
    nr, nw = C.c_size_t(), C.c_size_t()
    eo, et = C.c_int64(), C.c_int32()
    st = lib.orc_decode_span(ptr(arr), n, ptr(off), ptr(tag), ptr(v0), ptr(w_idx), ptr(w_rc), ptr(w_v1), ptr(w_vo),
                             ptr(w_vl), ptr(w_sub), cap, cap, C.byref(nr), C.byref(nw), C.byref(eo), C.byref(et))
    r, w = nr.value, nw.value
    recs = dict(off=off[:r], tag=tag[:r], v0=v0[:r], w_idx=w_idx[:w], w_rc=w_rc[:w], w_v1=w_v1[:w],
                w_var_off=w_vo[:w], w_var_len=w_vl[:w], w_sub=w_sub[:w])
    return st, recs, eo.value, et.value


class OracleLog:
    """ThreadCausalLogImpl model (C++)."""

    def __init__(self, component: int, depth: int = -1):
        self.h = lib.orc_log_new(component, depth)
        self.C = component

    def __del__(self):
        if getattr(self, "h", None):
            lib.orc_log_free(self.h)
            self.h = None

    @staticmethod
    def _ch(ch):
        return (ch[0], ch[1]) if isinstance(ch, tuple) else (int(ch), 0)

    def append(self, epoch, data: bytes):
        return lib.orc_log_append(self.h, epoch, bytes(data), len(data))

    def upstream(self, delta: bytes, off: int, epoch: int):
        return lib.orc_log_upstream(self.h, bytes(delta), len(delta), off, epoch)

    def has_delta(self, ch, epoch):
        v = C.c_int()
        lo, hi = self._ch(ch)
        st = lib.orc_log_has_delta(self.h, lo, hi, epoch, C.byref(v))
        return st, bool(v.value)

    def offset(self, ch):
        v = C.c_int32()
        lo, hi = self._ch(ch)
        st = lib.orc_log_offset(self.h, lo, hi, C.byref(v))
        return st, v.value

    def get_delta(self, ch, epoch):
        cap = max(self.state()["capacity"], 1)
        buf = np.zeros(cap, np.uint8)
        n = C.c_uint32()
        lo, hi = self._ch(ch)
        st = lib.orc_log_get_delta(self.h, lo, hi, epoch, ptr(buf), cap, C.byref(n))
        return st, buf[:n.value].tobytes()

    def get_determinants(self, epoch):
        cap = max(self.state()["capacity"], 1)
        buf = np.zeros(cap, np.uint8)
        n = C.c_uint32()
        st = lib.orc_log_get_determinants(self.h, epoch, ptr(buf), cap, C.byref(n))
        return st, buf[:n.value].tobytes()

    def log_length(self):
        v = C.c_int32()
        lib.orc_log_length(self.h, C.byref(v))
        return v.value

    def checkpoint_complete(self, cp):
        return lib.orc_log_checkpoint_complete(self.h, cp)

    def unregister(self, ch):
        lo, hi = self._ch(ch)
        return lib.orc_log_unregister(self.h, lo, hi)

    def state(self):
        w, c, n, ne = C.c_int32(), C.c_int32(), C.c_int32(), C.c_int32()
        ids = np.zeros(4096, np.int64)
        offs = np.zeros(4096, np.int32)
        lib.orc_log_state(self.h, C.byref(w), C.byref(c), C.byref(n), ptr(ids), ptr(offs), 4096, C.byref(ne))
        k = ne.value
        return dict(writer=w.value, capacity=c.value, n_components=n.value,
                    epochs=list(zip(ids[:k].tolist(), offs[:k].tolist())))

    def consumer(self, ch):
        ex, ep, off = C.c_int(), C.c_int64(), C.c_int32()
        lo, hi = self._ch(ch)
        lib.orc_log_consumer(self.h, lo, hi, C.byref(ex), C.byref(ep), C.byref(off))
        return (ep.value, off.value) if ex.value else None

    def read_phys(self, phys, n):
        buf = np.zeros(max(n, 1), np.uint8)
        st = lib.orc_log_read_phys(self.h, phys, n, ptr(buf))
        return st, buf[:n].tobytes()
