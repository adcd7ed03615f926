"""GPU: decode errors in many spans.  A config-3-like batch where a third (or a fifth) of the
spans hold a decode error (an invalid tag, a truncated record, a bad enum, a negative name
length) is decoded three ways:
  * the fast path keeping the errors (the default: the count pass records each span's error
    position and the records before it, k_err_classify confirms the error by the full rules,
    no robust decode -- decode_kept_errors);
  * the fast path with errors not kept (CLONOS_KEEP_ERRORS=0): every bad span in ONE robust
    run, the records placed by one kernel (engine.cpp span_fallback, k_sf_place);
  * the robust pipeline alone.
Every output array, every span's record base and the first error (status, span, offset, tag)
are identical, and the oracle agrees with each good span.  SimpleDeterminantEncoder.decodeNext
(:78-342)."""
import os
import numpy as np
import pytest

import _oracle as O
from clonos_amd import Engine, _lib, synth
from clonos_amd import determinants as D
from clonos_amd._lib import lib
from clonos_amd.engine import _np_ptr

pytestmark = pytest.mark.gpu


def _corrupt(b: bytes, offs, rng, kind: int) -> bytes:
    k = int(offs[int(rng.integers(1, max(2, len(offs) - 1)))])
    if kind == 0:  # an invalid tag where a record starts
        return b[:k] + b"\x0b" + b[k:]
    if kind == 1:  # a record past the span end
        return b + D.encode(D.TimestampDeterminant(3))[:6]
    if kind == 2:  # a TimerTrigger with an out-of-range type ordinal (bad enum)
        r = bytearray(D.encode(D.TimerTriggerDeterminant(1, 2, D.INTERNAL, b"x")))
        r[13] = 9
        return b[:k] + bytes(r) + b[k:]
    r = bytearray(D.encode(D.TimerTriggerDeterminant(1, 2, 6, b"abcd")))  # a negative name length
    r[14:18] = (0xFFFFFFF0).to_bytes(4, "big")
    return b[:k] + bytes(r) + b[k:]


def _raw_decode(eng, blob, spans):
    buf = np.frombuffer(blob, np.uint8)
    so = np.array([s[0] for s in spans], np.uint64)
    sl = np.array([s[1] for s in spans], np.uint64)
    cap, wcap = int(sl.sum()) // 2 + len(spans) + 1, int(sl.sum()) // 6 + len(spans) + 1
    d, arrs = Engine._host_outputs(cap, wcap)
    base = np.zeros(len(spans) + 1, np.uint64)
    st = lib.clg_decode_host(eng.handle, _np_ptr(buf), _np_ptr(so), _np_ptr(sl), len(spans), _lib.C.byref(d),
                             _np_ptr(base))
    nr, nw = d.n_rec, d.n_wide
    return (st, d.err_status, d.err_span, d.err_off, d.err_tag, nr, nw,
            {k: v[:nr if k in ("off", "tag", "v0") else nw].copy() for k, v in arrs.items()}, base.copy())


def check_spans_oracle(a, spans_b, key):
    rec0, recs = a[8], a[7]
    widx = recs["w_idx"].astype(np.int64)
    for s, b in enumerate(spans_b):
        st, rr, eo, _ = O.decode(b)
        lo, hi = int(rec0[s]), int(rec0[s + 1])
        assert hi - lo == len(rr["tag"]), (key, s, st)
        for f in ("off", "tag", "v0"):
            np.testing.assert_array_equal(recs[f][lo:hi], rr[f], err_msg=f"{key} span {s} {f}")
        w = (widx >= lo) & (widx < hi)
        np.testing.assert_array_equal(widx[w] - lo, rr["w_idx"].astype(np.int64), err_msg=f"{key} span {s} w_idx")
        for f in ("w_rc", "w_v1", "w_var_off", "w_var_len", "w_sub"):
            np.testing.assert_array_equal(recs[f][w], rr[f], err_msg=f"{key} span {s} {f}")


@pytest.mark.parametrize("n_spans,every", [(60, 3), (600, 5)])
def test_many_bad_spans_equal_robust(n_spans, every):
    rng = np.random.default_rng(n_spans)
    spans_b, bad = [], []
    for i in range(n_spans):
        b, offs = synth.config3_epoch(int(rng.integers(300, 3000)), rng)
        b = b.tobytes()
        if i % every == 1:
            b = _corrupt(b, offs, rng, len(bad) % 4)
            bad.append(i)
        spans_b.append(b)
    blob, spans = b"", []
    for b in spans_b:
        spans.append((len(blob), len(b)))
        blob += b
    res = {}
    for mode, keep in (("three_pass", "1"), ("three_pass", "0"), ("robust", "1")):
        os.environ["CLONOS_KEEP_ERRORS"] = keep
        try:
            with Engine(segment_bytes=16384, pool_segments=1 << 12, timing=True, decode=mode) as eng:
                res[mode, keep] = _raw_decode(eng, blob, spans)
                ks = eng.kernel_stats()
        finally:
            del os.environ["CLONOS_KEEP_ERRORS"]
        if mode == "three_pass":
            assert "decode_fallback" not in ks, ks
            if keep == "1":  # every error confirmed and kept: no robust decode at all
                assert "decode_kept_errors" in ks and "decode_span_fallback" not in ks, ks
            else:
                assert "decode_span_fallback" in ks and "decode_kept_errors" not in ks, ks
    r = res["robust", "1"]
    for key in (("three_pass", "1"), ("three_pass", "0")):
        a = res[key]
        assert a[0] != 0 and a[:7] == r[:7], key  # status, error fields, record and wide-row counts
        assert a[2] == bad[0]  # the lowest bad span's error
        for k in a[7]:
            np.testing.assert_array_equal(a[7][k], r[7][k], err_msg=f"{key} {k}")
        np.testing.assert_array_equal(a[8], r[8])
    # every span against the oracle, in every mode: a good span's records, a bad span's records
    # up to its first error (decodeNext stops there), with their wide rows
    for key, a in res.items():
        check_spans_oracle(a, spans_b, key)
