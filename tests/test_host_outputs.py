"""CPU: the host output arrays of a decode (Engine._host_outputs / _pooled_outputs) -- views of
one buffer, laid out for clg_decoded; the engine's reusable buffer is reused only when no
earlier result still references it, so a batch the caller keeps is never overwritten."""
import sys

import numpy as np

from clonos_amd.engine import Engine


class _E:  # what _pooled_outputs uses, without a GPU engine (no handle: nothing registered)
    _OUT_FIELDS = Engine._OUT_FIELDS
    _host_outputs = staticmethod(Engine._host_outputs)
    _out_bytes = staticmethod(Engine._out_bytes)
    _out_release = Engine._out_release

    def __init__(self):
        self._out_buf = None
        self._out_cache = None
        self._out_mapped = False
        self._h = None


def test_layout_matches_pointers():
    d, a = Engine._host_outputs(1000, 300)
    base = a["off"].base
    b0 = base.ctypes.data
    for k, dt, isz, wide in Engine._OUT_FIELDS:
        assert a[k].dtype == dt and a[k].size == (300 if wide else 1000)
        assert getattr(d, k) == a[k].ctypes.data and a[k].base is base
        assert (getattr(d, k) - b0) % 16 == 0
    ends = sorted((getattr(d, k), getattr(d, k) + a[k].nbytes) for k in a)
    assert all(e0 <= s1 for (_, e0), (s1, _) in zip(ends, ends[1:]))  # no overlap
    assert d.cap == 1000 and d.wcap == 300


def test_pool_never_overwrites_a_live_batch():
    e = _E()
    d0, a0 = Engine._pooled_outputs(e, 100, 10)
    assert a0["off"].base is e._out_buf and e._out_buf.ctypes.data % 4096 == 0  # page-aligned, views on it
    del a0
    d, a = Engine._pooled_outputs(e, 100, 10)
    a["off"][:3] = [1, 2, 3]
    kept = a["v0"][:2], a["off"][:5]
    del a
    first = id(e._out_buf)
    d2, a2 = Engine._pooled_outputs(e, 100, 10)
    assert id(e._out_buf) != first  # the kept slices hold the first buffer
    a2["off"][:3] = 7
    assert list(kept[1][:3]) == [1, 2, 3]
    del kept, a2
    second = id(e._out_buf)
    d3, a3 = Engine._pooled_outputs(e, 100, 10)
    assert id(e._out_buf) == second and d3 is d2  # free again: reused, views and struct too
    del a3
    small = e._out_buf.size
    Engine._pooled_outputs(e, 50000, 10)  # larger than the buffer: a new one
    assert e._out_buf.size > small
    assert sys.getrefcount(e._out_buf) > 3  # the cache's views hold it
