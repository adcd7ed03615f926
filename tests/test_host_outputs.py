"""CPU: the host output arrays of a decode (Engine._host_outputs / _pooled_outputs) -- views of
one buffer, laid out for clg_decoded; the engine's reusable buffer is reused only when no
earlier result still references it, so a batch the caller keeps is never overwritten."""
import sys

import numpy as np

from clonos_amd.engine import Engine


class _E:  # what _pooled_outputs uses, without a GPU engine (no handle: nothing registered)
    _OUT_FIELDS = Engine._OUT_FIELDS
    _OUT_SLOTS = Engine._OUT_SLOTS
    _host_outputs = staticmethod(Engine._host_outputs)
    _out_bytes = staticmethod(Engine._out_bytes)
    _slot_release = Engine._slot_release
    _out_release = Engine._out_release
    _out_buf = Engine._out_buf
    _out_cache = Engine._out_cache
    _out_mapped = Engine._out_mapped

    def __init__(self):
        self._out_slots = []
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
    first = e._out_buf.ctypes.data
    d2, a2 = Engine._pooled_outputs(e, 100, 10)
    assert e._out_buf.ctypes.data != first  # the kept slices hold the first buffer: a second slot
    a2["off"][:3] = 7
    assert list(kept[1][:3]) == [1, 2, 3]
    del a2
    second = e._out_buf.ctypes.data
    d3, a3 = Engine._pooled_outputs(e, 100, 10)
    assert e._out_buf.ctypes.data == second and d3 is d2  # free again: reused, views and struct too
    del a3
    # the caller keeps one batch while asking for the next: two slots alternate, no new buffer
    seen = set()
    prev = None
    for _ in range(6):
        d, a = Engine._pooled_outputs(e, 100, 10)
        seen.add(e._out_buf.ctypes.data)
        prev = a  # noqa: F841 (held across the next call)
    assert len(e._out_slots) <= Engine._OUT_SLOTS and len(seen) <= 2
    assert list(kept[1][:3]) == [1, 2, 3]  # (the kept batch is never handed out)
    del prev, a, kept
    small = max(sl["buf"].size for sl in e._out_slots)
    Engine._pooled_outputs(e, 50000, 10)  # larger than every buffer: a new one
    assert e._out_buf.size > small
