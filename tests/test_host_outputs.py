"""CPU: the host output arrays of a decode (Engine._host_outputs / _pooled_outputs) -- views of
one buffer, laid out for clg_decoded; the engine's reusable buffer is reused only when no
earlier result still references it, so a batch the caller keeps is never overwritten."""
import sys
import threading

import numpy as np

from clonos_amd.engine import Engine


class _E:  # what _pooled_outputs uses, without a GPU engine (no handle: nothing registered)
    _OUT_FIELDS = Engine._OUT_FIELDS
    _OUT_SLOTS = Engine._OUT_SLOTS
    _host_outputs = staticmethod(Engine._host_outputs)
    _out_bytes = staticmethod(Engine._out_bytes)
    _slot_capacity = staticmethod(Engine._slot_capacity)
    _slot_free = staticmethod(Engine._slot_free)
    _slot_done = Engine._slot_done
    _slot_use = Engine._slot_use
    _pooled_pick = Engine._pooled_pick
    _pooled_fast = Engine._pooled_fast
    _slot_release = Engine._slot_release
    _out_release = Engine._out_release
    _out_buf = Engine._out_buf
    _out_cache = Engine._out_cache
    _out_mapped = Engine._out_mapped

    def __init__(self):
        self._out_slots = []
        self._h = None
        self._pool_mu = threading.Lock()


def _take(e, cap, wcap, bcap=0):
    """A pick as a decode makes it: _pooled_outputs, then _finish ends the pick."""
    d, a, _ = Engine._pooled_outputs(e, cap, wcap, bcap)
    e._slot_done(a)
    return d, a


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
    d0, a0 = _take(e, 100, 10)
    assert a0["off"].base is e._out_buf and e._out_buf.ctypes.data % 4096 == 0  # page-aligned, views on it
    del a0
    d, a = _take(e, 100, 10)
    a["off"][:3] = [1, 2, 3]
    kept = a["v0"][:2], a["off"][:5]
    del a
    first = e._out_buf.ctypes.data
    d2, a2 = _take(e, 100, 10)
    assert e._out_buf.ctypes.data != first  # the kept slices hold the first buffer: a second slot
    a2["off"][:3] = 7
    assert list(kept[1][:3]) == [1, 2, 3]
    del a2
    second = e._out_buf.ctypes.data
    d3, a3 = _take(e, 100, 10)
    assert e._out_buf.ctypes.data == second and d3 is d2  # free again: reused, views and struct too
    del a3
    # the caller keeps one batch while asking for the next: two slots alternate, no new buffer
    seen = set()
    prev = None
    for _ in range(6):
        d, a = _take(e, 100, 10)
        seen.add(e._out_buf.ctypes.data)
        prev = a  # noqa: F841 (held across the next call)
    assert len(e._out_slots) <= Engine._OUT_SLOTS and len(seen) <= 2
    assert list(kept[1][:3]) == [1, 2, 3]  # (the kept batch is never handed out)
    del prev, a, kept
    small = max(sl["buf"].size for sl in e._out_slots)
    _take(e, 50000, 10)  # larger than every buffer: a new one
    assert e._out_buf.size > small


def test_views_cover_the_slot_and_serve_smaller_requests():
    e = _E()
    d, a = _take(e, 100, 10, 5)
    size = e._out_buf.size
    assert d.cap >= 100 and d.wcap >= 10 and a["base"].size >= 256  # carved at the slot's capacity
    assert Engine._out_bytes(d.cap, d.wcap, a["base"].size)[1] <= size
    assert a["base"].ctypes.data >= getattr(d, "w_sub") + d.wcap  # span_rec_base after the nine arrays
    del a
    d2, a2 = _take(e, 50, 3, 2)
    assert d2 is d and e._out_buf.size == size  # covered: the same views and struct
    assert len(e._out_slots) == 1


def test_a_picked_slot_is_busy_until_finish():
    e = _E()
    d, a, _ = Engine._pooled_outputs(e, 100, 10)  # picked, no _finish yet (e.g. an async decode)
    first = e._out_buf.ctypes.data
    for _ in range(2 * Engine._OUT_SLOTS):  # never handed out again, never evicted while busy
        _take(e, 100, 10)
        assert e._out_slots[0]["buf"].ctypes.data == first or any(
            sl["buf"].ctypes.data == first for sl in e._out_slots)
    assert all(sl["buf"].ctypes.data != first or sl["busy"] for sl in e._out_slots)
    e._slot_done(a)
    assert not any(sl["busy"] for sl in e._out_slots)


def test_fast_pick_needs_a_registered_slot_with_enough_span_entries():
    e = _E()
    _take(e, 100, 10, 5)
    assert e._pooled_fast(4) is None  # not registered (no device here)
    e._out_slots[0]["mapped"] = True
    nb = e._out_slots[0]["cache"][0][2]
    assert e._pooled_fast(nb) is None  # span_rec_base needs n_spans + 1 entries
    d, a, ref, bptr = e._pooled_fast(nb - 1)
    assert bptr == a["base"].ctypes.data and e._out_slots[-1]["busy"]
    assert e._pooled_fast(4) is None  # busy
    e._slot_done(a)
    e._out_slots[0]["mapped"] = False  # (nothing to unregister)
