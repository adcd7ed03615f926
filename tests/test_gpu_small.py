"""GPU: the single-launch small-batch decode (k_decode_small_tiles: a block per tile, each
entering at its predecessor's published exit, look-back over the earlier tiles' counts, host
outputs written straight into pinned memory) == the CPU
oracle's decodeNext loop, bit-exact; batches it does not finish (an invalid record, a
Serializable record) fall back to the three-pass path with the same result."""
import numpy as np
import pytest

import _oracle as O
from clonos_amd import ClonosError, Engine, synth
from test_gpu_decode import assert_span_equal

pytestmark = pytest.mark.gpu


def _eng(**kw):
    return Engine(segment_bytes=kw.pop("segment_bytes", 16384), pool_segments=4096, timing=True, **kw)


def _launches(eng, name):
    return eng.kernel_stats().get(name, {}).get("launches", 0)


def test_config1_decode_takes_the_small_path():
    rng = np.random.default_rng(synth.SEED_CONFIG1)
    graph, data = synth.config1_job(rng)
    with _eng(sharing_depth=1) as eng:
        logs = {lid: eng.open_log(lid) for lid in data}
        for lid, b in data.items():
            logs[lid].appendDeterminant(b, 0)
        lids = list(data)
        eng.kernel_stats_reset()
        dec = eng.decode_logs([logs[l] for l in lids], [0] * len(lids))
        assert _launches(eng, "decode_small") == 1 and _launches(eng, "decode_small_fallback") == 0
        assert _launches(eng, "decode_count") == 0
        for s, l in enumerate(lids):
            assert_span_equal(dec, s, data[l])


@pytest.mark.parametrize("seed", range(3))
@pytest.mark.parametrize("seg", [256, 16384])
def test_small_random_spans_multi_tile(seed, seg):
    """Spans of 0 .. 8 tiles (up to ~64 KB), every non-Serializable tag, logs across segments."""
    rng = np.random.default_rng(0x5A11 + seed)
    with _eng(segment_bytes=seg) as eng:
        from clonos_amd import CausalLogID
        bufs, logs = [], []
        # <= 8 tiles per span (records average ~28 bytes)
        sizes = [0, 1, 5, 50, 400, 1500] if seg == 16384 else [0, 1, 5, 20, 40]
        for i in range(int(rng.integers(1, 60))):
            n = int(rng.choice(sizes))
            b = synth.random_log(n, rng, allow_serializable=False)
            if len(b) > 60000:
                b = b[:0]
            lg = eng.open_log(CausalLogID.main(i))
            if b:
                lg.appendDeterminant(b, 0)
            bufs.append(b)
            logs.append(lg)
        eng.kernel_stats_reset()
        dec = eng.decode_logs(logs, [0] * len(logs))
        assert _launches(eng, "decode_small") == 1 and _launches(eng, "decode_small_fallback") == 0
        for s, b in enumerate(bufs):
            assert_span_equal(dec, s, b)
        assert dec.span_rec_base[-1] == dec.n_rec


@pytest.mark.parametrize("n_spans", [1, 7])
def test_small_all_empty_spans_need_no_launch(n_spans):
    """A batch of empty spans (a log truncated to its end, an empty replay batch) has no
    tiles: no records, every span starts at 0, and nothing is launched."""
    from clonos_amd import CausalLogID
    with _eng() as eng:
        logs = [eng.open_log(CausalLogID.main(i)) for i in range(n_spans)]
        eng.kernel_stats_reset()
        dec = eng.decode_logs(logs, [0] * n_spans)
        assert dec.n_rec == 0 and list(dec.span_rec_base) == [0] * (n_spans + 1)
        assert _launches(eng, "decode_small") == 0 and _launches(eng, "decode_count") == 0
        dec = eng.decode_host(b"", [(0, 0)] * n_spans)
        assert dec.n_rec == 0 and list(dec.span_rec_base) == [0] * (n_spans + 1)
        # a non-empty batch after it still decodes on the small path
        rng = np.random.default_rng(9)
        b = synth.random_log(300, rng, allow_serializable=False)
        logs[0].appendDeterminant(b, 0)
        dec = eng.decode_logs(logs, [0] * n_spans)
        assert_span_equal(dec, 0, b)
        assert _launches(eng, "decode_small") == 1


def test_small_host_input_spans():
    rng = np.random.default_rng(3)
    parts = [synth.random_log(int(rng.integers(0, 300)), rng, allow_serializable=False) for _ in range(200)]
    blob, spans = b"", []
    for p in parts:
        blob += bytes(int(rng.integers(0, 17)))
        spans.append((len(blob), len(p)))
        blob += p
    with _eng() as eng:
        eng.kernel_stats_reset()
        dec = eng.decode_host(blob, spans)
        assert _launches(eng, "decode_small") == 1
        for s, p in enumerate(parts):
            assert_span_equal(dec, s, p)


def test_small_error_falls_back_with_the_reference_error():
    rng = np.random.default_rng(4)
    good = [synth.random_log(200, rng, allow_serializable=False) for _ in range(10)]
    bad = good[3][:37] + bytes([9]) + good[3][37:]  # tag 9 at a record start? (the oracle decides)
    spans_b = good[:3] + [bad] + good[4:]
    blob = b"".join(spans_b)
    offs = np.cumsum([0] + [len(b) for b in spans_b])
    with _eng() as eng:
        eng.kernel_stats_reset()
        try:
            dec = eng.decode_host(blob, [(int(offs[i]), len(b)) for i, b in enumerate(spans_b)])
            got = None
        except ClonosError as e:
            got = e.status
        st, _, _, _ = O.decode(bad)
        assert _launches(eng, "decode_small") == 1  # launched (and, on an error, fallen back)
        if st != 0:
            assert got == st and _launches(eng, "decode_small_fallback") == 1
        else:
            assert got is None
            for s, b in enumerate(spans_b):
                assert_span_equal(dec, s, b)


def test_small_serializable_falls_back():
    rng = np.random.default_rng(5)
    buf = synth.random_log(500, rng, allow_serializable=True)
    with _eng() as eng:
        eng.kernel_stats_reset()
        dec = eng.decode_host(buf)
        assert_span_equal(dec, 0, buf)
        if b"\x03\xac\xed\x00\x05" in buf:
            assert _launches(eng, "decode_small_fallback") >= 1


def test_small_device_outputs():
    import torch
    from clonos_amd import _lib, CausalLogID
    rng = np.random.default_rng(6)
    with _eng() as eng:
        bufs = [synth.random_log(int(rng.integers(1, 800)), rng, allow_serializable=False) for _ in range(30)]
        logs = []
        for i, b in enumerate(bufs):
            lg = eng.open_log(CausalLogID.main(i))
            lg.appendDeterminant(b, 0)
            logs.append(lg)
        n_cap = sum(len(b) for b in bufs) // 2 + 1
        dev = torch.device("cuda", 0)
        o = [torch.empty(n_cap, dtype=t, device=dev) for t in (torch.int32, torch.uint8, torch.int64)]
        ow = [torch.empty(n_cap, dtype=t, device=dev) for t in
              (torch.int32, torch.int32, torch.int64, torch.int32, torch.int32, torch.uint8)]
        d = _lib.Decoded()
        d.off, d.tag, d.v0 = [t.data_ptr() for t in o]
        d.w_idx, d.w_rc, d.w_v1, d.w_var_off, d.w_var_len, d.w_sub = [t.data_ptr() for t in ow]
        d.cap, d.wcap, d.out_kind = n_cap, n_cap, _lib.CLG_MEM_DEVICE
        base = np.zeros(len(bufs) + 1, np.uint64)
        eng.kernel_stats_reset()
        eng.decode_logs_device(np.array([l.handle for l in logs], np.uint32), np.zeros(len(logs), np.int64), d, base)
        assert _launches(eng, "decode_small") == 1
        tag = o[1][:d.n_rec].cpu().numpy()
        v0 = o[2][:d.n_rec].cpu().numpy()
        for s, b in enumerate(bufs):
            st, r, _, _ = O.decode(b)
            lo, hi = int(base[s]), int(base[s + 1])
            np.testing.assert_array_equal(tag[lo:hi], r["tag"])
            np.testing.assert_array_equal(v0[lo:hi], r["v0"])


def test_small_mapped_outputs_kept_batches_stay_intact():
    """decode_logs' outputs are views of the engine's pooled, registered host buffer
    (CLG_MEM_MAPPED): the small decode writes them from the GPU.  A batch the caller keeps is
    never overwritten -- the next decode gets a new buffer -- and both equal the oracle; once
    the kept batch is dropped the pool's buffer is reused."""
    from clonos_amd import _lib
    rng = np.random.default_rng(synth.SEED_CONFIG1)
    graph, data = synth.config1_job(rng)
    with _eng(sharing_depth=1) as eng:
        logs = {lid: eng.open_log(lid) for lid in data}
        for lid, b in data.items():
            logs[lid].appendDeterminant(b, 0)
        lids = list(data)
        first = eng.decode_logs([logs[l] for l in lids], [0] * len(lids))
        assert eng._out_mapped and eng._out_cache[1].out_kind == _lib.CLG_MEM_MAPPED
        snap = first.v0.copy()
        buf1 = eng._out_buf.ctypes.data
        second = eng.decode_logs([logs[l] for l in lids], [0] * len(lids))
        assert eng._out_buf.ctypes.data != buf1  # the kept batch holds the first buffer
        np.testing.assert_array_equal(first.v0, snap)
        for dec in (first, second):
            for s, l in enumerate(lids):
                assert_span_equal(dec, s, data[l])
        del first, dec
        buf2 = eng._out_buf.ctypes.data
        del second
        third = eng.decode_logs([logs[l] for l in lids], [0] * len(lids))
        assert eng._out_buf.ctypes.data in (buf1, buf2) and len(eng._out_slots) == 2  # free again: reused
        for s, l in enumerate(lids):
            assert_span_equal(third, s, data[l])


def test_pooled_capacity_exceeded_is_decoded_again_sized():
    """decode_logs first tries the free registered slot at its whole capacity, without
    logLength; a batch with more records than the slot holds fails there with CLG_E_CAPACITY
    (nothing changed) and is decoded again into a slot sized from logLength."""
    rng = np.random.default_rng(synth.SEED_CONFIG1)
    graph, data = synth.config1_job(rng)
    with _eng(sharing_depth=1) as eng:
        logs = {lid: eng.open_log(lid) for lid in data}
        for lid, b in data.items():
            logs[lid].appendDeterminant(b, 0)
        lids = list(data)
        first = eng.decode_logs([logs[l] for l in lids], [0] * len(lids))
        cap = eng._out_cache[0][0]
        del first
        big = bytes(synth.config2_log(cap + 5000, rng)[0])  # more records than the slot holds
        logs[lids[0]].appendDeterminant(big, 0)
        dec = eng.decode_logs([logs[l] for l in lids], [0] * len(lids))
        assert eng._out_cache[0][0] > cap and dec.n_rec > cap
        assert_span_equal(dec, 0, data[lids[0]] + big)
        for s, l in enumerate(lids[1:], 1):
            assert_span_equal(dec, s, data[l])


@pytest.mark.parametrize("decode", ["auto", "three_pass"])
def test_multi_tile_spans_take_the_single_launch(decode):
    """A batch of 16 config-2 logs of ~45 KB (config 5's failed main logs, 6 tiles each) goes to
    the single launch (a block per tile; the chain's merge is the only serial part along a span)
    -- or, with it turned off (decode="three_pass"), three-pass -- with the same result."""
    per_tile = decode == "auto"
    rng = np.random.default_rng(0xC5)
    from clonos_amd import CausalLogID
    with _eng(decode=decode) as eng:
        bufs = [synth.config2_log(8000, rng)[0].tobytes() for _ in range(16)]
        small = [synth.config2_log(900, rng)[0].tobytes() for _ in range(4)]  # <= 2 tiles each
        logs = []
        for i, b in enumerate(bufs + small):
            lg = eng.open_log(CausalLogID.main(i))
            lg.appendDeterminant(b, 0)
            logs.append(lg)
        eng.kernel_stats_reset()
        dec = eng.decode_logs(logs[:16], [0] * 16)
        if per_tile:
            assert _launches(eng, "decode_small") == 1 and _launches(eng, "decode_count") == 0
        else:
            assert _launches(eng, "decode_small") == 0 and _launches(eng, "decode_count") == 1
        for s, b in enumerate(bufs):
            assert_span_equal(dec, s, b)
        eng.kernel_stats_reset()
        dec = eng.decode_logs(logs[16:], [0] * 4)
        assert _launches(eng, "decode_small") == (1 if per_tile else 0)
        for s, b in enumerate(small):
            assert_span_equal(dec, s, b)
