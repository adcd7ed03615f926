"""GPU: replay preparation after concurrent / connected failures (BASELINE config 5 shape).

Flow per failed vertex, as the reference runs it:
  * responders answer a DeterminantRequestEvent with the logs of the failed vertex they hold
    (JobCausalLogImpl.respondToDeterminantRequest :188-204 -> getDeterminants(startEpoch));
    different responders hold different lengths of the same log;
  * responses travel as DeterminantResponseEvent bytes (:93-125) and the failed task
    accumulates them (WaitingDeterminantsState :57, :102 -> merge :128-148);
  * ReplayingState decodes the main log for LogReplayerImpl and turns each subpartition
    recovery buffer into a BufferBuilt size list (:108-214).
Checked against the CPU oracle (oracle/response_ref.py + the C++ decodeNext oracle):
merged bytes, the decoded main-log SoA and the size lists bit-exact, and per-subpartition
error status / offset / tag for corrupt buffers.  The responders' logs are engine logs in
HBM that went through checkpoint truncation first (config 5: truncate on all logs).
"""
import os
import struct
import sys

import numpy as np
import pytest

import _oracle as O
from clonos_amd import CausalLogID, Engine, job, synth
from clonos_amd import _lib
from clonos_amd.replay import DeterminantResponseEvent, accumulate, prepare_replay

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "oracle"))
import response_ref as R  # noqa: E402  (checker)

pytestmark = pytest.mark.gpu


def _bb(rng, n):
    return b"".join(b"\x07" + struct.pack(">i", int(x)) for x in rng.integers(1, 1 << 20, n))


def _rid(lid: CausalLogID) -> R.LogId:
    if lid.is_main:
        return R.LogId.main(lid.vertex_id)
    return R.LogId.subpartition(lid.vertex_id, lid.irp_lower, lid.irp_upper, lid.subpartition)


def _check_main(main, span, want: bytes):
    st, r, _, _ = O.decode(want)
    assert st == 0
    sl = main.span_slice(span)
    np.testing.assert_array_equal(main.tag[sl], r["tag"])
    np.testing.assert_array_equal(main.v0[sl], r["v0"])
    np.testing.assert_array_equal(main.off[sl], r["off"])
    wsel = (main.w_idx >= sl.start) & (main.w_idx < sl.stop)
    np.testing.assert_array_equal(main.w_idx[wsel] - sl.start, r["w_idx"])
    np.testing.assert_array_equal(main.w_rc[wsel], r["w_rc"])


def _failed_vertices(graph, rng, k=16):
    """16 failed subtasks spread over the stages, including connected (adjacent-stage) pairs."""
    ids = [vid for _, _, vid in graph.all_vertex_ids()]
    p = graph.vertices[0].parallelism
    pairs = [(s * p + int(rng.integers(0, p)), (s + 1) * p + int(rng.integers(0, p))) for s in range(4)]
    out = sorted({v for pr in pairs for v in pr})
    rest = [v for v in ids if v not in out]
    out += [int(x) for x in rng.choice(rest, size=k - len(out), replace=False)]
    return out


def test_config5_replay_prep_after_truncation():
    rng = np.random.default_rng(0xC1050005)
    graph = job.dag(5, 8)
    failed = _failed_vertices(graph, rng)
    n_sub = 4
    with Engine(segment_bytes=4096, pool_segments=8192, timing=True) as eng:
        # the responders' copies: engine logs with epochs 0..2, truncated at checkpoint 1
        copies = {}  # failed vertex -> list of (responder, {CausalLogID: bytes})
        table = {}
        for v in failed:
            subs = [CausalLogID.sub(v, 1000 + v, 7, j) for j in range(n_sub)]
            table[v] = subs
            copies[v] = []
            for r in range(int(rng.integers(2, 4))):
                held = {}
                for lid in [CausalLogID.main(v)] + subs:
                    log = eng.open_log(CausalLogID(lid.vertex_id + 2000 * (r + 1), lid.is_main, lid.irp_lower,
                                                   lid.irp_upper, lid.subpartition))
                    for ep in range(3):
                        n = int(rng.integers(0, 1500))
                        data = synth.config3_epoch(n, rng, ep)[0].tobytes() if lid.is_main else _bb(rng, n)
                        if data:
                            log.appendDeterminant(data, ep)
                    held[lid] = log
                copies[v].append(held)
        assert eng.truncate_all(1)
        # responses (found unless the responder is beyond the sharing depth)
        wires = {}
        for v in failed:
            wires[v] = []
            for r, held in enumerate(copies[v]):
                found = r != 1 or rng.random() < 0.5
                ev = DeterminantResponseEvent(found, v, int(rng.integers(0, 1 << 62)))
                if found:
                    for lid, log in held.items():
                        if lid.is_main or rng.random() < 0.8:  # a responder may lack some logs
                            ev.put(lid, log.getDeterminants(int(rng.integers(1, 3))))
                wires[v].append(ev.write())
        # GPU replay preparation over all 16 vertices in one batch
        jobs = []
        for v in failed:
            acc = accumulate(v, [DeterminantResponseEvent.read(w)[0] for w in wires[v]])
            jobs.append((v, acc, table[v]))
        main, res = prepare_replay(eng, jobs)
        stats = eng.kernel_stats()
    for i, v in enumerate(failed):
        acc_o = R.accumulate(v, wires[v])
        assert jobs[i][1].write() == acc_o.write()
        spans = R.replay_spans(acc_o, v, [_rid(s) for s in table[v]])
        _check_main(main, i, spans[0])
        assert res[i].vertex_id == v
        for j, sp in enumerate(res[i].subpartitions):
            want = R.buffer_sizes(spans[1 + j])
            assert sp.status == _lib.CLG_OK
            np.testing.assert_array_equal(sp.buffer_sizes, np.array(want, np.int32))
    assert stats["replay_bufsizes"]["launches"] == 1


@pytest.mark.parametrize("case", ["order_inside", "truncated_tail", "corrupt_tag", "bad_enum", "empty", "absent"])
def test_subpartition_buffer_errors(case):
    rng = np.random.default_rng(5)
    good = _bb(rng, 3000)
    k = 1234 * 5
    buf = {
        "order_inside": good[:k] + b"\x00\x02" + good[k:],
        "truncated_tail": good + b"\x07\x00\x01",
        "corrupt_tag": good[:k] + b"\x09" + good[k:],
        "bad_enum": good[:k] + b"\x04" + struct.pack(">iqb", 1, 2, 9) + good[k:],
        "empty": b"",
        "absent": None,
    }[case]
    v = 3
    sub = CausalLogID.sub(v, 11, 12, 0)
    ev = DeterminantResponseEvent(True, v)
    ev.put(CausalLogID.main(v), synth.config2_log(500, rng)[0].tobytes())
    if buf is not None:
        ev.put(sub, buf)
    ev.put(CausalLogID.sub(v, 11, 12, 1), good)
    with Engine(segment_bytes=16384, pool_segments=64) as eng:
        main, res = prepare_replay(eng, [(v, accumulate(v, [ev]), [sub, CausalLogID.sub(v, 11, 12, 1)])])
    sp, other = res[0].subpartitions
    assert other.status == _lib.CLG_OK and len(other.buffer_sizes) == 3000
    if buf is None or buf == b"":
        assert sp.status == _lib.CLG_OK and len(sp.buffer_sizes) == 0
        return
    try:
        want = R.buffer_sizes(buf)
        want_err = None
    except ValueError as e:
        want_err, want = e.args
    np.testing.assert_array_equal(sp.buffer_sizes, np.array(want, np.int32))
    assert want_err is not None
    st, off, tag = want_err
    assert (sp.status, sp.err_off, sp.err_tag) == (st, off, tag)
