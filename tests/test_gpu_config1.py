"""GPU: BASELINE config 1 -- WordCount + causal TimeService / processing-time window,
parallelism 4, sharing depth 1, one epoch (modelled from the reference's producer call
sites, synth.config1_job; a JVM MiniCluster capture cannot run here).

Per task the engine holds its main log and one subpartition log per downstream subtask.
With depth 1 every consumer receives exactly its direct producers' logs
(AbstractDeltaSerializerDeserializer.java:165-194, JobCausalLogImpl.java:125-169) and,
with the Flat strategy, every shared log on every output channel
(FlatDeltaSerializerDeserializer.java:57-90).  Checked against the CPU oracle: every
(channel, log) delta of the epoch (two rounds, so the second sees only the new bytes),
the consumers' replicas after processUpstreamDelta, and the batched decode of all logs.
"""
import numpy as np
import pytest

import _oracle as O
from clonos_amd import CausalLogID, Engine, job, synth

pytestmark = pytest.mark.gpu


def test_config1_wordcount_depth1():
    rng = np.random.default_rng(synth.SEED_CONFIG1)
    graph, data = synth.config1_job(rng)
    depth = 1
    with Engine(segment_bytes=16384, pool_segments=4096, sharing_depth=depth) as eng, \
            Engine(segment_bytes=16384, pool_segments=4096, sharing_depth=depth) as down:
        logs = {lid: eng.open_log(lid) for lid in data}
        refs = {lid: O.OracleLog(16384, depth) for lid in data}
        # the epoch arrives in two halves (record boundaries), sliced after each
        cuts = {}
        for lid, b in data.items():
            st, r, _, _ = O.decode(b)
            assert st == 0
            k = int(r["off"][len(r["off"]) // 2]) if len(r["off"]) else 0
            cuts[lid] = (b[:k], b[k:])
        replicas = {}
        for half in range(2):
            for lid in data:
                part = cuts[lid][half]
                if part:
                    logs[lid].appendDeterminant(part, 0)
                    assert refs[lid].append(0, part) == 0
            # every producer -> consumer channel carries all of the producer's shared logs
            reqs, expect = [], []
            for prod, cons in (("source", "window"), ("window", "sink")):
                assert graph.distances(cons)[graph.vertex_id(prod, 0)] == -1
                assert job.shares_upstream_log(-1, depth) is False  # consumers do not re-share them
                for p in graph.vertex_ids(prod):
                    for c in graph.vertex_ids(cons):
                        ch = (p << 16 | c, 0xC1)
                        for lid in data:
                            if lid.vertex_id == p:
                                reqs.append((logs[lid], ch, 0, lid, c))
            res, out, _ = eng.slice_batch([(l, ch, ep) for l, ch, ep, _, _ in reqs])
            for (st, has, ofe, n, oo), (l, ch, ep, lid, c) in zip(res, reqs):
                st2, has2 = refs[lid].has_delta(ch, ep)
                assert st == st2 == 0 and has == has2
                if not has:
                    continue
                assert ofe == refs[lid].offset(ch)[1]
                d = out[oo:oo + n].tobytes()
                assert d == refs[lid].get_delta(ch, ep)[1]
                # the consumer's replica of the producer log (one per consuming subtask)
                key = (lid, c)
                if key not in replicas:
                    replicas[key] = down.open_log(CausalLogID(lid.vertex_id + 1000 * (c + 1), lid.is_main,
                                                              lid.irp_lower, lid.irp_upper, lid.subpartition))
                replicas[key].processUpstreamDelta(d, ofe, ep)
        for (lid, c), rep in replicas.items():
            assert rep.getDeterminants(0) == data[lid]
        # batched decode of every log (main logs: LogReplayer order; subpartitions: BufferBuilt sizes)
        lids = list(data)
        dec = eng.decode_logs([logs[l] for l in lids], [0] * len(lids))
        for s, lid in enumerate(lids):
            st, r, _, _ = O.decode(data[lid])
            sl = dec.span_slice(s)
            np.testing.assert_array_equal(dec.tag[sl], r["tag"])
            np.testing.assert_array_equal(dec.v0[sl], r["v0"])
            np.testing.assert_array_equal(dec.off[sl], r["off"])
            if not lid.is_main:
                assert (dec.tag[sl] == 7).all()
