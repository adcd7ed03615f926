"""GPU: piggybacked causal-log deltas (clg_enrich_batch / clg_process_delta) == the
reference's Flat and Grouping serializers (AbstractDeltaSerializerDeserializer.java:89-163,
FlatDeltaSerializerDeserializer.java:57-120, GroupingDeltaSerializerDeserializer.java:66-165)
as restated in oracle/delta_ref.py over the C++ ThreadCausalLogImpl oracle.

Each round appends to every producer log, then builds the piggyback bytes for four output
channels in one batch (header bytes + deltas, byte-exact, including the Grouping
strategy's erased empty vertices / partitions and its post-hasDelta subpartition filter),
and a downstream engine applies channel 0's messages with processCausalLogDelta: its
replicas must equal the oracle's replicas.
"""
import os
import sys

import numpy as np
import pytest

import _oracle as O
from clonos_amd import CausalLogID, Engine
from clonos_amd import _lib
from clonos_amd import determinants as D
from clonos_amd import synth

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "oracle"))
import delta_ref as R  # noqa: E402  (checker)

pytestmark = pytest.mark.gpu


def _tuple(lid: CausalLogID):
    return (lid.vertex_id, lid.is_main, lid.irp_lower if not lid.is_main else 0,
            lid.irp_upper if not lid.is_main else 0, lid.subpartition if not lid.is_main else 0)


@pytest.mark.parametrize("strategy", [_lib.CLG_DELTA_FLAT, _lib.CLG_DELTA_HIERARCHICAL])
@pytest.mark.parametrize("seed", range(3))
def test_enrich_and_process_match_oracle(strategy, seed):
    rng = np.random.default_rng(500 + seed)
    comp = [256, 4096, 16384][seed]
    ids = []
    for v in (3, 7, 12):
        if v != 7:  # vertex 7 has no main log in the shared structure
            ids.append(CausalLogID.main(v))
        for part in range(2):
            for sub in range(3):
                ids.append(CausalLogID.sub(v, 1000 * v + part, 77, sub))
    with Engine(segment_bytes=comp, pool_segments=1 << 13) as up, \
            Engine(segment_bytes=comp, pool_segments=1 << 13) as down:
        logs = {l: up.open_log(l) for l in ids}
        refs = {l: O.OracleLog(comp) for l in ids}
        replicas = {}  # downstream oracle replicas (channel 0's consumer)
        chans = [(9, c) for c in range(4)]
        epoch = 0
        for rnd in range(4):
            for l in ids:
                if rng.random() < 0.6:
                    rec = b"".join(D.encode(synth.random_determinant(rng)) for _ in range(int(rng.integers(1, 80))))
                    logs[l].appendDeterminant(rec, epoch)
                    assert refs[l].append(epoch, rec) == 0
            sends = {(c, l): (l.is_main or strategy == _lib.CLG_DELTA_FLAT or rng.random() < 0.7)
                     for c in range(4) for l in ids}
            reqs = [(chans[c], epoch, [(logs[l], sends[(c, l)]) for l in ids]) for c in range(4)]
            got = up.enrich_batch(strategy, reqs)
            for c in range(4):
                want = R.serialize(strategy, [(refs[l], _tuple(l), sends[(c, l)]) for l in ids], chans[c], epoch)
                st, b = got[c]
                assert st == 0 and b == want, (rnd, c)
            # downstream: processCausalLogDelta of channel 0's message
            ep, handles, used = down.process_delta(strategy, got[0][1])
            assert ep == epoch and used == len(got[0][1])
            _, items = R.parse(strategy, got[0][1])
            assert len(handles) == len(items)
            for cid, off, d in items:
                r = replicas.setdefault(cid, O.OracleLog(comp))
                assert r.upstream(d, off, epoch) == 0
            if rnd % 2 == 1:
                epoch += 1
        for cid, r in replicas.items():
            lid = CausalLogID.main(cid[0]) if cid[1] else CausalLogID.sub(cid[0], cid[2], cid[3], cid[4])
            rep = down.get_log(lid)
            assert rep is not None
            for e in range(epoch + 1):
                st, want = r.get_determinants(e)
                assert rep.getDeterminants(e) == want


def test_process_delta_truncated():
    with Engine(segment_bytes=4096, pool_segments=64) as eng:
        msg = bytes.fromhex("00000017" "0000000000000001" "0003" "01" "00000000" "00000004") + b"\x00\x01\x00\x02"
        assert eng.process_delta(_lib.CLG_DELTA_FLAT, msg)[0] == 1
        for cut in (5, 14, 20, len(msg) - 1):
            with pytest.raises(_lib.ClonosError) as ei:
                eng.process_delta(_lib.CLG_DELTA_FLAT, msg[:cut])
            assert ei.value.status == _lib.CLG_E_TRUNCATED
