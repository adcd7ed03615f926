"""GPU: the engine reproduces the committed golden fixtures (tests/golden/) exactly --
every decode case through both decode paths (the `engine` fixture runs fast and robust),
and every ThreadCausalLogImpl op script through the HBM log."""
import json
import os

import numpy as np
import pytest

from clonos_amd import ClonosError, CausalLogID, Engine
from test_golden import DECODE, FIELDS, LOG_OPS, expected, run_script

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("case", DECODE, ids=[c["name"] for c in DECODE])
def test_decode_fixture_gpu(engine, case):
    buf = bytes.fromhex(case["hex"])
    if case["status"]:
        with pytest.raises(ClonosError) as ex:
            engine.decode_host(buf)
        assert (ex.value.status, ex.value.err_off, ex.value.err_tag) == (case["status"], case["err_off"],
                                                                         case["err_tag"])
        return
    dec = engine.decode_host(buf)
    got = dict(off=dec.off, tag=dec.tag, v0=dec.v0, w_idx=dec.w_idx, w_rc=dec.w_rc, w_v1=dec.w_v1,
               w_var_off=dec.w_var_off, w_var_len=dec.w_var_len, w_sub=dec.w_sub)
    for f in FIELDS:
        assert np.asarray(got[f]).tolist() == expected(case, f), f


class EngineLog:
    """The engine's ThreadCausalLog behind the oracle's status-returning interface."""

    def __init__(self, eng, vid):
        self.l = eng.open_log(CausalLogID.main(vid))

    @staticmethod
    def _st(fn, *a):
        try:
            return 0, fn(*a)
        except ClonosError as e:
            return e.status, None

    def append(self, epoch, data):
        return self._st(self.l.appendDeterminant, data, epoch)[0]

    def upstream(self, delta, off, epoch):
        return self._st(self.l.processUpstreamDelta, delta, off, epoch)[0]

    def has_delta(self, ch, e):
        st, v = self._st(self.l.hasDeltaForConsumer, ch, e)
        return st, bool(v) if st == 0 else False

    def offset(self, ch):
        return self._st(self.l.getOffsetFromEpochForConsumer, ch, 0)

    def get_delta(self, ch, e):
        st, d = self._st(self.l.getDeltaForConsumer, ch, e)
        return st, d or b""

    def get_determinants(self, e):
        st, d = self._st(self.l.getDeterminants, e)
        return st, d or b""

    def checkpoint_complete(self, cp):
        return self._st(self.l.notifyCheckpointComplete, cp)[0]

    def log_length(self):
        return self.l.logLength()

    def state(self):
        return self.l.state()


@pytest.mark.parametrize("script", LOG_OPS, ids=[f"C{s['component']}_{i}" for i, s in enumerate(LOG_OPS)])
def test_log_fixture_gpu(script):
    with Engine(segment_bytes=script["component"], pool_segments=(1 << 24) // script["component"]) as eng:
        log = EngineLog(eng, 1)
        for i, res, state, cons in run_script(log, script, lambda lg, c: lg.l.consumer_state(c)):
            exp = script["expect"][i]
            assert res == exp["res"], (i, script["ops"][i])
            assert state == exp["state"], i
            assert [list(c) if c else None for c in cons] == [list(c) if c else None for c in exp["consumers"]], i
