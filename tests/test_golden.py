"""CPU: the committed golden fixtures (tests/golden/, made by make_golden.py from the
oracle and cross-checked against the independent Python restatement) still hold for both
restatements.  Pins the oracle itself: a drift in either shows up here, not as a GPU
mismatch."""
import json
import os

import pytest

import _oracle as O
from _oracle import pyref

HERE = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
DECODE = json.load(open(os.path.join(HERE, "decode.json")))
LOG_OPS = json.load(open(os.path.join(HERE, "log_ops.json")))
FIELDS = ("off", "tag", "v0", "w_idx", "w_rc", "w_v1", "w_var_off", "w_var_len", "w_sub")


def expected(case, f):
    return [int(x) for x in case[f]]


@pytest.mark.parametrize("case", DECODE, ids=[c["name"] for c in DECODE])
def test_decode_fixture_oracle(case):
    buf = bytes.fromhex(case["hex"])
    st, r, eo, et = O.decode(buf)
    assert st == case["status"]
    if st:
        assert (eo, et) == (case["err_off"], case["err_tag"])
        return
    for f in FIELDS:
        assert r[f].tolist() == expected(case, f), f


@pytest.mark.parametrize("case", DECODE, ids=[c["name"] for c in DECODE])
def test_decode_fixture_pyref(case):
    buf = bytes.fromhex(case["hex"])
    if case["status"]:
        with pytest.raises(pyref.DecodeError) as ex:
            pyref.decode_all(buf)
        assert (ex.value.status, ex.value.off) == (case["status"], case["err_off"])
        return
    recs = pyref.decode_all(buf)
    assert [x["off"] for x in recs] == expected(case, "off")
    assert [x["tag"] for x in recs] == expected(case, "tag")
    assert [x["v0"] for x in recs] == expected(case, "v0")
    assert [i for i, x in enumerate(recs) if x["wide"]] == expected(case, "w_idx")


def run_script(log, script, consumer):
    """Replays a log_ops.json script through a ThreadCausalLog-like object; yields
    (op index, result list, state list, consumer states) per op."""
    for i, op in enumerate(script["ops"]):
        kind = op[0]
        if kind == "append":
            res = [log.append(op[1], bytes.fromhex(op[2]))]
        elif kind == "upstream":
            res = [log.upstream(bytes.fromhex(op[3]), op[2], op[1])]
        elif kind == "delta":
            ch, e = (op[1], op[2]), op[3]
            st, has = log.has_delta(ch, e)
            res = [st, int(has)]
            if st == 0 and has:
                res.append(log.offset(ch)[1])
                st2, d = log.get_delta(ch, e)
                res += [st2, d.hex()]
        elif kind == "epoch":
            res = [0]
        elif kind == "checkpoint":
            res = [log.checkpoint_complete(op[1])]
        elif kind == "determinants":
            st, d = log.get_determinants(op[1])
            res = [st, d.hex() if st == 0 else ""]
        else:
            res = [log.log_length()]
        s = log.state()
        yield i, res, [s["writer"], s["capacity"], s["n_components"], [list(e) for e in s["epochs"]]], \
            [consumer(log, c) for c in ((1, 9), (2, 9), (3, 9))]


@pytest.mark.parametrize("script", LOG_OPS, ids=[f"C{s['component']}_{i}" for i, s in enumerate(LOG_OPS)])
def test_log_fixture_oracle(script):
    log = O.OracleLog(script["component"])
    for i, res, state, cons in run_script(log, script, lambda lg, c: lg.consumer(c)):
        exp = script["expect"][i]
        assert res == exp["res"], (i, script["ops"][i])
        assert state == exp["state"], i
        assert [list(c) if c else None for c in cons] == [list(c) if c else None for c in exp["consumers"]], i
