"""Generate tests/golden/inflight_ops.json (run from the repo root:
`python tests/golden/make_inflight_golden.py`).  Test infrastructure only.

Operation scripts over in-flight logs (log / notifyCheckpointComplete / replay batches) with
the results of oracle/inflight_ref.py, a literal simulation of
InMemorySubpartitionInFlightLogger + ReplayIterator (pinned by InFlightLogTest.
iteratorCountTest).  tests/test_golden.py re-derives them from the oracle and
tests/test_gpu_golden.py checks the engine against the committed bytes.
"""
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(HERE)), "oracle"))
from inflight_ref import InFlightLogRef  # noqa: E402


def run_script(ops, n_sub):
    refs = [InFlightLogRef() for _ in range(n_sub)]
    out = []
    for op in ops:
        if op[0] == "log":
            refs[op[1]].log(bytes.fromhex(op[3]), op[2])
        elif op[0] == "cp":
            refs[op[1]].notify_checkpoint_complete(op[2])
        else:
            res = []
            for sub, start, ign in op[1]:
                st, bufs, rem, eps, end = refs[sub].replay_full(start, ign)
                res.append([st, [b.hex() for b in bufs], rem if st != "state" else None, eps, end])
            out.append(res)
    return out


def make_case(seed, n_sub=4, rounds=6):
    rng = np.random.default_rng(0xF4 + seed)
    ops = []
    for e in range(rounds):
        for s in range(n_sub):
            if rng.random() < 0.35:
                continue  # this subpartition sends nothing in epoch e: a gap
            for _ in range(int(rng.integers(1, 6))):
                n = int(rng.choice([0, 1, 7, 16, 63, 64, 65, 200]))
                ops.append(["log", s, e, rng.integers(0, 256, n, dtype=np.uint8).tobytes().hex()])
        if e in (2, 4):
            for s in range(n_sub):
                ops.append(["cp", s, e - 1])
        reqs = [[s, int(rng.integers(max(0, e - 3), e + 2)), int(rng.integers(0, 3)) * int(rng.random() < 0.5)] for s in range(n_sub)
                for _ in range(2)]
        ops.append(["replay", reqs])
    # every start epoch of every subpartition, without and with a skip (covers the gaps)
    ops.append(["replay", [[s, st, ign] for s in range(n_sub) for st in range(rounds + 1) for ign in (0, 1)]])
    return {"seed": seed, "n_sub": n_sub, "ops": ops, "expect": run_script(ops, n_sub)}


if __name__ == "__main__":
    cases = [make_case(s) for s in range(6)]
    with open(os.path.join(HERE, "inflight_ops.json"), "w") as f:
        json.dump({"generator": "tests/golden/make_inflight_golden.py", "segment_bytes": 64, "cases": cases}, f)
    print(sum(len(c["ops"]) for c in cases), "ops")
