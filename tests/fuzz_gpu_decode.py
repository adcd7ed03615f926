"""GPU decode fuzzer (a checker, run by hand on a GPU box; not collected by pytest):
random batches of spans -- every tag, Serializable streams, long records, zero runs, dense
short strings, byte flips that make decode errors -- decoded by the engine (auto, the three-pass path, the one-pass
decode forced (CLONOS_ONE_PASS=2) and the robust pipeline alone), and the same bytes as logs in 4 KiB HBM segments delivered over a few
epochs (decode_logs from a random start epoch), compared with the C++ oracle's decodeNext
loop span by span: bit-exact records, or the lowest failing span's (status, offset, tag).  Prints one JSON line per
round; stops at the first mismatch with its seed.
usage: python tests/fuzz_gpu_decode.py [--minutes M] [--seed S]"""
import argparse
import json
import os
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
sys.path.insert(0, os.path.dirname(HERE))
import torch  # noqa: E402,F401
import _oracle as O  # noqa: E402
from clonos_amd import ClonosError, Engine, synth  # noqa: E402
from clonos_amd import determinants as D  # noqa: E402
from test_gpu_decode import assert_span_equal  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--minutes", type=float, default=5.0)
ap.add_argument("--seed", type=int, default=1)
args = ap.parse_args()


def flat_mutant(rng):
    """A Serializable record of one of the flat shapes the inline parsers measure, mutated where
    those parsers decide: a byte of the stream flipped or replaced by a grammar code (TC_NULL,
    TC_CLASSDESC, TC_ENDBLOCKDATA, a field typecode), or the stream cut short."""
    s = bytearray(rng.choice([D.jser_boolean(True), D.jser_integer(int(rng.integers(-99, 99))),
                              D.jser_long(int(rng.integers(0, 1 << 40))), D.jser_string("s" * int(rng.integers(0, 20)))]))
    op = int(rng.integers(0, 3))
    q = int(rng.integers(4, len(s)))
    if op == 0:
        s[q] = int(rng.integers(0, 256))
    elif op == 1:
        s[q] = int(rng.choice([0x70, 0x71, 0x72, 0x73, 0x74, 0x78, ord("I"), ord("Z"), ord("J"), ord("["), 0x00, 0x01, 0x02]))
    else:
        s = s[:q]
    return D.encode(D.SerializableDeterminant(bytes(s)))


def span_bytes(rng):
    k = int(rng.integers(0, 11))
    if k == 0:
        return b""
    if k == 10:  # mutated flat Serializable shapes among ordinary records
        return b"".join(flat_mutant(rng) if rng.random() < 0.2 else
                        D.encode(synth.random_determinant(rng, allow_serializable=False))
                        for _ in range(int(rng.integers(1, 200))))
    if k <= 4:
        return synth.random_log(int(rng.integers(1, 3000)), rng)
    if k == 5:  # config-3 epoch piece
        return synth.config3_epoch(int(rng.integers(100, 20000)), rng)[0].tobytes()
    if k == 6:  # a long record inside ordinary ones
        a = synth.random_log(int(rng.integers(0, 400)), rng)
        n = int(rng.integers(100, 40000))
        rec = D.encode(D.TimerTriggerDeterminant(1, 2, D.INTERNAL, b"N" * n)) if rng.random() < 0.5 else \
            D.encode(D.SerializableDeterminant(D.jser_string("s" * n)))
        return a + rec + synth.random_log(int(rng.integers(0, 400)), rng)
    if k == 7:  # a zero run (channel-0 Order records), either parity
        lead = D.encode(D.TimestampDeterminant(5)) if rng.random() < 0.5 else b""
        return lead + D.encode(D.OrderDeterminant(0)) * int(rng.integers(100, 40000))
    if k == 8:  # dense short Serializable strings / nulls
        recs = [D.encode(D.SerializableDeterminant(D.jser_string("s" * int(rng.integers(0, 13))) if rng.random() < 0.7
                                                   else D.jser_null())) for _ in range(int(rng.integers(10, 6000)))]
        return b"".join(recs)
    return synth.config2_log(int(rng.integers(1, 30000)), rng)[0].tobytes()


def corrupt(b, rng):
    """A few byte flips (a decode error, or valid different records)."""
    if not b:
        return b
    a = bytearray(b)
    for _ in range(int(rng.integers(1, 4))):
        a[int(rng.integers(0, len(a)))] = int(rng.integers(0, 256))
    return bytes(a)


def check(eng, spans):
    blob, sp = b"", []
    for b in spans:
        pad = bytes(int(np.random.default_rng(len(blob)).integers(0, 3)))
        blob += pad
        sp.append((len(blob), len(b)))
        blob += b
    errs = [(s, O.decode(b)) for s, b in enumerate(spans)]
    bad = [(s, r) for s, r in errs if r[0] != 0]
    try:
        dec = eng.decode_host(blob, sp)
    except ClonosError as e:
        if not bad:
            return f"unexpected error {e.status} span {e.err_span} off {e.err_off}"
        s, (st, _, eo, et) = bad[0]
        if (e.status, e.err_span, e.err_off, e.err_tag) != (st, s, eo, et):
            return f"error {(e.status, e.err_span, e.err_off, e.err_tag)} != oracle {(st, s, eo, et)}"
        return None
    if bad:
        return f"no error, oracle has span {bad[0][0]} status {bad[0][1][0]}"
    for s, b in enumerate(spans):
        assert_span_equal(dec, s, b)
    return None


def check_logs(eng, spans, rng):
    """The spans as logs in HBM segments (each delivered as upstream deltas over a few epochs),
    decoded from a random start epoch: each log's getDeterminants(start) against the oracle."""
    from clonos_amd import CausalLogID
    logs, start, want = [], [], []
    for i, b in enumerate(spans):
        l = eng.open_log(CausalLogID.main(i % 30000))
        n_ep = int(rng.integers(1, 4))
        cuts = sorted(int(x) for x in rng.integers(0, len(b) + 1, n_ep - 1)) if len(b) else [0] * (n_ep - 1)
        bounds = [0] + cuts + [len(b)]
        for e in range(n_ep):
            part = b[bounds[e]:bounds[e + 1]]
            if part:
                l.processUpstreamDelta(part, 0, e)
        logs.append(l)
        start.append(int(rng.integers(0, n_ep)))
        want.append(l.getDeterminants(start[-1]))
    try:
        errs = [(s, O.decode(b)) for s, b in enumerate(want)]
        bad = [(s, r) for s, r in errs if r[0] != 0]
        try:
            dec = eng.decode_logs(logs, start)
        except ClonosError as e:
            if not bad:
                return f"logs: unexpected error {e.status} span {e.err_span}"
            s, (st, _, eo, et) = bad[0]
            if (e.status, e.err_span, e.err_off, e.err_tag) != (st, s, eo, et):
                return f"logs: error {(e.status, e.err_span, e.err_off, e.err_tag)} != oracle {(st, s, eo, et)}"
            return None
        if bad:
            return "logs: no error, the oracle has one"
        for s, b in enumerate(want):
            assert_span_equal(dec, s, b)
        return None
    finally:
        for l in logs:
            l.close()


rng0 = np.random.default_rng(args.seed)
engines = {"auto": Engine(segment_bytes=16384, pool_segments=1 << 15, timing=True),
           "three_pass": Engine(segment_bytes=16384, pool_segments=1 << 15, timing=True, decode="three_pass"),
           "robust": Engine(segment_bytes=16384, pool_segments=1 << 15, timing=True, decode="robust")}
os.environ["CLONOS_ONE_PASS"] = "2"  # (read when an engine opens: the one-pass decode on every batch it may take)
engines["one_pass"] = Engine(segment_bytes=16384, pool_segments=1 << 15, timing=True, decode="three_pass")
del os.environ["CLONOS_ONE_PASS"]
log_eng = Engine(segment_bytes=4096, pool_segments=1 << 19, timing=True)  # logs over 4 KiB segments
t_end = time.time() + args.minutes * 60
rnd = 0
while time.time() < t_end:
    seed = int(rng0.integers(0, 2**31))
    rng = np.random.default_rng(seed)
    n = int(rng.integers(1, 60)) if rng.random() < 0.8 else int(rng.integers(60, 400))
    spans = [span_bytes(rng) for _ in range(n)]
    if rng.random() < 0.3:
        for s in rng.choice(n, int(rng.integers(1, min(n, 4) + 1)), replace=False):
            spans[int(s)] = corrupt(spans[int(s)], rng)
    for name, eng in engines.items():
        try:
            msg = check(eng, spans)
        except AssertionError as e:
            msg = f"records differ: {str(e)[:300]}"
        if msg:
            print(json.dumps({"round": rnd, "seed": seed, "engine": name, "FAIL": msg}), flush=True)
            sys.exit(1)
    msg = check_logs(log_eng, spans, rng)
    if msg:
        print(json.dumps({"round": rnd, "seed": seed, "engine": "logs", "FAIL": msg}), flush=True)
        sys.exit(1)
    ks = engines["auto"].kernel_stats()
    paths = sorted(k for k in ks if k in ("decode_fallback", "decode_span_fallback", "decode_kept_errors",
                                          "decode_jser_retry", "decode_jser_grow", "decode_small"))
    engines["auto"].kernel_stats_reset()
    print(json.dumps({"round": rnd, "seed": seed, "spans": n, "bytes": sum(len(b) for b in spans), "ok": True,
                      "paths": paths}), flush=True)
    rnd += 1
for e in list(engines.values()) + [log_eng]:
    e.close()
print(json.dumps({"rounds": rnd, "ok": True}), flush=True)
