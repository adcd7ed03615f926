"""Pure-Python model of the fused decode's chain logic (decode_fused.hip), for offline
checks of the speculation / merge / settle rules on real byte streams.  Developer tool,
not test infrastructure: it restates the KERNEL, not the reference."""
import sys

R, TILE, SPEC_MAX, CANON_LANES = 128, 8192, 256, 16
LUT = {0: 2, 1: 9, 2: 5, 6: 13, 7: 5}


def be32(b, a):
    v = (b[a] << 24) | (b[a + 1] << 16) | (b[a + 2] << 8) | b[a + 3]
    return v - (1 << 32) if v >= 1 << 31 else v


def s8(x):
    return x - 256 if x > 127 else x


def zlen(b, a, end):
    t = b[a]
    if t in LUT:
        return LUT[t] if a + LUT[t] <= end else -1
    avail = end - a
    if t == 4:
        if avail < 14 or not 0 <= s8(b[a + 13]) <= 6:
            return -1
        if s8(b[a + 13]) != 6:
            L = 14
        else:
            if avail < 18 or be32(b, a + 14) < 0:
                return -1
            L = 18 + be32(b, a + 14)
        return L if L <= avail else -1
    if t == 5:
        if avail < 23:
            return -1
        L = 23
        if b[a + 22] != 0:
            if avail < 27 or be32(b, a + 23) < 0:
                return -1
            L = 27 + be32(b, a + 23)
        if not 0 <= s8(b[a + 21]) <= 1:
            return -1
        return L if L <= avail else -1
    return -1  # 3 (Serializable: the kernel aborts) and > 7


def spec_step(b, q, end):
    L = zlen(b, q, end)
    return (q + L, True) if 0 < L <= SPEC_MAX else (q + 1, False)


WARM = 96


def spec_walk(b, ws, rs, re, end):
    q, bm, bad = ws, set(), 0
    while q < rs:
        nq, ok = spec_step(b, q, end)
        if not ok:
            bad = q + 1
        q = nq
    first = q
    while q < re:
        nq, ok = spec_step(b, q, end)
        if ok:
            bm.add(q)
        else:
            bad = q + 1
        q = nq
    return dict(bm=bm, exit=q, bad=bad, first=first)


def canon_walk(b, rs, re, end, e, s):
    if e >= re:
        return e
    p, q = e, s["first"]
    while True:
        if p == q:
            return s["exit"]
        if p >= re:
            return p
        if p < q:
            p = spec_step(b, p, end)[0]
        else:
            q = spec_step(b, q, end)[0]


def merge_walk(b, rs, re, end, e, s):
    """True chain from e until it lands on a speculative start past the last skip."""
    if e >= re:
        return dict(bm=set(), exit=e, bad=0)
    p, pb = e, set()
    while p < re:
        if p in s["bm"] and p >= s["bad"]:
            return dict(bm=pb | {x for x in s["bm"] if x >= p}, exit=s["exit"], bad=0)
        L = zlen(b, p, end)
        if L <= 0:
            return dict(bm=set(), exit=s["exit"], bad=1)
        pb.add(p)
        p += L
    return dict(bm=pb, exit=p, bad=0)


def decode_tile(b, lo, hi, end, first, e_true_fn):
    regs = []
    for l in range(64):
        r0 = l * R
        rs, re = min(max(r0, lo), hi), min(r0 + R, hi)
        ws = rs - WARM if rs >= lo + WARM else lo
        regs.append((rs, re, spec_walk(b, ws, rs, re, end) if rs < re else dict(bm=set(), exit=rs, bad=0, first=rs)))
    cx = [g[2]["exit"] for g in regs]
    last_l = (hi - 1) >> 7 if hi > lo else 0
    c0 = max(0, last_l - (CANON_LANES - 1))

    def mw(l, e):
        rs, re, sp = regs[l]
        return merge_walk(b, rs, re, end, e, sp) if rs < re else dict(bm=set(), exit=e, bad=0)

    ent = [None] * 64
    res = [None] * 64
    x_pub = None
    if not first:
        for _ in range(65):
            want = [None if l <= c0 else cx[l - 1] for l in range(64)]
            ch = [want[l] != ent[l] for l in range(64)]
            if not any(ch):
                break
            for l in range(64):
                if ch[l]:
                    rs, re, sp = regs[l]
                    ent[l] = want[l]
                    res[l] = mw(l, want[l])
                    cx[l] = canon_walk(b, rs, re, end, want[l], sp) if rs < re else want[l]
        x_pub = cx[63]
    e_true = e_true_fn(x_pub)
    spx = [g[2]["exit"] for g in regs]
    entry = list(ent)
    for l in range(64):
        if entry[l] is None:
            entry[l] = e_true if l == 0 else spx[l - 1]
            res[l] = mw(l, entry[l])
    for _ in range(65):
        want = [e_true] + [res[l - 1]["exit"] for l in range(1, 64)]
        ch = [want[l] != entry[l] for l in range(64)]
        if not any(ch):
            break
        for l in range(64):
            if ch[l]:
                entry[l] = want[l]
                res[l] = mw(l, want[l])
    return x_pub, res


def check_stream(buf, offs=None):
    """Decode a whole span tile by tile; returns (ok, reason, tile)."""
    b = list(buf) + [0] * 128
    n = len(buf)
    e_prev = 0
    starts = []
    for t0 in range(0, n, TILE):
        hi = min(TILE, n - t0)
        sub = b[t0:t0 + hi + 64] + [0] * 64
        first = t0 == 0
        x_pub, res = decode_tile(sub, 0, hi, n - t0, first, lambda xp: 0 if first else e_prev - t0)
        if any(r["bad"] for r in res):
            return False, "bad", t0 // TILE
        x_true = res[63]["exit"]
        if t0 + hi >= n:
            if x_true != n - t0:
                return False, "end", t0 // TILE
        elif not first and x_true != x_pub:
            return False, "exit", t0 // TILE
        for r in res:
            starts.extend(sorted(t0 + x for x in r["bm"]))
        e_prev = t0 + (x_pub if not first else x_true)
    if offs is not None and list(offs) != starts:
        return False, "starts", -1
    return True, None, None


if __name__ == "__main__":
    import numpy as np
    sys.path.insert(0, __file__.rsplit("/tools/", 1)[0])
    from clonos_amd import synth
    rng = np.random.default_rng(int(sys.argv[1]) if len(sys.argv) > 1 else 77)
    for i in range(int(sys.argv[2]) if len(sys.argv) > 2 else 2):
        buf, offs = synth.config2_log(200000, rng)
        print("config2", i, check_stream(buf.tolist(), offs.tolist()), flush=True)
        raw = synth.random_log(20000, rng, allow_serializable=False)
        st = []
        o = 0
        print("random", i, check_stream(list(raw)), flush=True)
