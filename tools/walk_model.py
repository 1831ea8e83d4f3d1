#!/usr/bin/env python3
"""CPU model of the hot chains' allow walk (rl_hot.hpp `walk`, k_hot_summ's per-ms table,
k_hot_fill's walk verdicts) for ONE key's record stream, checked against the sequential
semantics (SlidingWindowRateLimiter.java:85-180, TokenBucketRateLimiter Lua :38-68) record by
record. It mirrors the device loop step for step (cursor chunk with up to 4 pending allows,
remaining-0 chunks, bursts, fifth allows, specials; the device's 64-ms table views are one
loop over ms here), so a logic error or a loop that does not end shows up here instead of on
the GPU (tests/test_walk_model.py runs it). Test tooling only: nothing in the product imports it.

usage: tools/walk_model.py [--algo sw|tb] [--n N] [--rate R] [--seed S] [--specials F]
"""
import argparse
import math
import random

INT64_MIN = -(1 << 63)


def d2l(d):
    if d != d:
        return 0
    return int(d)


# ---------------------------------------------------------------- exact single-key state
class SW:
    def __init__(self, mx, w):
        self.mx, self.w = mx, w
        self.b = {}                            # bucket start -> [count, expire_at]

    def copy(self):
        s = SW(self.mx, self.w)
        s.b = {k: list(v) for k, v in self.b.items()}
        return s

    def get(self, start, now):
        e = self.b.get(start)
        return e[0] if e and not (now > e[1]) else 0

    def est(self, t):
        w = self.w
        W = (t // w) * w
        curr, prev = self.get(W, t), self.get(W - w, t)
        pw = 1.0 - float(t % w) / float(w)
        return d2l(float(prev) * pw + float(curr))

    def pred(self, t, p):                     # an acquire of p allowed at t (:104)
        return self.est(t) + p <= self.mx

    def step(self, t, p, op=0):               # -> (allowed, remaining)
        w = self.w
        W = (t // w) * w
        if op == 2:                           # reset: DEL current and previous (:139-153)
            self.b.pop(W, None); self.b.pop(W - w, None)
            return 0, 0
        e = self.est(t)
        if op == 1 or e + p > self.mx:
            return 0, max(0, self.mx - e)
        c = self.get(W, t) + 1
        self.b[W] = [c, t + w]
        for k in [k for k in self.b if k < W - w]:
            del self.b[k]
        return int(c <= self.mx), max(0, self.mx - self.est(t))


class TB:
    def __init__(self, cap, rate_per_s, w):
        self.cap, self.rate, self.ttl = float(cap), rate_per_s / 1000.0, 2 * w
        self.s = None                          # (tokens, last)

    def copy(self):
        x = TB.__new__(TB)
        x.cap, x.rate, x.ttl, x.s = self.cap, self.rate, self.ttl, self.s
        return x

    def bal(self, t):
        if self.s is None or t > self.s[1] + self.ttl:
            return self.cap
        x = self.s[0] + float(t - self.s[1]) * self.rate
        return x if x < self.cap else self.cap

    def pred(self, t, p):
        return self.bal(t) >= p

    def step(self, t, p, op=0):
        if op == 2:
            self.s = None
            return 0, 0
        if p > self.cap:
            return 0, -1
        b = self.bal(t)
        if op == 1:
            return 0, d2l(b)
        if b >= p:
            b -= p
            self.s = (b, t)
            return 1, d2l(b)
        return 0, d2l(b)


# ---------------------------------------------------------------- the walk
def walk(recs, st0, algo, w, stats):
    """recs: [(t, p, op[, mine])] in arrival order — the walked key's records (mine, the
    default) among other keys' records (mine False: they only take their place in the
    region's 64-record chunks, as on the device). The key's times are non-decreasing.
    Returns the results [(allowed, remaining)] the walk + fill produce for the key's records
    (None for the others)."""
    recs = [r if len(r) == 4 else (r[0], r[1], r[2], True) for r in recs]
    n = len(recs)
    nch = (n + 63) // 64
    lo, hi = min(r[0] for r in recs), max(r[0] for r in recs)
    first1, first2 = {}, {}
    for j, (t, p, op, mine) in enumerate(recs):
        if mine and op == 0 and p == 1 and t not in first1:
            first1[t] = j
        if mine and op == 0 and p <= 2 and t not in first2:
            first2[t] = j
    special = [any(r[3] and r[2] != 0 for r in recs[c * 64:(c + 1) * 64]) for c in range(nch)]
    mxs = [max((r[0] for r in recs[c * 64:(c + 1) * 64] if r[3] and r[2] == 0), default=None)
           for c in range(nch)]
    res = [None] * n
    verdict = {}                               # chunk -> (state copy, allow offsets)
    S = st0

    def detail(c, S):
        for j in range(c * 64, min(n, c * 64 + 64)):
            t, p, op, mine = recs[j]
            if mine:
                res[j] = S.step(t, p, op)
        stats["detail"] += 1

    def plain_before(c):                       # the key's last plain acquire before chunk c
        return next((mxs[k] for k in range(c - 1, -1, -1) if mxs[k] is not None), None)

    def thresholds(S, W, C):                   # SW: T1(C), T2(C) in window W (thr_build)
        s = S.copy()
        # the state rolled into W with count C in the current bucket
        s.b = {k: v for k, v in s.b.items() if k >= W - w}
        if W - w in s.b and W not in s.b:
            pass
        s.b[W] = [C, W + w] if C else s.b.get(W, [0, W + w])
        if C == 0:
            s.b.pop(W, None)
        out = []
        for q in (1, 2):
            t = W
            while t < W + w and not s.pred(t, q):
                t += 1
            out.append(t)
        return out

    def rem0(c, tq1):                          # every acquire of chunk c is denied with remaining 0
        return mxs[c] is not None and (tq1 is None or mxs[c] < tq1)

    st = dict(cc=0, po=[], ts=lo, must=False, mlast=None, K=S.copy())

    def detail_at(c):                          # rl_hot.hpp walk: detail_at
        detail(c, S)
        if mxs[c] is not None:
            st["mlast"] = mxs[c]
        elif special[c]:
            st["mlast"] = plain_before(c)
        ml = st["mlast"]
        if special[c]:                         # a reset may grant more: search again
            st["ts"] = lo if ml is None else ml + 1
        elif ml is not None:
            st["ts"] = max(st["ts"], ml + 1)
        st["must"] = ml is not None and S.pred(ml, 1)
        st["cc"], st["K"], st["po"] = c + 1, S.copy(), []

    guard = 0
    while True:
        guard += 1
        assert guard < 10 * (nch + (hi - lo) + 100), "walk does not end"
        cc, po, ts = st["cc"], st["po"], st["ts"]
        if cc >= nch:
            break
        if not po and (st["must"] or special[cc]):
            st["must"] = False
            detail_at(cc)
            continue
        tf = None
        tq1 = None                             # the first ms >= ts the state grants (q >= 1)
        while ts <= hi:
            lim = hi
            if algo == "sw":
                W = (ts // w) * w
                C = S.get(W, ts)
                T1, T2 = thresholds(S, W, C)
                lim = min(lim, W + w - 1)
            for t in range(ts, lim + 1):
                if algo == "tb":
                    b = S.bal(t)
                    q = 2 if b >= 2 else 1 if b >= 1 else 0
                else:
                    q = 2 if t >= T2 else 1 if t >= T1 else 0
                if q >= 1 and tq1 is None:
                    tq1 = t
                cand = first2.get(t) if q >= 2 else first1.get(t) if q == 1 else None
                if cand is not None:
                    tf, rf = t, cand
                    pf = 2 if (q >= 2 and first1.get(t) != first2.get(t)) else 1
                    break
            if tf is not None:
                break
            ts = lim + 1
        st["ts"] = ts
        cs = nch - 1 if tf is None else rf // 64
        sp = next((c for c in range(cc + 1, cs + 1) if special[c]), None)
        if sp is not None:
            verdict[cc] = (st["K"].copy(), list(po), False)
            for c in range(cc + 1, sp):
                verdict[c] = (S.copy(), [], rem0(c, tq1))
            detail_at(sp)
            continue
        if tf is None:
            verdict[cc] = (st["K"].copy(), list(po), False)
            for c in range(cc + 1, nch):
                verdict[c] = (S.copy(), [], rem0(c, tq1))
            break
        if cs == cc and len(po) == 4:            # a fifth allow in the cursor chunk
            stats["conflict"] += 1
            S = st["K"].copy()
            detail_at(cc)
            continue
        assert cs >= cc, ("allow before the cursor", cs, cc)
        if cs > cc:
            verdict[cc] = (st["K"].copy(), list(po), False)
            for c in range(cc + 1, cs):
                verdict[c] = (S.copy(), [], rem0(c, tq1))
            st["cc"], st["K"], st["po"] = cs, S.copy(), []
        st["po"].append(rf % 64)
        a, _ = S.step(tf, pf)
        assert a == 1, "walk allow denied by the exact step"
        stats["allows"] += 1
        st["ts"] = tf + 1
        if S.pred(tf, 1):
            stats["burst"] += 1
            S = st["K"].copy()
            detail_at(st["cc"])
    # fill: the verdict chunks
    for c, (Sv, o, z) in verdict.items():
        s = Sv.copy()
        for j in range(c * 64, min(n, c * 64 + 64)):
            t, p, op, mine = recs[j]
            if not mine:
                continue
            assert op == 0
            if j - c * 64 in o:
                res[j] = s.step(t, p)
                assert res[j][0] == 1
            else:
                r = s.step(t, p)
                assert r[0] == 0 or (algo == "tb" and r[1] == -1), ("verdict chunk allows", c, j)
                if z:                          # a remaining-0 verdict (the fill writes 0 unread)
                    assert r[1] in (0, -1), ("rem-0 chunk with remaining", c, j, r)
                    stats["rem0"] = stats.get("rem0", 0) + 1
                res[j] = r
    return res


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--algo", default="sw")
    ap.add_argument("--n", type=int, default=20000)
    ap.add_argument("--per-ms", type=float, default=20.0)
    ap.add_argument("--seed", type=int, default=1)
    ap.add_argument("--specials", type=float, default=0.0)
    ap.add_argument("--pmax", type=int, default=2)
    a = ap.parse_args()
    rnd = random.Random(a.seed)
    t0 = 1_700_000_000_000
    span = int(a.n / a.per_ms)
    ts = sorted(t0 + rnd.randrange(span) for _ in range(a.n))
    recs = [(t, rnd.randint(1, a.pmax), (rnd.choice([1, 2]) if rnd.random() < a.specials else 0))
            for t in ts]
    if a.algo == "sw":
        mk = lambda: SW(100, 1000)
        w = 1000
    else:
        mk = lambda: TB(1000, 100.0, 60000)
        w = 60000
    want = []
    s = mk()
    for t, p, op in recs:
        want.append(s.step(t, p, op))
    stats = {"detail": 0, "allows": 0, "conflict": 0, "burst": 0}
    got = walk(recs, mk(), a.algo, w, stats)
    bad = [j for j in range(len(recs)) if got[j] != want[j]]
    print(a.algo, len(recs), "records:", stats, "mismatches", len(bad), bad[:5])
    if bad:
        j = bad[0]
        print("first", j, recs[j], "got", got[j], "want", want[j])


if __name__ == "__main__":
    main()
