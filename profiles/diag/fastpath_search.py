#!/usr/bin/env python3
"""profiles/diag/fastpath_search.py -- looks for extensions on which the
round-5 local-mode fast path (k_dp dp_ungapped + ungapped_wide, restated
below) accepts a cell that the full banded DP (og_mapper.c dp_extend,
restated below) beats, and writes them as GPU probe fixtures
(tests/golden/fastpath_two_diagonal.json: read, quality, reference, centre)
for tests/test_gpu_fastpath.py.  Also restates round 6's bound, which must
reject every such case.  CPU only; a development tool, not the product.

    python3 profiles/diag/fastpath_search.py [n_tries] [out.json]
"""
import json
import sys

import numpy as np

MA, GMIN, OE, EX, GBAR, NPEN, HALF = 2, 13, 13, 3, 4, 1, 15


def pen(q):
    q = min(max(ord(q) - 33, 0), 40)
    return 2 + q // 10


def scores(rd, pens, g, c0, m):
    """s[i, k] for lanes k = 0 .. 2*HALF (diagonal c0 - HALF + k)."""
    W = 2 * HALF + 1
    s = np.empty((m, W), dtype=np.int64)
    for k in range(W):
        j = np.arange(m) + c0 - HALF + k
        gg = np.where((j >= 0) & (j < len(g)), g[np.clip(j, 0, len(g) - 1)], 4)
        amb = (rd > 3) | (gg > 3)
        s[:, k] = np.where(amb, -NPEN, np.where(rd == gg, MA, -pens))
    return s


def full_dp(s, m):
    """og_mapper.c dp_extend, local mode: (best, row, lane)."""
    W = s.shape[1]
    NEG = -(1 << 29)
    Hp = np.zeros(W, dtype=np.int64)
    Ep = np.full(W, NEG, dtype=np.int64)
    best, bi, bk = NEG, -1, -1
    for i in range(m):
        gap_ok = GBAR <= i < m - GBAR
        Hd = Hp + s[i]
        E = np.full(W, NEG, dtype=np.int64)
        if gap_ok:
            E[:-1] = np.maximum(Ep[1:] - EX, Hp[1:] - OE)
        H1 = np.maximum(np.maximum(Hd, E), 0)
        H = np.empty(W, dtype=np.int64)
        F = NEG
        for k in range(W):
            if gap_ok and k > 0:
                F = max(F - EX, H[k - 1] - OE)
            else:
                F = NEG
            H[k] = max(H1[k], F)
            if H[k] > best:
                best, bi, bk = int(H[k]), i, k
        Hp, Ep = H, E
    return best, bi, bk


def nonmatch(s):
    return s != MA


def fast_path(s, m, wide_rule):
    """dp_ungapped (local): (S, istar) if accepted, else None."""
    kb = HALF
    nmr = nonmatch(s[:, kb])
    nm = int(nmr.sum())
    gb_max = MA * m - GMIN
    wide = nm <= 3
    if MA * (m - nm) <= gb_max and not wide:
        return None
    P = np.cumsum(s[:, kb])
    mins = np.minimum.accumulate(np.minimum(P, 0))
    H = P - mins
    S = int(H.max())
    istar = int(np.argmax(H))
    crude = S > gb_max
    if not crude and not wide:
        return None
    if S <= 0:
        return None
    for k in range(s.shape[1]):
        if k != kb and MA * (m - int(nonmatch(s[:, k]).sum())) >= S:
            return None
    z = [r for r in range(istar + 1) if H[r] == 0]
    istop = z[-1] if z else -1
    lo = istop if istop > 0 else 0
    bad = any(r >= GBAR and H[r] < MA * (r + 1) - GMIN for r in range(lo, istar + 1))
    if not crude or bad:
        if not wide or not wide_rule(s, m, nm):
            return None
    return S, istar


def _runs(s, nm):
    kb = HALF
    xs = [int(x) for x in np.flatnonzero(nonmatch(s[:, kb]))[:nm]]
    es = [MA - int(s[x, kb]) for x in xs]
    return xs, es


def wide_r05(s, m, nm):
    xs, es = _runs(s, nm)
    if any(e >= GMIN for e in es) or sum(es) >= 2 * GMIN:
        return False
    if nm <= 1:
        return True
    x0, x1, xl = xs[0], xs[1], xs[-1]
    for k in range(s.shape[1]):
        if k == HALF:
            continue
        nk = nonmatch(s[:, k])
        c1 = int(nk[x0 + 1:x1].sum())
        c2 = int(nk[x1 + 1:xl].sum()) if nm == 3 else 0
        d = abs(k - HALF)
        gc = OE + EX * (d - 1)
        if es[0] + es[1] - MA * c1 >= gc:
            return False
        if nm == 3 and (es[1] + es[2] - MA * c2 >= gc or sum(es) - MA * (c1 + c2) >= gc):
            return False
    return True


def wide_r06(s, m, nm):
    xs, es = _runs(s, nm)
    if any(e >= GMIN for e in es) or sum(es) >= 2 * GMIN:
        return False
    if nm <= 1:
        return True
    if not wide_r05(s, m, nm):      # shape (i), unchanged
        return False
    runs = [(xs[0], xs[1], -1, es[0] + es[1])]
    if nm == 3:
        runs += [(xs[1], xs[2], -1, es[1] + es[2]), (xs[0], xs[2], xs[1], sum(es))]
    for lo, hi, ex, esum in runs:
        R = esum - GMIN
        if R < 0:
            continue
        n = R // MA + 1
        fmax, gmin_ = -1, 1 << 30
        for k in range(s.shape[1]):
            if k == HALF:
                continue
            rows = [r for r in range(lo + 1, hi) if r != ex and s[r, k] != MA]
            f = rows[n - 1] if len(rows) >= n else hi
            g = rows[-n] if len(rows) >= n else lo
            fmax, gmin_ = max(fmax, f), min(gmin_, g)
        if gmin_ < fmax:
            return False
    return True


def candidate(rng):
    """A read that sits on diagonal +a up to row c and on +b after it, over a
    reference whose stretches are periodic with those shifts' periods, with
    the seeded diagonal (0) crossing both with a few non-matches."""
    m = int(rng.choice([100, 150, 251]))
    a, b = 0, 0
    while a == b:
        a, b = (int(x) for x in rng.integers(-7, 8, 2))
    c = int(rng.integers(25, m - 25))
    pa = abs(a) if a else int(rng.integers(1, 4))
    pb = abs(b) if b else int(rng.integers(1, 4))
    ua = rng.integers(0, 4, pa)
    ub = rng.integers(0, 4, pb)
    r = np.empty(m, dtype=np.int64)
    r[:c + 1] = np.resize(ua, c + 1)
    r[c + 1:] = np.resize(ub, m - c - 1)
    # the reference along diagonal 0 is the read, except where the two legs'
    # shifts disagree with it; then a few random substitutions
    L = m + 40
    g = rng.integers(0, 4, L)
    off = 20
    g[off:off + m] = r
    for i in range(c + 1):
        j = off + i + a
        if 0 <= j < L:
            g[j] = r[i]
    for i in range(c + 1, m):
        j = off + i + b
        if 0 <= j < L:
            g[j] = r[i]
    for _ in range(int(rng.integers(0, 3))):
        j = int(rng.integers(0, L))
        g[j] = (g[j] + 1 + int(rng.integers(0, 3))) % 4
    q = ''.join(rng.choice(list('I5'), size=m))
    return r, q, g, off


def main(n_tries=20000, out=None):
    rng = np.random.default_rng(7)
    found = []
    accepted = kept = 0
    for t in range(n_tries):
        r, q, g, c0 = candidate(rng)
        m = len(r)
        pens = np.array([pen(x) for x in q])
        s = scores(r, pens, g, c0, m)
        acc = fast_path(s, m, wide_r05)
        if acc is None:
            continue
        accepted += 1
        kept += fast_path(s, m, wide_r06) is not None
        best, bi, bk = full_dp(s, m)
        if (best, bi, bk) != (acc[0], acc[1], HALF):
            new = fast_path(s, m, wide_r06)
            found.append(dict(read=''.join('ACGT'[x] for x in r), qual=q,
                              ref=''.join('ACGT'[x] for x in g), centre=c0,
                              r05=[acc[0], acc[1], HALF], full=[best, bi, bk],
                              r06_accepts=new is not None))
            print('case', len(found), 'try', t, 'fast', acc, 'full', (best, bi, bk), 'r06 accepts', new is not None,
                  flush=True)
            if len(found) >= 40:
                break
    print('tries', t + 1, 'accepted by r05', accepted, 'still accepted by r06', kept, 'r05 wrong', len(found))
    if out:
        with open(out, 'w') as f:
            json.dump({'generator': 'profiles/diag/fastpath_search.py', 'cases': found}, f, indent=0)


if __name__ == '__main__':
    main(int(sys.argv[1]) if len(sys.argv) > 1 else 20000, sys.argv[2] if len(sys.argv) > 2 else None)
