"""The exact ungapped fast path of k_dp (mh_map.hip dp_ungapped) against the
CPU oracle's full banded DP (og_mapper.c dp_extend): reads built to sit on
both sides of every bound the fast path relies on -- 0/1/2/3 mismatches at
every quality band and at the read ends, adjacent or a few rows apart, local clips, Ns, reference ends,
tandem repeats (other diagonals with few mismatches), indels, short and long
reads.  The launch must take both branches (fast path and full DP) and agree
with the oracle bit for bit."""
import numpy as np
import pytest

import oracle
from micall_amd import _native, projects

pytestmark = pytest.mark.gpu

SEEDS = projects.load_default().seed_sequences()
POL = SEEDS['HIV1B-pol-seed']
COMP = {'A': 'T', 'C': 'G', 'G': 'C', 'T': 'A', 'N': 'N'}


def _revcomp(s):
    return ''.join(COMP[c] for c in reversed(s))


def _reference():
    rng = np.random.default_rng(17)
    unit = 'ACGTTGCA'
    rep = unit * 40 + ''.join('ACGT'[x] for x in rng.integers(0, 4, 200)) + 'AAT' * 60
    return [POL, rep + POL[:400]]


def _cases():
    rng = np.random.default_rng(23)
    refs = _reference()
    seqs, quals = [], []

    def add(s, q):
        seqs.append(s)
        quals.append(q)

    def mutate(s, at):
        s = list(s)
        for p in at:
            s[p] = 'ACGT'[('ACGT'.index(s[p]) + 1 + int(rng.integers(0, 3))) % 4]
        return ''.join(s)

    qchars = ['#', '+', '5', '?', 'G', 'I']   # penalties 2..6
    for m in (251, 300, 150, 40, 17, 12, 512, 600):
        for _ in range(6):
            ref = refs[int(rng.integers(0, 2))] if m <= 600 else POL
            if len(ref) < m:
                ref = POL
            st = int(rng.integers(0, len(ref) - m + 1))
            base = ref[st:st + m]
            qc = qchars[int(rng.integers(0, len(qchars)))]
            q = qc * m
            add(base, q)                                    # exact
            for p in (0, 1, 3, 5, 6, 7, m // 2, m - 8, m - 6, m - 2, m - 1):
                if 0 <= p < m:
                    add(mutate(base, [p]), q)               # one mismatch
            for a, b in ((m // 3, 2 * m // 3), (2, m - 3), (5, 9), (m - 9, m - 5)):
                if 0 <= a < b < m:
                    for q2 in ('#', 'G'):
                        add(mutate(base, [a, b]), q2 * m)   # two mismatches
            add(mutate(base, list(range(10, min(m, 90), 12))), q)
            if m > 40:
                add(base[:m // 2] + 'N' + base[m // 2 + 1:], q)   # an N
                ins = base[:m // 2] + 'ACG' + base[m // 2:m - 3]
                add(ins, q)                                        # insertion
                dele = base[:m // 2] + ref[st + m // 2 + 2:st + m + 2]
                if len(dele) == m:
                    add(dele, q)                                   # deletion
            add(_revcomp(base), q)                          # reverse strand
    # two or three non-matches on the seeded diagonal (local mode takes these
    # on the fast path when no other diagonal of the band matches the read
    # across the span between them well enough to pay for a gap): spread,
    # adjacent, a few rows apart, at the read ends, with an N, at low and
    # high quality, and inside tandem repeats (diagonals 3 and 8 away match
    # every row between the non-matches)
    for m in (251, 150, 300):
        st = int(rng.integers(0, len(POL) - m + 1))
        base = POL[st:st + m]
        for qc in ('#', '5', 'I'):
            q = qc * m
            for at in ((m // 4, m // 2, 3 * m // 4), (m // 2, m // 2 + 1), (m // 2, m // 2 + 2),
                       (m // 2, m // 2 + 3, m // 2 + 6), (40, 44, 48), (1, m - 2), (0, 4, m - 1),
                       (m // 3, m // 3 + 4), (60, 70), (60, 61, 62)):
                add(mutate(base, list(at)), q)
            nb = mutate(base, [m // 3, 2 * m // 3])
            add(nb[:m // 2] + 'N' + nb[m // 2 + 1:], q)
    for m in (251, 120):
        rep = refs[1]
        for st in (8, 330, 420):
            for at in ((m // 2, m // 2 + 5), (m // 3, m // 2, 2 * m // 3), (10, 12), (m // 2, m // 2 + 9)):
                for qc in ('#', 'I'):
                    add(mutate(rep[st:st + m], list(at)), qc * m)
    # reference-end overhangs and tandem-repeat reads
    for m in (251, 120):
        add(POL[:m - 30].rjust(m, 'A'), 'G' * m)
        add(POL[-(m - 25):] + 'C' * 25, 'G' * m)
        rep = refs[1]
        for st in (0, 16, 40, 320, 400):
            add(rep[st:st + m], 'G' * m)
            add(mutate(rep[st:st + m], [m // 2]), 'G' * m)
    return refs, seqs, quals


def _gpu(ctx, refs, mode, seqs, quals):
    ctx.index_build(['ref%d' % i for i in range(len(refs))], refs, oracle.seed_len(mode))
    ctx.reads_load(seqs, quals, False)
    ctx.map(_native.params(mode))
    return ctx.fetch(), ctx.map_stats()


@pytest.mark.parametrize('mode', [oracle.E2E, oracle.LOCAL])
def test_fast_path_equals_oracle_full_dp(mode):
    refs, seqs, quals = _cases()
    ix = oracle.Index(refs, oracle.seed_len(mode))
    ref = np.frombuffer(bytes(oracle.map_reads(ix, oracle.params(mode), seqs, quals, False)),
                        dtype=_native.ALN_DTYPE)[:len(seqs)]
    ctx = _native.Context(0)
    try:
        fast, st_fast = _gpu(ctx, refs, mode, seqs, quals)
    finally:
        ctx.close()
    assert st_fast[3] > 0.2 * st_fast[1], st_fast    # the fast path is exercised
    assert st_fast[3] < st_fast[1], st_fast          # and so is the fallback
    for name, got in (('fast path', fast),):
        for i in range(len(ref)):
            for f in _native.ALN_FIELDS:
                assert got[i][f] == ref[i][f], (name, i, f, got[i][f], ref[i][f], seqs[i][:40])
            n = ref[i]['n_cigar']
            assert np.array_equal(got[i]['cigar'][:n], ref[i]['cigar'][:n]), (
                name, i, _native.cigar_text(got[i]), _native.cigar_text(ref[i]))


def _low_complexity_reference(rng):
    """Homopolymer runs, di- and trinucleotide repeats and short random
    stretches: many diagonals of a band match the read over long stretches,
    so a one-gap path between two diagonals that are both off the seeded one
    can beat the seeded diagonal's two or three non-matches."""
    parts, prev = [], ''
    while sum(map(len, parts)) < 3000:
        kind = int(rng.integers(0, 5))
        if kind <= 1:
            b = 'ACGT'[int(rng.integers(0, 4))]
            while b == prev:
                b = 'ACGT'[int(rng.integers(0, 4))]
            parts.append(b * int(rng.integers(6, 70)))
            prev = b
        elif kind == 2:
            unit = ['AC', 'AT', 'GT', 'CG', 'AG'][int(rng.integers(0, 5))]
            parts.append(unit * int(rng.integers(5, 30)))
            prev = ''
        elif kind == 3:
            unit = ['AAC', 'GGT', 'ACT', 'TTG'][int(rng.integers(0, 4))]
            parts.append(unit * int(rng.integers(4, 20)))
            prev = ''
        else:
            parts.append(''.join('ACGT'[x] for x in rng.integers(0, 4, int(rng.integers(4, 20)))))
            prev = ''
    return ''.join(parts)


def _low_complexity_cases():
    rng = np.random.default_rng(2029)
    ref = _low_complexity_reference(rng)
    seqs, quals = [], []
    for _ in range(6000):
        m = int(rng.choice([251, 150, 300]))
        st = int(rng.integers(0, len(ref) - m - 8))
        s = list(ref[st:st + m + 8])
        # one or two small indels (a run one or two bases shorter or longer):
        # the read then sits on two or three diagonals of the band
        for _ in range(int(rng.integers(0, 3))):
            p = int(rng.integers(10, m - 10))
            n = int(rng.integers(1, 3))
            if rng.integers(0, 2):
                del s[p:p + n]
            else:
                s[p:p] = [s[p]] * n
        s = s[:m]
        # two or three substitutions (non-matches of the seeded diagonal)
        for p in rng.choice(m, size=int(rng.integers(0, 4)), replace=False):
            s[p] = 'ACGT'[('ACGT'.index(s[p]) + 1 + int(rng.integers(0, 3))) % 4]
        seq = ''.join(s)
        if rng.integers(0, 4) == 0:
            seq = _revcomp(seq)
        qc = 'I' if rng.integers(0, 3) else 'G'
        seqs.append(seq)
        quals.append(qc * m)
    return [ref, POL], seqs, quals


def test_fast_path_low_complexity_equals_oracle():
    """Local mode over low-complexity reference: every fast-path decision must
    agree with the full DP (og_mapper.c dp_extend), including the one-gap
    paths between two diagonals that are both off the seeded one."""
    refs, seqs, quals = _low_complexity_cases()
    mode = oracle.LOCAL
    ix = oracle.Index(refs, oracle.seed_len(mode))
    ref = np.frombuffer(bytes(oracle.map_reads(ix, oracle.params(mode), seqs, quals, False)),
                        dtype=_native.ALN_DTYPE)[:len(seqs)]
    ctx = _native.Context(0)
    try:
        got, st = _gpu(ctx, refs, mode, seqs, quals)
    finally:
        ctx.close()
    assert 0 < st[3] < st[1], st
    def same(a, b):
        n = int(b['n_cigar'])
        return (all(a[f] == b[f] for f in _native.ALN_FIELDS)
                and np.array_equal(a['cigar'][:n], b['cigar'][:n]))
    bad = [i for i in range(len(ref)) if not same(got[i], ref[i])]
    assert not bad, [(i, _native.cigar_text(got[i]), int(got[i]['score']), _native.cigar_text(ref[i]),
                      int(ref[i]['score'])) for i in bad[:5]]


def _periodic_pieces(rng, n):
    """A reference stretch of periodic pieces (period 1 to 4, random units
    and lengths): diagonals a period apart match the read along a whole
    piece."""
    out = []
    while len(out) < n:
        per = int(rng.integers(1, 5))
        unit = rng.integers(0, 4, per)
        out.extend(np.resize(unit, int(rng.integers(8, 90))).tolist())
    return np.array(out[:n], dtype=np.int64)


def _two_diagonal_cases(n_cases, seed):
    """Reads that sit exactly on one diagonal up to a row c and on another
    after it (one gap, 1 to 12 lanes apart), over periodic reference pieces,
    with up to one substitution: a centre between or beside the two (probed
    at every offset of the band) sees only two or three non-matches on its
    own diagonal while the best path is the two-diagonal one -- the shape
    ADVICE r05 found the ungapped fast path's bound missing."""
    rng = np.random.default_rng(seed)
    refs, reads, quals, items = [], [], [], []
    for t in range(n_cases):
        m = int(rng.choice([251, 150, 300]))
        g = _periodic_pieces(rng, m + 80)
        p = 40
        s1, s2 = 0, 0
        while s1 == s2:
            s1, s2 = (int(x) for x in rng.integers(-6, 7, 2))
        c = int(rng.integers(20, m - 20))
        rows = np.arange(m)
        r = np.where(rows <= c, g[p + rows + s1], g[p + rows + s2])
        if rng.integers(0, 2):
            x = int(rng.integers(0, m))
            r[x] = (r[x] + 1 + int(rng.integers(0, 3))) % 4
        refs.append(''.join('ACGT'[v] for v in g))
        reads.append(''.join('ACGT'[v] for v in r))
        quals.append(('I' if rng.integers(0, 3) else '5') * m)
        for d in range(-8, 9):
            items.append((t, 0, t, p + d))
    return refs, reads, quals, np.array(items, dtype=np.int32)


@pytest.mark.parametrize('seed', [5, 6])
def test_fast_path_cell_equals_full_dp_two_diagonals(seed):
    """mh_probe_extend: for every probed extension the fast path accepts,
    the full banded DP on the same staged tables must find the same best
    cell (score, row, band lane).  The probe runs both k_dp paths."""
    refs, reads, quals, items = _two_diagonal_cases(4000, seed)
    ctx = _native.Context(0)
    try:
        ctx.index_build(['t%d' % i for i in range(len(refs))], refs, oracle.seed_len(oracle.LOCAL))
        ctx.reads_load(reads, quals, False)
        out = ctx.probe_extend(_native.params(oracle.LOCAL), items)
    finally:
        ctx.close()
    fast = out[:, 0] == 1
    assert fast.sum() > 100, fast.sum()   # (B) declines most: periodic pieces
    bad = np.flatnonzero(fast & np.any(out[:, 1:4] != out[:, 5:8], axis=1))
    assert len(bad) == 0, [(int(i), items[i].tolist(), out[i].tolist()) for i in bad[:5]]


def test_fast_path_round5_counterexamples():
    """Extensions on which round 5's fast path (restated in
    profiles/diag/fastpath_search.py) accepted the seeded diagonal's cell
    while the full banded DP finds a better one on a path between two other
    diagonals (tests/golden/fastpath_two_diagonal.json, found by that
    search).  Through mh_probe_extend: the full DP must find the fixture's
    cell, and the fast path must decline or agree with it."""
    import json
    import os
    path = os.path.join(os.path.dirname(__file__), 'golden', 'fastpath_two_diagonal.json')
    with open(path) as f:
        cases = json.load(f)['cases']
    assert len(cases) >= 10
    ctx = _native.Context(0)
    try:
        ctx.index_build(['t%d' % i for i in range(len(cases))], [c['ref'] for c in cases],
                        oracle.seed_len(oracle.LOCAL))
        ctx.reads_load([c['read'] for c in cases], [c['qual'] for c in cases], False)
        items = np.array([(t, 0, t, c['centre']) for t, c in enumerate(cases)], dtype=np.int32)
        out = ctx.probe_extend(_native.params(oracle.LOCAL), items)
    finally:
        ctx.close()
    for t, c in enumerate(cases):
        full = c['full']
        # the full DP's cell: score, row, band lane (lane 16 = the centre)
        assert out[t, 5:8].tolist() == [full[0], full[1], full[2] - 15 + 16], (t, out[t].tolist(), full)
        assert out[t, 0] == 0 or out[t, 1:4].tolist() == out[t, 5:8].tolist(), (t, out[t].tolist())
