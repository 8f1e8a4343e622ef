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
