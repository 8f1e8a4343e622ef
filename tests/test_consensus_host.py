"""consensus.Pileup.tokens / _assemble (byte arrays, deletion stretches
vectorised) against a per-position restatement of remap.py:309-333 on
random pileups that mix seed prefill, 'N' / '-' sentinels, empty positions,
insertion tokens and deletion runs of every length."""
from collections import Counter

import numpy as np
import pytest

from micall_amd.consensus import Pileup, _assemble, find_top_token


def _tokens_per_position(pile, r, seed):
    end = max(int(pile.max_pos[r]), len(seed) if seed else 0) + 1
    out = []
    for pos in range(1, end):
        c = pile.counter_at(r, pos, seed)
        out.append(find_top_token(c) if c else None)
    return out


def _assemble_loop(tokens):
    """remap.py:322-332 token by token."""
    out, deletion = [], 0
    for t in tokens:
        if t is None:
            out.append('N')
        elif t == '-':
            deletion += 1
        else:
            if deletion:
                if deletion % 3 != 0:
                    out.append('-' * deletion)
                deletion = 0
            out.append(t)
    return ''.join(out)


@pytest.mark.parametrize('seed_len', [0, 40, 120])
@pytest.mark.parametrize('rs', range(12))
def test_tokens_and_assembly_match_the_loop(rs, seed_len):
    rng = np.random.default_rng(rs)
    length, cap = 150, 160
    dense = np.zeros((1, cap, 4), dtype=np.int32)
    nflag = np.zeros((1, cap), dtype=np.uint8)
    dflag = np.zeros((1, cap), dtype=np.uint8)
    kind = rng.integers(0, 6, size=length)
    for p in range(length):
        if kind[p] == 0:
            dense[0, p] = rng.integers(0, 3, size=4)        # ties included
        elif kind[p] == 1:
            dflag[0, p] = 1
        elif kind[p] == 2:
            nflag[0, p] = 1
            dflag[0, p] = rng.integers(0, 2)
    # deletion runs of 1..7 positions
    for _ in range(4):
        a = int(rng.integers(0, length - 8))
        n = int(rng.integers(1, 8))
        dense[0, a:a + n] = 0
        nflag[0, a:a + n] = 0
        dflag[0, a:a + n] = 1
    events = []
    for p in rng.choice(np.arange(1, length + 1), size=6, replace=False):
        for _ in range(int(rng.integers(1, 3))):
            tok = 'ACGT'[int(rng.integers(0, 4))] + ''.join(rng.choice(list('ACGT'), size=3))
            events.append((0, int(p), tok, int(rng.integers(1, 4))))
    seed = ''.join(rng.choice(list('ACGTRY'), size=seed_len)) if seed_len else None
    fetched = dict(dense=dense, nflag=nflag, dflag=dflag, read_counts=np.array([5]),
                   first_unit=np.array([0]), max_pos=np.array([length - int(rng.integers(0, 20))]),
                   cap=cap, events=events)
    pile = Pileup(fetched, ['r'])
    want = _tokens_per_position(pile, 0, seed)
    tok, longer = pile.tokens(0, seed)
    got = [None if b == 0 else chr(b) for b in tok]
    for i, t in longer.items():
        got[i] = t
    assert got == want
    assert _assemble(tok, longer) == _assemble_loop(want)


@pytest.mark.parametrize('rs', range(20))
def test_event_positions_match_the_counter(rs):
    """Positions with insertion tokens (resolved vectorised in
    Pileup._event_tokens) against counter_at + find_top_token: many tokens
    per position with tied counts, tokens tying the best base both ways
    ('AC' < 'C', 'A' < 'AC'), positions with no base at all (only 'N' / '-'
    flags, or nothing), one-character tokens, repeated (pos, token) entries,
    seeds with N / R / Y, and tokens past the reference's end."""
    rng = np.random.default_rng(100 + rs)
    length, cap = 120, 130
    dense = np.zeros((1, cap, 4), dtype=np.int32)
    nflag = np.zeros((1, cap), dtype=np.uint8)
    dflag = np.zeros((1, cap), dtype=np.uint8)
    for p in range(length):
        k = int(rng.integers(0, 5))
        if k < 3:
            dense[0, p] = rng.integers(0, 4, size=4)
        elif k == 3:
            nflag[0, p] = rng.integers(0, 2)
            dflag[0, p] = rng.integers(0, 2)
    events = []
    for p in rng.choice(np.arange(1, length + 6), size=40, replace=False):
        for _ in range(int(rng.integers(1, 5))):
            n = int(rng.choice([1, 2, 3, 4]))
            tok = ''.join(rng.choice(list('ACGT'), size=n))
            events.append((0, int(p), tok, int(rng.integers(1, 5))))
    if events and rs % 3 == 0:
        events.append(events[0])            # a repeated (pos, token)
    if rs % 2:
        events.sort(key=lambda e: (e[1], e[2]))   # the device's (pos, token) order
    seed = ''.join(rng.choice(list('ACGTNRY'), size=int(rng.integers(0, 140)))) or None
    fetched = dict(dense=dense, nflag=nflag, dflag=dflag, read_counts=np.array([5]),
                   first_unit=np.array([0]), max_pos=np.array([length]), cap=cap, events=events)
    pile = Pileup(fetched, ['r'])
    want = _tokens_per_position(pile, 0, seed)
    for vectorised in (False, True):
        # tokens() for the positions without events, then each event path
        # over the event positions
        tok = pile.tokens(0, seed)[0].copy()
        longer = {}
        end = len(tok)
        d, nf, df = pile._slice(0, end)
        run = pile._event_tokens if vectorised else pile._event_tokens_loop
        run(0, seed, end, d, nf, df, tok, longer)
        got = [None if b == 0 else chr(b) for b in tok]
        for i, t in longer.items():
            got[i] = t
        assert got == want, vectorised


def test_assembly_edge_cases():
    def run(tokens):
        tok = np.array([0 if t is None else ord(t[0]) for t in tokens], dtype=np.uint8)
        longer = {i: t for i, t in enumerate(tokens) if t and len(t) > 1}
        return _assemble(tok, longer), _assemble_loop(tokens)
    for tokens in ([], ['-'], [None], ['-', '-', '-', 'A'], ['-', None, '-', 'C'],
                   ['A', '-', '-', None, None], ['ACCT', '-', 'G'], [None, 'ACGT', None],
                   ['-', '-', 'T', '-', '-', '-', '-', 'G', '-']):
        got, want = run(tokens)
        assert got == want, tokens


def _random_pileup(rng, n_refs, cap):
    dense = np.zeros((n_refs, cap, 4), dtype=np.int32)
    nflag = np.zeros((n_refs, cap), dtype=np.uint8)
    dflag = np.zeros((n_refs, cap), dtype=np.uint8)
    max_pos = np.zeros(n_refs, dtype=np.int32)
    events = []
    for r in range(n_refs):
        kind = int(rng.integers(0, 5))
        if kind == 0:
            continue                                     # nothing counted: no consensus
        length = int(rng.integers(5, cap - 5))
        max_pos[r] = length
        k = rng.integers(0, 6, size=length)
        dense[r, :length][k <= 1] = rng.integers(0, 4, size=(int((k <= 1).sum()), 4))
        nflag[r, :length][k == 2] = 1
        dflag[r, :length][(k == 3) | ((k == 2) & (rng.random(length) < 0.5))] = 1
        for _ in range(int(rng.integers(0, 4))):         # deletion runs of 1..7
            a = int(rng.integers(0, max(1, length - 8)))
            n = int(rng.integers(1, 8))
            dense[r, a:a + n] = 0
            nflag[r, a:a + n] = 0
            dflag[r, a:a + n] = 1
        if kind == 4:                                    # only sentinels and events
            dense[r] = 0
        for p in rng.choice(np.arange(1, length + 1), size=min(length, int(rng.integers(0, 12))),
                            replace=False):
            for _ in range(int(rng.integers(1, 4))):
                n = int(rng.choice([1, 2, 4, 7]))
                tok = ''.join(rng.choice(list('ACGT'), size=n))
                events.append((r, int(p), tok, int(rng.integers(1, 4))))
    return dict(dense=dense, nflag=nflag, dflag=dflag, read_counts=rng.integers(1, 9, size=n_refs),
                first_unit=np.arange(n_refs), max_pos=max_pos, cap=cap, events=events)


@pytest.mark.parametrize('rs', range(30))
def test_native_counts_to_conseqs_matches_the_counter(rs):
    """consensus.counts_to_conseqs (the library's mh_conseqs_build, every
    reference in one call) against the per-position Counter + find_top_token
    + token-by-token assembly (remap.py:309-333), and against
    counts_to_conseqs_py: several references, some with nothing counted or
    only sentinels and insertion tokens, seeds shorter and longer than the
    counted span (with N / R / Y), one-character and long tokens, ties."""
    from micall_amd.consensus import counts_to_conseqs, counts_to_conseqs_py
    rng = np.random.default_rng(500 + rs)
    n_refs, cap = 6, 90
    fetched = _random_pileup(rng, n_refs, cap)
    names = ['r%d' % r for r in range(n_refs)]
    seeds = {}
    for r in range(n_refs):
        if rng.random() < 0.7:
            seeds[names[r]] = ''.join(rng.choice(list('ACGTNRY'), size=int(rng.integers(1, cap + 20))))
    pile = Pileup(fetched, names)
    order = list(range(n_refs))
    want = {}
    for r in order:
        seed = seeds.get(names[r])
        toks = _tokens_per_position(pile, r, seed)
        positive = (pile.dense[r] > 0).any() or any(e[0] == r for e in fetched['events'])
        if positive:
            want[names[r]] = _assemble_loop(toks)
    got = counts_to_conseqs(pile, order, seeds=seeds)
    assert got == want
    assert list(got) == list(want)
    assert counts_to_conseqs_py(pile, order, seeds=seeds) == want
