"""The aln2counts oracle (oracle/og_aln2counts.py) against the reference's own
outputs -- every call of micall/tests/aln2counts_test.py replayed
(tests/golden/aln2counts_golden.json), aln2counts() on every e2e case's
aligned.csv (tests/golden/e2e/*/a2c_*.csv.gz) and on the edge-case texts
(tests/golden/aln2counts_edge.json) -- plus the host pieces of the drop-in
that need no device: the codon table and the vectorised consensus letters."""
import gzip
import json
import os

import numpy as np
import pytest

import a2c_replay
import og_aln2counts as og
from micall_amd import aln2counts as a2c
from micall_amd import translation

HERE = os.path.dirname(os.path.abspath(__file__))
GOLDEN = os.path.join(HERE, 'golden')
SCRIPTS = a2c_replay.scripts()
E2E = sorted(os.listdir(os.path.join(GOLDEN, 'e2e')))
EDGE = json.load(open(os.path.join(GOLDEN, 'aln2counts_edge.json')))
ORACLE = dict(SequenceReport=og.Report, InsertionWriter=og.Inserts, SeedAmino=og.AminoTally,
              SeedNucleotide=og.NucTally, projects=og.Projects)


def _gz(path):
    with gzip.open(path, 'rt') as f:
        return f.read()


@pytest.mark.parametrize('k', range(len(SCRIPTS)))
def test_oracle_replays_reference_calls(k):
    assert a2c_replay.replay(SCRIPTS[k], ORACLE) == []


@pytest.mark.parametrize('case', E2E)
def test_oracle_matches_reference_e2e(case):
    d = os.path.join(GOLDEN, 'e2e', case)
    got = og.aln2counts(_gz(os.path.join(d, 'aligned.csv.gz')), og.default_projects())
    for k, text in got.items():
        assert text == _gz(os.path.join(d, 'a2c_{}.csv.gz'.format(k))), k


@pytest.mark.parametrize('k', range(len(EDGE['cases'])))
def test_oracle_matches_reference_edge(k):
    case = EDGE['cases'][k]
    assert og.aln2counts(case['text'], og.Projects(EDGE['config'])) == case['outputs']


def test_codon_table_matches_oracle_translation():
    table = translation.codon_chars().decode()
    alpha = translation.READ_ALPHABET
    for i, ch in enumerate(table):
        codon = alpha[i // 36] + alpha[i // 6 % 6] + alpha[i % 6]
        assert ch == og.codon_to_amino(codon), codon
    pol = 'ATGGCNCCRATT---AAYNNNTGA'
    for off in range(3):
        assert translation.translate(pol, off, '-') == og.translate(pol, off, '-')


@pytest.mark.parametrize('cutoff', ['MAX', 0.01, 0.1, 0.25, 0.5, 0.9])
def test_vectorised_consensus_letters_match_seed_nucleotide(cutoff):
    """_nuc_letters (the drop-in's per-position consensus) against the
    oracle's SeedNucleotide on random counters, first-seen orders included."""
    rng = np.random.default_rng(5)
    n = 4000
    cnt = rng.integers(0, 6, size=(n, 6)) * (rng.random((n, 6)) < 0.5)
    cnt[rng.random(n) < 0.1, :4] = 0                          # only N / '-' read
    first = np.full((n, 6), 0xffffffff, dtype=np.uint32)
    for i in range(n):
        order = rng.permutation(6)
        for rank, b in enumerate(order):
            if cnt[i, b] > 0 or rng.random() < 0.05:          # zero counts can be keys too
                first[i, b] = rank
    letters, cov = a2c._nuc_letters(cnt.astype(np.int64), first, cutoff)
    for i in range(n):
        tally = og.NucTally()
        for b in np.argsort(first[i], kind='stable'):
            if first[i, b] != 0xffffffff:
                tally.counts['ACGTN-'[b]] = int(cnt[i, b])
        assert letters[i] == tally.get_consensus(cutoff), (i, cnt[i], first[i])
        assert cov[i] == sum(tally.counts.values())
