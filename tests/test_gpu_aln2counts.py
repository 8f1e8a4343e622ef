"""aln2counts on the device (mh_a2c_*, micall_amd.aln2counts) against the
reference's own outputs -- every call of micall/tests/aln2counts_test.py
replayed, aln2counts() on every e2e case's aligned.csv and on the edge-case
texts -- and against the oracle (oracle/og_aln2counts.py) on a larger
synthetic aligned.csv: byte-identical CSV text, equal counters."""
import gzip
import io
import json
import os
import random

import numpy as np
import pytest

import a2c_replay
import og_aln2counts as og
from micall_amd import _native, projects, session
from micall_amd import aln2counts as a2c

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))
GOLDEN = os.path.join(HERE, 'golden')
SCRIPTS = a2c_replay.scripts()
E2E = sorted(os.listdir(os.path.join(GOLDEN, 'e2e')))
EDGE = json.load(open(os.path.join(GOLDEN, 'aln2counts_edge.json')))
PRODUCT = dict(SequenceReport=a2c.SequenceReport, InsertionWriter=a2c.InsertionWriter,
               SeedAmino=a2c.SeedAmino, SeedNucleotide=a2c.SeedNucleotide,
               projects=projects.ProjectConfig.from_config)
OUTS = ('nuc', 'amino', 'coord_ins', 'conseq', 'failed', 'coverage')


def _gz(path):
    with gzip.open(path, 'rt') as f:
        return f.read()


def _run(text, json_path=None):
    outs = {k: io.StringIO() for k in OUTS}
    a2c.aln2counts(io.StringIO(text), outs['nuc'], outs['amino'], outs['coord_ins'],
                   outs['conseq'], failed_align_csv=outs['failed'],
                   coverage_summary_csv=outs['coverage'], json=json_path)
    return {k: v.getvalue() for k, v in outs.items()}


@pytest.mark.parametrize('k', range(len(SCRIPTS)))
def test_aln2counts_replays_reference_calls(k):
    assert a2c_replay.replay(SCRIPTS[k], PRODUCT) == []


@pytest.mark.parametrize('case', E2E)
def test_aln2counts_drop_in_matches_reference_e2e(case):
    d = os.path.join(GOLDEN, 'e2e', case)
    got = _run(_gz(os.path.join(d, 'aligned.csv.gz')))
    for k in OUTS:
        assert got[k] == _gz(os.path.join(d, 'a2c_{}.csv.gz'.format(k))), k


def test_aln2counts_matches_reference_edge(tmp_path):
    path = str(tmp_path / 'projects.json')
    with open(path, 'w') as f:
        json.dump(EDGE['config'], f)
    for k, case in enumerate(EDGE['cases']):
        assert _run(case['text'], path) == case['outputs'], k


def _synthetic_aligned(n_rows, seed):
    """aligned.csv rows over HIV-1 pol: a sample with an inserted codon,
    substitutions, N, '-', 'n', tied counts, two qcut groups."""
    rng = random.Random(seed)
    pol = projects.load_default().seed_sequences()['HIV1B-pol-seed']
    sample = pol[:1500] + 'GGA' + pol[1500:]
    rows, seen = [], set()
    for qcut in ('15', '20'):
        for rank in range(n_rows // 2):
            off = rng.randrange(0, len(sample) - 120)
            s = list(sample[off:off + rng.randint(60, 420)])
            for i in range(len(s)):
                r = rng.random()
                if r < 0.02:
                    s[i] = rng.choice('ACGT')
                elif r < 0.03:
                    s[i] = 'N'
            if rng.random() < 0.2:
                i = rng.randrange(10, len(s) - 20)
                s[i:i + 5] = ['n'] * 5
            if rng.random() < 0.1:
                i = rng.randrange(10, len(s) - 20)
                s[i:i + 3] = ['-'] * 3
            s = ''.join(s).strip('-')
            if (qcut, off, s) in seen:
                continue
            seen.add((qcut, off, s))
            rows.append('HIV1B-pol-seed,{},{},{},{},{}\n'.format(qcut, rank, rng.choice([1, 2, 3, 7]),
                                                                   off, s))
    return 'refname,qcut,rank,count,offset,seq\n' + ''.join(rows)


def test_aln2counts_vs_oracle_synthetic():
    text = _synthetic_aligned(3000, 11)
    want = og.aln2counts(text, og.default_projects())
    got = _run(text)
    for k in OUTS:
        assert got[k] == want[k], k
    assert got['coord_ins'].count('\n') > 1


def test_counters_match_oracle_tallies():
    """mh_a2c_counts (count + first row per counter) against the oracle's
    Counter objects, including their insertion order."""
    text = _synthetic_aligned(800, 3)
    ctx = session.context()
    n = ctx.a2c_load_csv(0, text, a2c._CODON_CHARS)
    assert n == 2
    import csv
    rows = list(csv.DictReader(io.StringIO(text)))
    for g in range(n):
        info = ctx.a2c_group(0, g)
        grp = rows[info['first']:info['first'] + info['n_rows']]
        rep = og.Report(og.Inserts(io.StringIO()), og.Projects({'regions': {}, 'projects': {}}), [])
        rep.projects.seqs[grp[0]['refname']] = 'A'
        rep.read(grp)
        for f in range(3):
            tallies = rep.seed_aminos[f]
            assert info['ncod'][f] == len(tallies)
            aa_c, aa_f, nt_c, nt_f = ctx.a2c_counts(0, g, f, info['ncod'][f])
            for j, t in enumerate(tallies):
                order = [a2c.AMINO_ALPHABET[k] for k in np.argsort(aa_f[j], kind='stable')
                         if aa_f[j][k] != 0xffffffff]
                assert order == list(t.counts), (g, f, j)
                assert [int(aa_c[j][a2c.AMINO_ALPHABET.index(a)]) for a in order] == \
                    list(t.counts.values())
                for p in range(3):
                    cnt, fst = nt_c[j][6 * p:6 * p + 6], nt_f[j][6 * p:6 * p + 6]
                    order = ['ACGTN-'[k] for k in np.argsort(fst, kind='stable') if fst[k] != 0xffffffff]
                    assert order == list(t.nucleotides[p].counts), (g, f, j, p)
                    assert [int(cnt['ACGTN-'.index(b)]) for b in order] == \
                        list(t.nucleotides[p].counts.values())


def test_aln2counts_rejects_what_it_cannot_count():
    ctx = session.context()
    head = 'refname,qcut,rank,count,offset,seq\n'
    with pytest.raises(_native.NativeError, match='not one of'):
        ctx.a2c_load_csv(0, head + 'R,15,0,1,0,ACGXT\n', a2c._CODON_CHARS)
    with pytest.raises(_native.NativeError, match='offset'):
        ctx.a2c_load_csv(0, head + 'R,15,0,1,-3,ACGT\n', a2c._CODON_CHARS)
    with pytest.raises(_native.NativeError, match='int'):
        ctx.a2c_load_csv(0, head + 'R,15,0,x,0,ACGT\n', a2c._CODON_CHARS)
    assert ctx.a2c_load_csv(0, head, a2c._CODON_CHARS) == 0
    assert ctx.a2c_load_csv(0, '', a2c._CODON_CHARS) == 0
