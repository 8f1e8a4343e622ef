"""sam2aln on the device (mh_sam2aln_csv, micall_amd.sam2aln) against the
reference's own outputs (tests/golden/sam2aln_e2e.json and
tests/golden/e2e/*/{aligned,insert,failed}.csv.gz, from the reference's
sam2aln() on the same remap.csv) and against the oracle restatement on
larger synthetic remap.csv texts: byte-identical CSV text."""
import csv
import gzip
import io
import json
import os

import numpy as np
import pytest

import og_sam2aln
from micall_amd import _native, projects, synth
from micall_amd import sam2aln as s2a

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))
GOLDEN = os.path.join(HERE, 'golden')
CASES = json.load(open(os.path.join(GOLDEN, 'sam2aln_e2e.json')))['cases']
E2E = sorted(os.listdir(os.path.join(GOLDEN, 'e2e')))


@pytest.fixture(scope='module')
def ctx():
    c = _native.Context(0)
    yield c
    c.close()


def _gz(path):
    with gzip.open(path, 'rt') as f:
        return f.read()


def _device(ctx, text):
    ctx.sam2aln_csv(text)
    return ctx.sam2aln_output('aligned'), ctx.sam2aln_output('insert'), ctx.sam2aln_output('failed')


@pytest.mark.parametrize('k', range(len(CASES)))
def test_sam2aln_matches_reference_calls(ctx, k):
    case = CASES[k]
    al, ins, fa = _device(ctx, case['remap_csv'])
    assert al == case['aligned']
    if case['insert'] is not None:
        assert ins == case['insert']
    if case['failed'] is not None:
        assert fa == case['failed']


@pytest.mark.parametrize('case', E2E)
def test_sam2aln_drop_in_matches_reference_e2e(case):
    d = os.path.join(GOLDEN, 'e2e', case)
    al, ins, fa = io.StringIO(), io.StringIO(), io.StringIO()
    s2a.sam2aln(io.StringIO(_gz(os.path.join(d, 'remap.csv.gz'))), al, ins, fa)
    assert al.getvalue() == _gz(os.path.join(d, 'aligned.csv.gz'))
    assert ins.getvalue() == _gz(os.path.join(d, 'insert.csv.gz'))
    assert fa.getvalue() == _gz(os.path.join(d, 'failed.csv.gz'))


def _synthetic_remap_csv(ctx, n_pairs, seed):
    """remap.csv text from the GPU mapper (--local vs HIV pol) on synthetic
    reads with indels, Ns and low-quality stretches."""
    pol = projects.load_default().seed_sequences()['HIV1B-pol-seed']
    pairs = synth.make_pairs(n_pairs, genomes={'HIV1B-pol-seed': pol}, genome_seed=seed,
                             read_seed=seed + 1, indel_rate=0.01, err_rate=0.02)
    names, seqs, quals = synth.interleave(pairs)
    rng = np.random.default_rng(seed)
    quals = [q if rng.random() > 0.05 else '#' * len(q) for q in quals]
    ctx.index_build(['HIV1B-pol-seed'], [pol], 20)
    names = [n[1:].split()[0] for n in names]      # bowtie2's QNAME: mates share it
    ctx.reads_load(seqs, quals, True, names=names)
    ctx.map(_native.params(_native.LOCAL))
    rows = ctx.format_rows(1, 0, len(seqs))
    return 'qname,flag,rname,pos,mapq,cigar,rnext,pnext,tlen,seq,qual\n' + rows


def test_sam2aln_vs_oracle_synthetic(ctx):
    text = _synthetic_remap_csv(ctx, 3000, 41)
    # duplicate a share of the pairs under new names: counts > 1
    rows = list(csv.reader(io.StringIO(text)))
    extra = [[r[0] + 'x'] + r[1:] for r in rows[1:1201]]
    out = io.StringIO()
    w = csv.writer(out, lineterminator='\n')
    w.writerows(rows + extra)
    text = out.getvalue()
    want = og_sam2aln.sam2aln(text)
    got = _device(ctx, text)
    assert got[0] == want[0]
    assert got[1] == want[1]
    assert got[2] == want[2]
    st = ctx.sam2aln_stats()
    assert st[0] == 3600 and st[1] > 2000 and st[2] < st[1], st   # pairs, merged, distinct
    assert 'manyNs' in got[2] and got[1].count('\n') > 20


def test_sam2aln_rejects_bad_cigar_like_the_reference(ctx):
    text = ('qname,flag,rname,pos,mapq,cigar,rnext,pnext,tlen,seq,qual\n'
            'r1,99,R,1,44,3H3M,=,1,3,ACG,AAA\n'
            'r1,147,R,1,44,3M,=,1,-3,ACG,AAA\n')
    with pytest.raises(RuntimeError, match='Unsupported CIGAR token'):
        ctx.sam2aln_csv(text)
    with pytest.raises(RuntimeError, match='too long'):
        ctx.sam2aln_csv(text.replace('3H3M', '4M'))


def test_sam2aln_matchmaker_order_vs_oracle(ctx):
    """The matchmaker (sam2aln.py:291-312) on rows shuffled so mates sit far
    apart, with qnames seen three and four times (a third row waits for a
    fourth) and mates that never come: byte-identical to the oracle."""
    text = _synthetic_remap_csv(ctx, 1500, 53)
    rows = list(csv.reader(io.StringIO(text)))
    head, body = rows[0], rows[1:]
    rng = np.random.default_rng(5)
    body = [body[i] for i in rng.permutation(len(body))]
    extra = [list(r) for r in body[:300]]                     # third and fourth rows of 300 qnames
    lone = [[r[0] + 'lone'] + r[1:] for r in body[300:420]]   # mates that never come
    body = body + extra[:150] + lone + extra[150:] + [list(r) for r in body[:150]]
    out = io.StringIO()
    csv.writer(out, lineterminator='\n').writerows([head] + body)
    text = out.getvalue()
    want = og_sam2aln.sam2aln(text)
    got = _device(ctx, text)
    assert got[0] == want[0]
    assert got[1] == want[1]
    assert got[2] == want[2]
    assert 'unmatched' in want[2]


@pytest.mark.parametrize('case', E2E)
def test_sam2aln_drop_in_on_files_streamed(tmp_path, case):
    """The drop-in on real files, as bin/micall calls it: remap.csv mmap'd,
    every output formatted and written in one pass (mh_sam2aln_write
    without a size query) at the handle's position, after what the caller
    had written through the handle."""
    d = os.path.join(GOLDEN, 'e2e', case)
    rp = tmp_path / 'remap.csv'
    rp.write_text(_gz(os.path.join(d, 'remap.csv.gz')))
    outs = {k: tmp_path / (k + '.csv') for k in ('aligned', 'insert', 'failed')}
    with open(rp) as remap, open(outs['aligned'], 'w') as al, open(outs['insert'], 'w') as ins, \
            open(outs['failed'], 'w') as fa:
        for h in (al, ins, fa):
            h.write('lead\n')
        s2a.sam2aln(remap, al, ins, fa)
        for h in (al, ins, fa):
            h.write('tail\n')
    for k, p in outs.items():
        assert p.read_text() == 'lead\n' + _gz(os.path.join(d, k + '.csv.gz')) + 'tail\n'


def test_sam2aln_streamed_write_matches_collected(ctx, tmp_path):
    """Many formatting jobs (more rows than one 4096-row job): the streamed
    file output equals the collected text, byte for byte."""
    text = _synthetic_remap_csv(ctx, 20000, 7)
    al_want, ins_want, fa_want = _device(ctx, text)
    assert al_want.count('\n') > 3 * 4096
    rp = tmp_path / 'remap.csv'
    rp.write_text(text)
    outs = {k: tmp_path / (k + '.csv') for k in ('aligned', 'insert', 'failed')}
    with open(rp) as remap, open(outs['aligned'], 'w') as al, open(outs['insert'], 'w') as ins, \
            open(outs['failed'], 'w') as fa:
        s2a.sam2aln(remap, al, ins, fa)
    assert outs['aligned'].read_text() == al_want
    assert outs['insert'].read_text() == ins_want
    assert outs['failed'].read_text() == fa_want
