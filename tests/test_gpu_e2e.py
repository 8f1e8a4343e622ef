"""End-to-end parity of the drop-in prelim_map() / remap() on the GPU against
the stock reference pipeline's own outputs on the same FASTQ files
(tests/golden/e2e/, produced by tests/golden/gen_golden.py e2e with the CPU
oracle mapper standing in for bowtie2, see oracle/bowtie2_shim.py).

Every output file must be byte-identical: prelim.csv, remap.csv,
remap_counts.csv, remap_conseq.csv and the unmapped FASTQs."""
import gzip
import io
import os

import pytest

from micall_amd import prelim_map as pm
from micall_amd import remap as rm

pytestmark = pytest.mark.gpu

CASES = sorted(os.listdir(os.path.join(os.path.dirname(__file__), 'golden', 'e2e')))


def _golden(d, name):
    with gzip.open(os.path.join(d, name + '.gz'), 'rt') as f:
        return f.read()


def _inputs(d):
    r1 = os.path.join(d, 'R1.fastq.gz')
    r2 = os.path.join(d, 'R2.fastq.gz')
    return r1, (r2 if os.path.exists(r2) else None)


@pytest.mark.parametrize('case', CASES)
def test_prelim_map_matches_reference(golden_dir, case):
    d = os.path.join(golden_dir, 'e2e', case)
    r1, r2 = _inputs(d)
    out = io.StringIO()
    pm.prelim_map(r1, r2, out, gzip=True)
    assert out.getvalue() == _golden(d, 'prelim.csv')


@pytest.mark.parametrize('case', CASES)
def test_remap_matches_reference(golden_dir, case, tmp_path):
    d = os.path.join(golden_dir, 'e2e', case)
    r1, r2 = _inputs(d)
    outs = {k: io.StringIO() for k in ('remap.csv', 'remap_counts.csv', 'remap_conseq.csv')}
    un1 = open(tmp_path / 'u1.fastq', 'w+')
    un2 = open(tmp_path / 'u2.fastq', 'w+')
    rm.remap(r1, r2, io.StringIO(_golden(d, 'prelim.csv')), outs['remap.csv'],
             outs['remap_counts.csv'], outs['remap_conseq.csv'], un1, un2, gzip=True,
             work_path=str(tmp_path))
    un1.close()
    un2.close()
    for name, buf in outs.items():
        assert buf.getvalue() == _golden(d, name), name
    assert open(tmp_path / 'u1.fastq').read() == _golden(d, 'unmapped1.fastq')
    assert open(tmp_path / 'u2.fastq').read() == _golden(d, 'unmapped2.fastq')


@pytest.mark.parametrize('case', ['syn_pol', 'syn_chimera', 'c1_example', 'syn_maxremaps'])
def test_chained_dropins_reuse_resident_prelim(golden_dir, case, tmp_path):
    """bin/micall's chain in one process: prelim_map() writes prelim.csv, then
    remap() reads that same unchanged file and takes the prelim rows from the
    records still resident instead of parsing it (session.prelim_resident);
    every file must still be the reference's."""
    from micall_amd import session
    d = os.path.join(golden_dir, 'e2e', case)
    r1, r2 = _inputs(d)
    prelim = tmp_path / 'prelim.csv'
    with open(prelim, 'w') as f:
        pm.prelim_map(r1, r2, f, gzip=True)
    assert prelim.read_text() == _golden(d, 'prelim.csv')
    names = ('remap.csv', 'remap_counts.csv', 'remap_conseq.csv', 'unmapped1.fastq',
             'unmapped2.fastq')
    with open(prelim) as f:
        outs = [open(tmp_path / n, 'w+') for n in names]
        rm.remap(r1, r2, f, *outs, gzip=True, work_path=str(tmp_path))
        for h in outs:
            h.close()
    assert session.stats['prelim_source'] == 'device'
    for n in names:
        assert (tmp_path / n).read_text() == _golden(d, n), n


def test_edited_prelim_csv_is_parsed_again(golden_dir, tmp_path):
    """The resident prelim records are used only for the unchanged file:
    rewriting the same bytes keeps them, other bytes (here '\r\n' line
    ends, which parse to the same rows) make remap() parse the file."""
    from micall_amd import session
    d = os.path.join(golden_dir, 'e2e', 'syn_pol')
    r1, r2 = _inputs(d)
    prelim = tmp_path / 'prelim.csv'
    for edit, source in ((lambda b: b, 'device'), (lambda b: b.replace(b'\n', b'\r\n'), 'csv')):
        with open(prelim, 'w') as f:
            pm.prelim_map(r1, r2, f, gzip=True)
        prelim.write_bytes(edit(prelim.read_bytes()))
        out = io.StringIO()
        with open(prelim) as f:
            rm.remap(r1, r2, f, out)
        assert session.stats['prelim_source'] == source
        assert out.getvalue() == _golden(d, 'remap.csv')
