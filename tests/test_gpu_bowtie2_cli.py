"""The bowtie2 command contract over the HIP mapper (micall-lite_amd/bin),
run as the reference runs it, on the GPU.

prelim: `bowtie2-build-s` over the seed FASTA, then `bowtie2` with
prelim_map.py:114-131's arguments; its SAM lines go through prelim_map.py:
134-151's row handling (restated below) and must give the reference's own
prelim.csv of every e2e golden case byte for byte (tests/golden/e2e, made by
the stock pipeline).  remap: `bowtie2 --local` against the case's final
consensus must print the SAM text the oracle mapper prints for the same
FASTQ files (the text remap.py:740-761 consumes, tags included)."""
import csv
import gzip
import io
import os
import subprocess
import sys

import pytest

import oracle
from micall_amd import projects

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))
BIN = os.path.join(os.path.dirname(HERE), 'micall-lite_amd', 'bin')
CASES = ['c1_example', 'micro_1234A-V3LOOP', 'micro_2090A-HCV', 'syn_chimera', 'syn_unpaired300',
         'micro_2030A-V3LOOP']
FIELDS = ['qname', 'flag', 'rname', 'pos', 'mapq', 'cigar', 'rnext', 'pnext', 'tlen', 'seq', 'qual']


def _golden(d, name):
    with gzip.open(os.path.join(d, name + '.gz'), 'rt') as f:
        return f.read()


def _reads_args(d):
    r1, r2 = os.path.join(d, 'R1.fastq.gz'), os.path.join(d, 'R2.fastq.gz')
    return (['-1', r1, '-2', r2] if os.path.exists(r2) else ['-U', r1]), r1, \
        (r2 if os.path.exists(r2) else None)


def _run(cmd, args):
    p = subprocess.run([sys.executable, os.path.join(BIN, cmd)] + args, stdout=subprocess.PIPE,
                       stderr=subprocess.PIPE, universal_newlines=True, timeout=300)
    assert p.returncode == 0, p.stderr
    return p.stdout


def _prelim_csv(sam_text):
    """prelim_map.py:134-151: rows grouped by rname in first-seen order, the
    first eleven SAM fields of each line."""
    output = {}
    for line in sam_text.splitlines(True):
        output.setdefault(line.split('\t')[2], []).append(line.split('\t')[:11])
    buf = io.StringIO()
    writer = csv.DictWriter(buf, FIELDS, lineterminator=os.linesep)
    writer.writeheader()
    for rows in output.values():
        for row in rows:
            writer.writerow(dict(zip(FIELDS, row)))
    return buf.getvalue()


@pytest.mark.parametrize('case', CASES)
def test_prelim_through_bowtie2_commands(golden_dir, case, tmp_path):
    d = os.path.join(golden_dir, 'e2e', case)
    fasta = tmp_path / 'micall.fasta'
    with open(fasta, 'w') as f:
        projects.load_default().writeSeedFasta(f)
    template = str(tmp_path / 'reference')
    _run('bowtie2-build-s', ['--wrapper', 'micall-0', '--quiet', '-f', str(fasta), template])
    reads, _r1, _r2 = _reads_args(d)
    sam = _run('bowtie2', ['--wrapper', 'micall-0', '--quiet', '-x', template] + reads +
               ['--rdg', '10,3', '--rfg', '10,3', '--no-hd', '-X', '1200', '-p', '4'])
    assert _prelim_csv(sam) == _golden(d, 'prelim.csv')


@pytest.mark.parametrize('case', CASES)
def test_local_pass_through_bowtie2_commands(golden_dir, case, tmp_path):
    d = os.path.join(golden_dir, 'e2e', case)
    conseqs = list(csv.DictReader(io.StringIO(_golden(d, 'remap_conseq.csv'))))
    if not conseqs:
        pytest.skip('no consensus: the remap loop never ran for this case')
    names = [r['region'] for r in conseqs]
    seqs = [r['sequence'] for r in conseqs]
    fasta = tmp_path / 'conseq.fasta'
    fasta.write_text(''.join('>{}\n{}\n'.format(n, s) for n, s in zip(names, seqs)))
    template = str(tmp_path / 'reference')
    _run('bowtie2-build-s', ['--wrapper', 'micall-0', '--quiet', '-f', str(fasta), template])
    reads, r1, r2 = _reads_args(d)
    sam = _run('bowtie2', ['--wrapper', 'micall-0', '--quiet', '-x', template, '--rdg', '10,3',
                           '--rfg', '10,3'] + reads + ['--no-hd', '--local', '-X', '1200', '-p', '4'])
    want = ''.join(oracle.map_fastq_to_sam(names, seqs, oracle.LOCAL, r1, r2, (10, 3), (10, 3), 1200))
    assert sam == want
    with_header = _run('bowtie2', ['-x', template, '--local', '-X', '1200', '--rdg', '10,3',
                                   '--rfg', '10,3'] + reads)
    head = [x for x in with_header.splitlines(True) if x.startswith('@')]
    assert head[0] == '@HD\tVN:1.0\tSO:unsorted\n'
    assert head[1:1 + len(names)] == ['@SQ\tSN:{}\tLN:{}\n'.format(n, len(s)) for n, s in zip(names, seqs)]
    assert with_header[sum(map(len, head)):] == sam
