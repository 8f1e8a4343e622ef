"""BASELINE C5's chain through the drop-ins on the GPU, as bin/micall:91-169
runs it: read_errors -> write_phix_csv -> report_bad_cycles -> censor (R2
with the exhausted bad-cycles reader, bin/micall:116,126) -> prelim_map (-U
for unpaired input) -> remap.  Every intermediate and output file must be
byte-equal to what the stock reference wrote on the same inputs
(tests/golden/chain/, tests/golden/gen_golden.py chain)."""
import csv
import gzip
import io
import json
import os

import pytest

from micall_amd import censor_fastq, filter_quality, parse_interop
from micall_amd import prelim_map as pm
from micall_amd import remap as rm

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))
CASES = ['c5_unpaired300', 'c5_paired251']


def _golden(d, name, mode='rt'):
    with gzip.open(os.path.join(d, name + '.gz'), mode) as f:
        return f.read()


@pytest.mark.parametrize('case', CASES)
def test_c5_chain_matches_reference(case, tmp_path):
    d = os.path.join(HERE, 'golden', 'chain', case)
    lengths = json.load(open(os.path.join(d, 'read_lengths.json')))
    with open(os.path.join(d, 'ErrorMetricsOut.bin'), 'rb') as f:
        records = parse_interop.read_errors(f)
        quality = io.StringIO()
        parse_interop.write_phix_csv(out_file=quality, records=records, read_lengths=lengths)
    assert quality.getvalue() == _golden(d, 'quality.csv')
    bad = io.StringIO()
    filter_quality.report_bad_cycles(io.StringIO(quality.getvalue()), bad)
    assert bad.getvalue() == _golden(d, 'bad_cycles.csv')
    reader = csv.DictReader(io.StringIO(bad.getvalue()))
    censored = []
    for mate in (1, 2):
        src = os.path.join(d, 'R%d.fastq.gz' % mate)
        if not os.path.exists(src):
            break
        dst = str(tmp_path / ('R%d.censor.fastq.gz' % mate))
        with open(src, 'rb') as fi, open(dst, 'wb') as fo:
            censor_fastq.censor(src=fi, bad_cycles_reader=reader, dest=fo, use_gzip=True)
        with gzip.open(dst) as f:
            assert f.read() == _golden(d, 'R%d.censor.fastq' % mate, 'rb'), mate
        censored.append(dst)
    r1, r2 = censored[0], (censored[1] if len(censored) > 1 else None)
    prelim = tmp_path / 'prelim.csv'
    with open(prelim, 'w') as f:
        pm.prelim_map(r1, r2, f, gzip=True)
    assert prelim.read_text() == _golden(d, 'prelim.csv')
    names = ('remap.csv', 'remap_counts.csv', 'remap_conseq.csv', 'unmapped1.fastq',
             'unmapped2.fastq')
    with open(prelim) as pre:
        outs = [open(tmp_path / n, 'w+') for n in names]
        rm.remap(r1, r2, pre, *outs, gzip=True, work_path=str(tmp_path))
        for h in outs:
            h.close()
    for n in names:
        assert (tmp_path / n).read_text() == _golden(d, n), n
