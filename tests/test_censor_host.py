"""The censor stage's CPU parts against outputs of the reference itself
(tests/golden/censor/, gen_golden.py censor): the oracle restatement of
censor (oracle/og_censor.py) and the host-side InterOp / bad-cycle modules
of the product (micall_amd.parse_interop, micall_amd.filter_quality)."""
import base64
import csv
import gzip
import io
import json
import os

import pytest

import og_censor
from micall_amd import filter_quality, parse_interop

HERE = os.path.dirname(os.path.abspath(__file__))
CDIR = os.path.join(HERE, 'golden', 'censor')
G = json.load(open(os.path.join(CDIR, 'censor_golden.json')))


class _Named(io.BytesIO):
    name = 'ErrorMetricsOut.bin'


def test_interop_to_phix_csv_matches_reference():
    out = io.StringIO()
    summary = {}
    recs = parse_interop.read_errors(_Named(base64.b64decode(G['error_metrics_b64'])))
    parse_interop.write_phix_csv(out, recs, G['read_lengths'], summary)
    assert out.getvalue() == G['quality_csv']
    assert summary == G['phix_summary']


def test_read_records_errors():
    with pytest.raises(IOError, match='less than minimum version 3'):
        list(parse_interop.read_records(_Named(bytes([1, 4]) + b'ABCD'), 3))
    with pytest.raises(IOError, match='Partial record of length 1'):
        list(parse_interop.read_records(_Named(bytes([1, 3]) + b'ABCD'), 1))


def test_report_bad_cycles_matches_reference():
    bad, tiles = io.StringIO(), io.StringIO()
    filter_quality.report_bad_cycles(io.StringIO(G['quality_csv']), bad, tiles)
    assert bad.getvalue() == G['bad_cycles_csv']
    assert tiles.getvalue() == G['bad_tiles_csv']


EDGE = json.load(open(os.path.join(CDIR, 'interop_edge.json')))


@pytest.mark.parametrize('case', EDGE['phix'], ids=lambda c: c['name'])
def test_phix_csv_edge_cases_match_reference(case):
    """Duplicates, cycle 0, gaps at lane ends, index cycles, one-direction
    lanes, random tables: write_phix_csv's rows and summary as the
    reference wrote them (gen_golden.py interop_edge)."""
    out, summary = io.StringIO(), {}
    parse_interop.write_phix_csv(out, iter([dict(r) for r in case['records']]),
                                 case['read_lengths'], summary)
    assert out.getvalue() == case['csv']
    assert summary == case['summary']


@pytest.mark.parametrize('case', EDGE['quality'], ids=lambda c: c['name'])
def test_bad_cycles_edge_cases_match_reference(case):
    """Blank rates inside a run, a tile that comes back, direction flips,
    rows missing the rate column, unparsable rates after the first bad one."""
    bad, tiles = io.StringIO(), io.StringIO()
    filter_quality.report_bad_cycles(io.StringIO(case['quality_csv']), bad, tiles)
    assert bad.getvalue() == case['bad_cycles_csv']
    assert tiles.getvalue() == case['bad_tiles_csv']


def test_read_records_zero_length_and_stream():
    """A zero record length yields nothing (the reference's read(0) loop
    stops at once); whole records come out in order before a partial one
    raises."""
    assert list(parse_interop.read_records(_Named(bytes([3, 0]) + b'xyz'), 3)) == []
    got = []
    with pytest.raises(IOError, match='Partial record of length 2'):
        for rec in parse_interop.read_records(_Named(bytes([3, 3]) + b'abcdefgh'), 3):
            got.append(rec)
    assert got == [b'abc', b'def']


@pytest.mark.parametrize('k', range(len(G['cases'])))
def test_oracle_censor_scenarios(k):
    case = G['cases'][k]
    bad = {(t, int(c)) for t, c in case['bad_cycles']}
    out, n, total = og_censor.censor_bytes(case['fastq'].encode(), bad)
    assert out.decode() == case['censored']
    avg = '' if n == 0 else repr(float(total) / n)
    assert case['summary'] == 'avg_quality,base_count\n{},{}\n'.format(avg, n)


def test_oracle_censor_synthetic_pair():
    bad = {(row['tile'], int(row['cycle'])) for row in csv.DictReader(io.StringIO(G['bad_cycles_csv']))}
    for mate, cycles in ((1, bad), (2, set())):    # R2 gets the exhausted reader (bin/micall:126)
        with open(os.path.join(CDIR, 'R{}.fastq.gz'.format(mate)), 'rb') as f:
            out, n, total = og_censor.censor_bytes(f.read(), cycles, use_gzip=True)
        with gzip.open(os.path.join(CDIR, 'R{}.censor.fastq.gz'.format(mate))) as f:
            assert out == f.read()
        assert G['summary_r{}'.format(mate)] == 'avg_quality,base_count\n{},{}\n'.format(
            repr(float(total) / n), n)
