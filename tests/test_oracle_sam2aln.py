"""The sam2aln restatement (oracle/og_sam2aln.py) against outputs of the
reference's own sam2aln() (tests/golden/gen_golden.py s2a): every call of
micall/tests/sam2aln_test.py, the edge-case remap.csv texts and every e2e
case's remap.csv."""
import gzip
import json
import os

import pytest

import og_sam2aln

HERE = os.path.dirname(os.path.abspath(__file__))
GOLDEN = os.path.join(HERE, 'golden')
CASES = json.load(open(os.path.join(GOLDEN, 'sam2aln_e2e.json')))['cases']
E2E = sorted(os.listdir(os.path.join(GOLDEN, 'e2e')))


def _gz(path):
    with gzip.open(path, 'rt') as f:
        return f.read()


@pytest.mark.parametrize('k', range(len(CASES)))
def test_oracle_matches_reference_calls(k):
    case = CASES[k]
    al, ins, fa = og_sam2aln.sam2aln(case['remap_csv'])
    assert al == case['aligned']
    if case['insert'] is not None:
        assert ins == case['insert']
    if case['failed'] is not None:
        assert fa == case['failed']


@pytest.mark.parametrize('case', E2E)
def test_oracle_matches_reference_e2e(case):
    d = os.path.join(GOLDEN, 'e2e', case)
    al, ins, fa = og_sam2aln.sam2aln(_gz(os.path.join(d, 'remap.csv.gz')))
    assert al == _gz(os.path.join(d, 'aligned.csv.gz'))
    assert ins == _gz(os.path.join(d, 'insert.csv.gz'))
    assert fa == _gz(os.path.join(d, 'failed.csv.gz'))


def test_apply_cigar_rejects_like_the_reference():
    with pytest.raises(RuntimeError, match='Invalid CIGAR'):
        og_sam2aln.apply_cigar('3M,', 'ACG', 'AAA')
    with pytest.raises(RuntimeError, match='Unsupported CIGAR token'):
        og_sam2aln.apply_cigar('3H3M', 'ACG', 'AAA')
    with pytest.raises(RuntimeError, match='too short'):
        og_sam2aln.apply_cigar('2M', 'ACG', 'AAA')
    with pytest.raises(RuntimeError, match='too long'):
        og_sam2aln.apply_cigar('4M', 'ACG', 'AAA')
