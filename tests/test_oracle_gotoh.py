"""Oracle Gotoh restatement vs the reference extension's own answers
(tests/golden/gotoh_golden.json: micall/alignment/tests/test.py KATs +
seeded random pairs, produced by _gotoh2.c built from source)."""
import json
import os

import pytest

import oracle


def _cases(golden_dir):
    with open(os.path.join(golden_dir, 'gotoh_golden.json')) as f:
        return json.load(f)['cases']


def test_golden_gotoh(golden_dir):
    cases = _cases(golden_dir)
    assert len(cases) > 100
    for c in cases:
        if c['error']:
            with pytest.raises(RuntimeError):
                oracle.gotoh_align(c['seq1'], c['seq2'], c['gop'], c['gep'], c['is_global'],
                                   c['alphabet'], c['matrix'])
            continue
        got = oracle.gotoh_align(c['seq1'], c['seq2'], c['gop'], c['gep'], c['is_global'],
                                 c['alphabet'], c['matrix'])
        if len(got[0]) == len(c['seq1']) + len(c['seq2']):
            # No column pairs the sequences: the reference writes the NUL one
            # past its l1+l2 stack buffers (_gotoh2.c:425, :481-482), so its
            # strings are undefined; check the score and our own consistency.
            assert got[2] == c['score']
            assert got[0].replace('-', '') == c['seq1'] and got[1].replace('-', '') == c['seq2']
            continue
        assert got == (c['aligned1'], c['aligned2'], c['score']), c


def test_reference_kats_explicit():
    """The literal expectations of micall/alignment/tests/test.py:174-286."""
    nuc = os.path.join(os.path.dirname(__file__), '..', 'micall-lite_amd', 'micall_amd', 'data')
    mat, alpha = [5, -4, -4, -4, 0, -4, 5, -4, -4, 0, -4, -4, 5, -4, 0, -4, -4, -4, 5, 0,
                  0, 0, 0, 0, 0], 'ACGT?'
    assert oracle.gotoh_align('ACGT', 'ACT', 5, 1, True, alpha, mat) == ('ACGT', 'AC-T', 9)
    assert oracle.gotoh_align('TACGTA', 'ACGT', 5, 1, False, alpha, mat) == ('TACGTA', '-ACGT-', 20)
    assert oracle.gotoh_align('AT', 'ATTTTTT', 5, 1, True, alpha, mat) == ('AT-----', 'ATTTTTT', 5 + 5 - 5 - 1 - 4)
    assert oracle.gotoh_align('GCA', 'CA', 10, 1, True, alpha, mat) == ('GCA', '-CA', -1)
    assert oracle.gotoh_align('A', 'ATTTTT', 5, 1, False, alpha, mat) == ('A-----', 'ATTTTT', 5)


def test_levenshtein():
    assert oracle.levenshtein('kitten', 'sitting') == 3
    assert oracle.levenshtein('', 'abc') == 3
    assert oracle.levenshtein('ACGT', 'ACGT') == 0
