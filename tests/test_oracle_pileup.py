"""Oracle pileup + consensus vs the reference's sam_to_conseqs
(tests/golden/pileup_golden.json: every call made by micall/tests/remap_test.py,
answered by the reference code itself, plus oracle-mapped synthetic SAMs)."""
import json
import os

import oracle

# micall/alignment/models/HYPHY_NUC.csv (used by remap.py:33 through gotoh2.Aligner)
HYPHY_NUC = ([5, -4, -4, -4, 0, -4, 5, -4, -4, 0, -4, -4, 5, -4, 0, -4, -4, -4, 5, 0,
              0, 0, 0, 0, 0], 'ACGT?')


def _cases(golden_dir):
    with open(os.path.join(golden_dir, 'pileup_golden.json')) as f:
        return json.load(f)


def test_golden_sam_to_conseqs(golden_dir):
    data = _cases(golden_dir)
    assert data['n_tests'] >= 30
    for c in data['cases']:
        report = {} if c['distance_report'] is not None else None
        got = oracle.sam_to_conseqs(c['sam'].splitlines(True), c['quality_cutoff'],
                                    seeds=c['seeds'], is_filtered=c['is_filtered'],
                                    filter_coverage=c['filter_coverage'], distance_report=report,
                                    nuc_model=HYPHY_NUC)
        assert got == c['conseqs'], c['sam'][:400]
        assert list(got) == list(c['conseqs'])  # dict order feeds the next mapping pass
        if report is not None:
            assert report == c['distance_report']
