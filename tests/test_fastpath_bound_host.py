"""The round-6 fast-path bound on the host (CPU): the counterexamples in
tests/golden/fastpath_two_diagonal.json are extensions where round 5's
local-mode fast path accepted the seeded diagonal's cell although a path
between two other diagonals scores higher.  With the
restatement of the kernel's decision and of the oracle's full DP in
profiles/diag/fastpath_search.py: round 5's rule accepts each one with the
recorded cell, the full DP finds the recorded better cell, and round 6's
rule (k_dp ungapped_wide, scan_run) declines every one.  The GPU side of
the same fixtures is tests/test_gpu_fastpath.py."""
import importlib.util
import json
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
_spec = importlib.util.spec_from_file_location(
    'fastpath_search', os.path.join(HERE, '..', 'profiles', 'diag', 'fastpath_search.py'))
fs = importlib.util.module_from_spec(_spec)
_spec.loader.exec_module(fs)


def test_round5_counterexamples_are_declined_by_round6():
    with open(os.path.join(HERE, 'golden', 'fastpath_two_diagonal.json')) as f:
        cases = json.load(f)['cases']
    assert len(cases) >= 10
    code = {c: i for i, c in enumerate('ACGT')}
    for c in cases:
        r = np.array([code[x] for x in c['read']])
        g = np.array([code[x] for x in c['ref']])
        pens = np.array([fs.pen(x) for x in c['qual']])
        m = len(r)
        s = fs.scores(r, pens, g, c['centre'], m)
        acc = fs.fast_path(s, m, fs.wide_r05)
        assert acc is not None and [acc[0], acc[1], fs.HALF] == c['r05']
        assert list(fs.full_dp(s, m)) == c['full']
        assert c['full'][0] > acc[0] or c['full'][1:] != c['r05'][1:]
        assert fs.fast_path(s, m, fs.wide_r06) is None


def test_round6_keeps_most_acceptances():
    """The bound is not a blanket refusal: on the search's own adversarial
    family round 6 still accepts most of what round 5 did, and every cell
    it accepts is the full DP's."""
    rng = np.random.default_rng(11)
    acc5 = acc6 = 0
    for _ in range(400):
        r, q, g, c0 = fs.candidate(rng)
        m = len(r)
        pens = np.array([fs.pen(x) for x in q])
        s = fs.scores(r, pens, g, c0, m)
        if fs.fast_path(s, m, fs.wide_r05) is not None:
            acc5 += 1
        a6 = fs.fast_path(s, m, fs.wide_r06)
        if a6 is not None:
            acc6 += 1
            assert list(fs.full_dp(s, m)) == [a6[0], a6[1], fs.HALF]
    assert acc5 > 50 and acc6 > 0.7 * acc5, (acc5, acc6)
