"""consensus.filter_conseqs (one batch of alignments and edit distances,
each sequence cleaned once) against the reference's loop over every seed
(remap.py:231-262: the first other seed in name order with the smallest
distance) on sets with lengths far apart and with ties (copies of one
sequence): the same decisions and distance report.  CPU: the
distances come from the oracle's Gotoh and Levenshtein (test
infrastructure) through a stand-in context; tests/test_gpu_parity.py holds
the device batch to the same oracle."""
import random

import numpy as np
import pytest

import oracle
from micall_amd.consensus import (FILTER_GEP, FILTER_GOP, HYPHY_NUC, HYPHY_NUC_ALPHABET,
                                  clean_sequence, extract_relevant_seed, filter_conseqs)


class _OracleAligner:
    """Stands in for the context's gotoh_distance_many (the device batch):
    the oracle's alignment, relevant seed and edit distance per triple."""
    def gotoh_distance_many(self, triples, gop, gep, is_global, alphabet, matrix):
        out = []
        for a, b, text in triples:
            a_seed, a_conseq, _ = oracle.gotoh_align(a, b, gop, gep, is_global, alphabet, list(matrix))
            out.append(oracle.levenshtein(extract_relevant_seed(a_conseq, a_seed), text))
        return out


class _FullCoverage:
    def __init__(self, names):
        self.refnames = list(names)

    def position_sums(self, r, seed, length):
        return np.full(length, 100, dtype=np.int64)


def _reference_loop(new_conseqs, seeds):
    """remap.py:231-262 over every seed (no pruning), oracle Levenshtein."""
    report, kept = {}, {}
    for name in sorted(new_conseqs):
        relevant = new_conseqs[name]
        seed_dist = other_dist = other_seed = None
        for seed_name in sorted(new_conseqs):
            a_seed, a_conseq, _ = oracle.gotoh_align(
                clean_sequence(seeds[seed_name]), clean_sequence(relevant), FILTER_GOP, FILTER_GEP,
                True, HYPHY_NUC_ALPHABET, HYPHY_NUC)
            d = oracle.levenshtein(extract_relevant_seed(a_conseq, a_seed), relevant)
            if seed_name == name:
                seed_dist = d
            elif other_dist is None or d < other_dist:
                other_seed, other_dist = seed_name, d
        if seed_dist <= other_dist:
            kept[name] = relevant
        report[name] = dict(seed_dist=seed_dist, other_dist=other_dist, other_seed=other_seed)
    return kept, report


def _mutate(rng, s, rate):
    return ''.join(rng.choice('ACGT') if rng.random() < rate else c for c in s)


@pytest.mark.parametrize('seed', range(6))
def test_pruned_filter_equals_the_full_loop(seed):
    rng = random.Random(seed)
    base = ''.join(rng.choice('ACGT') for _ in range(900))
    seeds = {
        'A-long': base + ''.join(rng.choice('ACGT') for _ in range(600)),
        'B-short': base[100:220],
        'C-mid': _mutate(rng, base[:700], 0.05),
        'D-copy': base[:700],          # two seeds at one distance: ties
        'E-copy': base[:700],
        'F-tiny': base[400:430],
    }
    names = sorted(seeds)
    new_conseqs = {n: _mutate(rng, seeds[n], 0.08) for n in names}
    order = list(range(len(names)))
    report = {}
    kept = filter_conseqs(_OracleAligner(), _FullCoverage(names), order, new_conseqs, seeds, 1,
                          report)
    want_kept, want_report = _reference_loop(new_conseqs, seeds)
    assert report == want_report
    assert kept == want_kept
