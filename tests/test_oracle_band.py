"""The oracle mapper's DP band (og_mapper.c og_band_half) against a plain
restatement of bowtie2's rule: the seed extension's DP rectangle reaches
maxgap = min(max(read gaps, ref gaps), maxhalf = 15) diagonals either side
of the seed diagonal, with the gap counts from the score budget between the
perfect score and --score-min (bowtie2 Scoring::maxReadGaps / maxRefGaps,
DynProgFramer::frameSeedExtensionRect).  CPU only."""
import math

import pytest

import oracle


def _min_score(mode, length):
    if mode == oracle.LOCAL:
        return max(0, int(20.0 + 8.0 * math.log(max(length, 1))))
    return min(0, int(-0.6 + -0.6 * length))


def _max_gaps(perfect, minsc, gap_open, gap_ext):
    # the first gap costs open + extend, each further one extend
    sc, num = perfect, 0
    while sc >= minsc:
        sc -= gap_open + gap_ext if num == 0 else gap_ext
        num += 1
    return num - 1


def _band_half(mode, rdg, rfg, length):
    perfect = 2 * length if mode == oracle.LOCAL else 0
    minsc = _min_score(mode, length)
    gaps = max(_max_gaps(perfect, minsc, *rdg), _max_gaps(perfect, minsc, *rfg))
    return max(0, min(15, gaps))


@pytest.mark.parametrize('mode', [oracle.E2E, oracle.LOCAL])
@pytest.mark.parametrize('rdg,rfg', [((10, 3), (10, 3)), ((4, 3), (14, 2)), ((20, 5), (6, 1))])
def test_band_half_matches_bowtie2_rule(mode, rdg, rfg):
    par = oracle.params(mode, rdg=rdg, rfg=rfg)
    for length in list(range(0, 130)) + [150, 200, 251, 300, 1024]:
        assert oracle.band_half(par, length) == _band_half(mode, rdg, rfg, length), (mode, length)


def test_band_half_at_micall_settings():
    """2x251 reads with MiCall's --rdg/--rfg 10,3: the full maxhalf of 15 in
    both modes; 50-nt reads end-to-end get 6 (budget 30: 13 + 5 x 3 = 28)."""
    for mode in (oracle.E2E, oracle.LOCAL):
        assert oracle.band_half(oracle.params(mode), 251) == 15
    assert oracle.band_half(oracle.params(oracle.E2E), 50) == 6
