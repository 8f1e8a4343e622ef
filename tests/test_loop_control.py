"""Remap loop control (remap.py:544-606) of RemapPipeline.run, with the
mapping and consensus steps scripted: the reference's three stopping rules,
the max_iterations cap of the benchmark configs and the min_iterations
forcing of BASELINE C3 ("3 remap iterations", bench.py --force-iterations)."""
from collections import Counter

from micall_amd.pipeline import RemapPipeline


class _Scripted(RemapPipeline):
    """Every mapping pass maps `mapped[i]` lines to one reference 'R'; the
    consensus set never changes."""

    def __init__(self, mapped, prelim_count=10):
        self.mapped = list(mapped)
        self.prelim_count = prelim_count
        self.passes = 0
        self.log = []
        self.callback = None
        self.shard = None

    def prelim(self):
        return None

    def prelim_groups(self):
        return [('R', self.prelim_count, self.prelim_count)]

    def select_seeds(self, groups):
        return {'R': self.prelim_count}

    def prelim_conseqs(self, seed_counts):
        return {'R': 'ACGT'}, {'R': self.prelim_count}

    def map_to_reference(self, refseqs):
        n = self.mapped[min(self.passes, len(self.mapped) - 1)]
        self.passes += 1
        return Counter({'R': n}), 0

    def build_conseqs_filtered(self, refseqs, distance_report=None):
        return {'R': 'ACGT'}


def test_stops_when_counts_do_not_grow():
    # pass 1 maps 8 <= prelim 10: same seeds, no growth -> stop (remap.py:586-588)
    p = _Scripted([8, 50, 60])
    p.run(raw_count=100)
    assert p.passes == 1


def test_stops_on_mapping_efficiency():
    # counts grow (20 > 10) but 96 / 100 > 0.95 -> stop after the second pass
    p = _Scripted([20, 96, 97])
    p.run(raw_count=100)
    assert p.passes == 2


def test_stops_at_max_remaps():
    # growing counts, low efficiency: the reference's MAX_REMAPS (3) ends it
    p = _Scripted([20, 30, 40, 50, 60])
    p.run(raw_count=1000)
    assert p.passes == 3


def test_max_iterations_caps_passes():
    p = _Scripted([20, 30, 40, 50, 60])
    p.run(raw_count=1000, max_iterations=1)
    assert p.passes == 1


def test_min_iterations_forces_passes():
    # the rules would stop after pass 1 (100 % mapped); C3 forces three passes
    p = _Scripted([100, 100, 100, 100])
    p.run(raw_count=100, max_iterations=3, min_iterations=3)
    assert p.passes == 3
    assert [e['iteration'] for e in p.log] == [1, 2, 3]
