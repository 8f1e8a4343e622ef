"""profiles/diag/filter_batch_once.py -- one full C4-all filter batch (the
24 consensuses of filter_phases.py against their 24 seeds), for a PMC pass
over k_gotoh_fwd / k_gotoh_bwd / k_gotoh_tb / k_lev."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [REPO, os.path.join(REPO, 'micall-lite_amd'), os.path.join(REPO, 'profiles', 'diag')]

from filter_phases import NAMES, clean, ctx, crel, rel  # noqa: E402
from micall_amd.consensus import FILTER_GEP, FILTER_GOP, HYPHY_NUC, HYPHY_NUC_ALPHABET  # noqa: E402

jobs = [(n, s) for n in NAMES for s in NAMES]
d = ctx.gotoh_distance_many([(clean[s], crel[n], rel[n]) for n, s in jobs], FILTER_GOP, FILTER_GEP, True,
                            HYPHY_NUC_ALPHABET, HYPHY_NUC)
print(sum(d))
