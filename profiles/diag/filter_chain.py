"""profiles/diag/filter_chain.py -- is the filter's K x K batch bound by its
longest alignment's chain of strips or by the batch's total cells?  Device
time per kernel of: SARS-CoV-2's consensus against its own seed alone; the
batch without any SARS-CoV-2 pair; the batch without the self pair; the
full batch (C4-all's 24 consensuses, as filter_phases.py).
    python3 profiles/diag/filter_chain.py [repeats]"""
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [REPO, os.path.join(REPO, 'micall-lite_amd'), os.path.join(REPO, 'profiles', 'diag')]

from filter_phases import NAMES, clean, ctx, crel, kern, rel  # noqa: E402  (builds the consensuses)
from micall_amd.consensus import FILTER_GEP, FILTER_GOP, HYPHY_NUC, HYPHY_NUC_ALPHABET  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 2
S = 'SARS-CoV-2'
sets = {'sars_self': [(S, S)],
        'no_sars': [(n, s) for n in NAMES for s in NAMES if S not in (n, s)],
        'sars_row_col': [(n, s) for n in NAMES for s in NAMES if S in (n, s)],
        'full_but_self': [(n, s) for n in NAMES for s in NAMES if (n, s) != (S, S)],
        'full': [(n, s) for n in NAMES for s in NAMES]}
ctx.profile(True)
for rep in range(reps):
    out = {}
    for name, jobs in sets.items():
        kern()
        t = time.perf_counter()
        ctx.gotoh_distance_many([(clean[s], crel[n], rel[n]) for n, s in jobs], FILTER_GOP, FILTER_GEP, True,
                                HYPHY_NUC_ALPHABET, HYPHY_NUC)
        out[name] = dict(ms=round((time.perf_counter() - t) * 1e3, 2), **kern())
    print(json.dumps(out), flush=True)
