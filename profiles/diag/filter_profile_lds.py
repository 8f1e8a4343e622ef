"""profiles/diag/filter_profile_lds.py -- k_gotoh_fwd with the score profile
in LDS (one 64-lane strip per workgroup, up to 64 KiB of LDS each) against
the profile streamed from global memory, on filter batches whose profiles
fit the LDS: C4-all's pairs without SARS-CoV-2 (HCV seeds, 48 KiB
profiles), the HIV-only pairs (C4), and single small alignments.
    python3 profiles/diag/filter_profile_lds.py [repeats]"""
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [REPO, os.path.join(REPO, 'micall-lite_amd'), os.path.join(REPO, 'profiles', 'diag')]

from filter_phases import NAMES, clean, ctx, crel, kern, rel  # noqa: E402
from micall_amd.consensus import FILTER_GEP, FILTER_GOP, HYPHY_NUC, HYPHY_NUC_ALPHABET  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 2
S = 'SARS-CoV-2'
hiv = [n for n in NAMES if n.startswith('HIV')]
sets = {'no_sars': [(n, s) for n in NAMES for s in NAMES if S not in (n, s)],
        'hcv': [(n, s) for n in NAMES for s in NAMES if n.startswith('HCV') and s.startswith('HCV')],
        'hiv': [(n, s) for n in hiv for s in hiv]}
ctx.profile(True)
for rep in range(reps):
    for limit in ('65536', '0'):
        os.environ['MH_GOTOH_PROF_LDS_MAX'] = limit
        out = {'lds_max': limit}
        for name, jobs in sets.items():
            kern()
            t = time.perf_counter()
            got = ctx.gotoh_distance_many([(clean[s], crel[n], rel[n]) for n, s in jobs], FILTER_GOP, FILTER_GEP,
                                          True, HYPHY_NUC_ALPHABET, HYPHY_NUC)
            out[name] = dict(ms=round((time.perf_counter() - t) * 1e3, 2), sum=sum(got), **kern())
        print(json.dumps(out), flush=True)
