"""k_gotoh timing: the C4 filter's shape (6 consensus x 6 seeds of the HIV-1
seeds, global, gop 15 / gep 3, HYPHY_NUC) in one mh_gotoh_align_batch, and
one pol-sized alignment alone; HIP-event kernel time (mh_profile)."""
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(REPO, 'micall-lite_amd'))

from micall_amd import _native, projects, synth  # noqa: E402
from micall_amd.consensus import HYPHY_NUC, HYPHY_NUC_ALPHABET  # noqa: E402

seeds = projects.load_default().seed_sequences()
names = ['HIV1B-env-seed', 'HIV1B-gag-seed', 'HIV1B-nef-seed', 'HIV1B-pol-seed', 'HIV1B-vif-seed',
         'HIV1B-vpr-seed']
rng = np.random.default_rng(5)
cons = {k: synth.sample_genome(seeds[k], rng, 0.08, 0.004).tobytes().decode() for k in names}
pairs = [(seeds[s], cons[c]) for c in names for s in names]
ctx = _native.Context(0)
ctx.profile(True)
out = {}
for label, batch in (('filter_36', pairs), ('pol_1', [(seeds['HIV1B-pol-seed'], cons['HIV1B-pol-seed'])])):
    ctx.gotoh_align_many(batch, 15, 3, True, HYPHY_NUC_ALPHABET, HYPHY_NUC)   # warm-up
    kern = ('k_gotoh_fwd', 'k_gotoh_bwd', 'k_gotoh')   # strips forward, backward, traceback
    before = {k: ctx.profile_get(k)[0] for k in kern}
    t0 = time.perf_counter()
    reps = 3
    for _ in range(reps):
        ctx.gotoh_align_many(batch, 15, 3, True, HYPHY_NUC_ALPHABET, HYPHY_NUC)
    wall = (time.perf_counter() - t0) / reps
    ms = {k: (ctx.profile_get(k)[0] - before[k]) / reps for k in kern}
    out[label] = {'alignments': len(batch), 'cells': int(sum(len(a) * len(b) for a, b in batch)),
                  'k_gotoh_ms': round(sum(ms.values()), 3),
                  'parts_ms': {k: round(v, 3) for k, v in ms.items()}, 'call_ms': round(wall * 1e3, 3)}
print(json.dumps(out))
