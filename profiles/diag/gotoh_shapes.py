"""k_gotoh_fwd / k_gotoh_bwd time against the grid's shape, to split a
strip's per-step cost from the lag between strips: one alignment of random
nucleotides per shape (global, gop 15 / gep 3, HYPHY_NUC).  A wide shape
(2 strips, n columns) prices a step; a tall one (many strips, few columns)
prices the lag."""
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(REPO, 'micall-lite_amd'))

from micall_amd import _native  # noqa: E402
from micall_amd.consensus import HYPHY_NUC, HYPHY_NUC_ALPHABET  # noqa: E402

rng = np.random.default_rng(7)


def seq(n):
    return ''.join(rng.choice(list('ACGT'), size=n))


ctx = _native.Context(0)
ctx.profile(True)
out = {}
kern = ('k_gotoh_fwd', 'k_gotoh_bwd', 'k_gotoh')
for m, n in ((127, 3000), (127, 12000), (1023, 3000), (64 * 48 - 1, 200), (64 * 48 - 1, 3000)):
    batch = [(seq(m), seq(n))]
    ctx.gotoh_align_many(batch, 15, 3, True, HYPHY_NUC_ALPHABET, HYPHY_NUC)
    before = {k: ctx.profile_get(k)[0] for k in kern}
    reps = 3
    for _ in range(reps):
        ctx.gotoh_align_many(batch, 15, 3, True, HYPHY_NUC_ALPHABET, HYPHY_NUC)
    ms = {k: round((ctx.profile_get(k)[0] - before[k]) / reps, 4) for k in kern}
    out['%dx%d' % (m, n)] = ms
print(json.dumps(out))
