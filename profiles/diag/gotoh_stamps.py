"""Where a strip's time goes in k_gotoh_fwd / k_gotoh_bwd: one alignment per
shape run with MH_GOTOH_STAMPS (shader-clock stamps before and after each
block's wait), summarised per pass as: the start lag between consecutive
strips, the mean wait per block and the mean compute per block (middle
strips, first 3 blocks vs the rest; general strips)."""
import json
import os
import sys
import tempfile

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(REPO, 'micall-lite_amd'))
path = os.path.join(tempfile.mkdtemp(), 'stamps.bin')
os.environ['MH_GOTOH_STAMPS'] = path

from micall_amd import _native  # noqa: E402
from micall_amd.consensus import HYPHY_NUC, HYPHY_NUC_ALPHABET  # noqa: E402

rng = np.random.default_rng(7)
ctx = _native.Context(0)
out = {}
for m, n in ((1023, 3000), (3071, 3000)):
    a = ''.join(rng.choice(list('ACGT'), size=m))
    b = ''.join(rng.choice(list('ACGT'), size=n))
    ctx.gotoh_align_many([(a, b)], 15, 3, True, HYPHY_NUC_ALPHABET, HYPHY_NUC)
    ctx.gotoh_align_many([(a, b)], 15, 3, True, HYPHY_NUC_ALPHABET, HYPHY_NUC)
    raw = np.fromfile(path, dtype=np.int64)
    strips, nb = int(raw[0]), int(raw[1])
    st = raw[2:].view(np.uint64).reshape(2, strips, nb, 2).astype(np.int64)
    res = {}
    for p, name in ((0, 'fwd'), (1, 'bwd')):
        s = st[p]
        used = (s[:, :, 0] > 0)
        nblk = used.sum(axis=1)
        t0 = s[:, 0, 0]
        wait = np.where(used, s[:, :, 1] - s[:, :, 0], 0)
        comp = np.zeros_like(wait)
        comp[:, :-1] = np.where(used[:, 1:], s[:, 1:, 0] - s[:, :-1, 1], 0)
        mid = slice(1, strips - 1) if p == 0 else slice(1, strips)   # ticket order
        res[name] = {
            'strips': strips, 'blocks': int(nblk[0]),
            'span_cycles': int(s[:, :, 1][used].max() - t0.min()),
            'start_lag_mean': float(np.diff(np.sort(t0)).mean()),
            'middle_wait_per_block': float(wait[mid, 3:-2].mean()),
            'middle_wait_first3': float(wait[mid, :3].mean()),
            'middle_comp_first3_per_block': float(comp[mid, :3].mean()),
            'middle_comp_rest_per_block': float(comp[mid, 3:-3].mean()),
            'ticket0_comp_per_block': float(comp[0, :-2].mean()),
            'last_ticket_comp_per_block': float(comp[-1, 3:-3].mean()),
            'last_ticket_wait_per_block': float(wait[-1, 3:-3].mean()),
        }
        if m == 3071 and os.environ.get('GOTOH_STAMP_DETAIL'):
            for sidx in (1, 2, 24, strips - 2):
                print(name, sidx, 'wait', (wait[sidx, :nblk[sidx]] // 100).tolist(), file=sys.stderr)
                print(name, sidx, 'comp', (comp[sidx, :nblk[sidx] - 1] // 100).tolist(), file=sys.stderr)
    out['%dx%d' % (m, n)] = res
print(json.dumps(out, indent=1))
