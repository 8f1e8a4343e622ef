"""profiles/diag/gotoh_sars_stamps.py -- the stamps of gotoh_stamps.py for
the filter's longest alignment alone (C4-all's SARS-CoV-2 consensus against
its 30 kb seed, global, HYPHY_NUC): start lag between consecutive strips,
wait and compute per block, the span, for k_gotoh_fwd and k_gotoh_bwd."""
import json
import os
import sys
import tempfile

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [REPO, os.path.join(REPO, 'micall-lite_amd'), os.path.join(REPO, 'profiles', 'diag')]
path = os.path.join(tempfile.mkdtemp(), 'stamps.bin')
os.environ['MH_GOTOH_STAMPS'] = path

from filter_phases import clean, crel, ctx  # noqa: E402
from micall_amd.consensus import HYPHY_NUC, HYPHY_NUC_ALPHABET  # noqa: E402

S = 'SARS-CoV-2'
out = {}
for rep in range(2):
    ctx.gotoh_align_many([(clean[S], crel[S])], 15, 3, True, HYPHY_NUC_ALPHABET, HYPHY_NUC)
raw = np.fromfile(path, dtype=np.int64)
strips, nb = int(raw[0]), int(raw[1])
st = raw[2:].view(np.uint64).reshape(2, strips, nb, 2).astype(np.int64)
for p, name in ((0, 'fwd'), (1, 'bwd')):
    s = st[p]
    used = s[:, :, 0] > 0
    nblk = used.sum(axis=1)
    t0 = s[:, 0, 0]
    wait = np.where(used, s[:, :, 1] - s[:, :, 0], 0)
    comp = np.zeros_like(wait)
    comp[:, :-1] = np.where(used[:, 1:], s[:, 1:, 0] - s[:, :-1, 1], 0)
    mid = slice(1, strips - 1)
    end = np.where(used, s[:, :, 1], 0).max(axis=1)
    out[name] = {
        'strips': strips, 'blocks': int(nblk.max()),
        'span_cycles': int(end.max() - t0.min()),
        'start_lag_mean': float(np.diff(np.sort(t0)).mean()),
        'strip_life_mean': float((end - t0).mean()),
        'middle_wait_per_block': float(wait[mid, 3:-2].mean()),
        'middle_comp_per_block': float(comp[mid, 3:-3].mean()),
        'ticket0_comp_per_block': float(comp[0, :-2].mean()),
        'wait_by_strip_decile': [float(wait[q, 3:-2].mean()) for q in np.linspace(1, strips - 2, 10).astype(int)],
        'comp_by_strip_decile': [float(comp[q, 3:-3].mean()) for q in np.linspace(1, strips - 2, 10).astype(int)],
        'first_blocks_wait_mean': [float(wait[mid, b].mean()) for b in range(6)],
        'first_blocks_comp_mean': [float(comp[mid, b].mean()) for b in range(6)],
        'life_minus_steady': float((end - t0).mean() - nblk.mean() * (comp[mid, 3:-3].mean() + wait[mid, 3:-2].mean())),
    }
    if os.environ.get('GOTOH_STAMP_DETAIL'):
        for q in (1, 100, 234, 400, strips - 2):
            print(name, q, 'comp', (comp[q, :nblk[q] - 1:25] // 100).tolist(), file=sys.stderr)
            print(name, q, 'wait', (wait[q, :nblk[q]:25] // 100).tolist(), file=sys.stderr)
print(json.dumps(out, indent=1))
