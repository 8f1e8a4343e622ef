"""Where the C4-all filter batch's time goes in k_gotoh_fwd / k_gotoh_bwd:
the 576-alignment batch of filter_timing.py run once with MH_GOTOH_STAMPS
(shader-clock stamps before and after each block's wait, per ticket), then
per pass: the batch span, how many strips hold a wave over time (resident)
and how many of them are computing rather than waiting, and along the
longest alignment's chain of strips the start lag per strip and the
compute / wait cycles per block.
    python3 profiles/diag/gotoh_batch_stamps.py [out.json]"""
import json
import os
import sys
import tempfile

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [REPO, os.path.join(REPO, 'micall-lite_amd')]
path = os.path.join(tempfile.mkdtemp(), 'stamps.bin')

from micall_amd import _native, projects  # noqa: E402
from micall_amd.consensus import (FILTER_GEP, FILTER_GOP, HYPHY_NUC, HYPHY_NUC_ALPHABET,  # noqa: E402
                                  clean_sequence)

out_path = sys.argv[1] if len(sys.argv) > 1 else os.path.join(REPO, 'gpurun_out', 'gotoh_batch_stamps.json')
NAMES = ['ERCC-00002-seed', 'ERCC-00003-seed', 'ERCC-00007-seed', 'ERCC-00014-seed', 'ERCC-00017-seed',
         'ERCC-00025-seed', 'ERCC-00033-seed', 'ERCC-00099-seed', 'HCV-1a', 'HCV-1b', 'HCV-2c', 'HCV-3i',
         'HCV-4b', 'HCV-5a', 'HCV-6u', 'HCV-7a', 'HIV1B-env-seed', 'HIV1B-gag-seed', 'HIV1B-nef-seed',
         'HIV1B-pol-seed', 'HIV1B-vif-seed', 'HIV1B-vpr-seed', 'HLA-B-seed', 'SARS-CoV-2']
seeds = projects.load_default().seed_sequences()
rng = np.random.default_rng(1)
cons = {}
for n in NAMES:
    s = np.frombuffer(seeds[n].encode(), dtype=np.uint8).copy()
    sub = rng.random(len(s)) < 0.1
    s[sub] = np.frombuffer(b'ACGT', dtype=np.uint8)[rng.integers(0, 4, int(sub.sum()))]
    cons[n] = s.tobytes().decode()
jobs = [(clean_sequence(seeds[s]), clean_sequence(cons[n])) for n in NAMES for s in NAMES]
ctx = _native.Context(0)
ctx.gotoh_align_many(jobs, FILTER_GOP, FILTER_GEP, True, HYPHY_NUC_ALPHABET, HYPHY_NUC)   # warm-up
os.environ['MH_GOTOH_STAMPS'] = path
ctx.gotoh_align_many(jobs, FILTER_GOP, FILTER_GEP, True, HYPHY_NUC_ALPHABET, HYPHY_NUC)
ctx.close()
raw = np.fromfile(path, dtype=np.int64)
strips, nb = int(raw[0]), int(raw[1])
st = raw[2:].view(np.uint64).reshape(2, strips, nb, 2).astype(np.int64)
# the host's ticket order (mh_gotoh.hip gotoh_batch_once): key descending, stable
tick, key = [], []
for t, (a, b) in enumerate(jobs):
    nsx = (len(a) + 1 + 63) // 64
    for q in range(nsx):
        tick.append((t, q))
        key.append((nsx - 1 - q) * 128 + len(b) + 64)
order = sorted(range(len(tick)), key=lambda x: -key[x])
tick = [tick[x] for x in order]
assert len(tick) == strips, (len(tick), strips)
longest = max(range(len(jobs)), key=lambda t: (len(jobs[t][0]) + 64) * len(jobs[t][1]))
res = {'strips': strips, 'blocks_cap': nb, 'longest': {'m': len(jobs[longest][0]), 'n': len(jobs[longest][1])}}
for p, name in ((0, 'fwd'), (1, 'bwd')):
    s = st[p]
    used = s[:, :, 0] > 0
    first = np.where(used.any(axis=1), np.where(used, s[:, :, 0], np.iinfo(np.int64).max).min(axis=1), 0)
    last = np.where(used, s[:, :, 1], 0).max(axis=1)
    t_min = first[used.any(axis=1)].min()
    span = int(last.max() - t_min)
    wait = np.where(used, s[:, :, 1] - s[:, :, 0], 0)
    # resident and computing strips over time (100 samples over the span)
    grid = t_min + np.linspace(0, span, 100)
    resident = [int(((first <= g) & (last >= g)).sum()) for g in grid]
    waiting = []
    for g in grid:
        w = (used & (s[:, :, 0] <= g) & (s[:, :, 1] >= g)).any(axis=1)
        waiting.append(int(w.sum()))
    chain = [u for u in range(strips) if tick[u][0] == longest]
    chain.sort(key=lambda u: tick[u][1])
    starts = np.array([first[u] for u in chain])
    comp = []
    for u in chain[len(chain) // 2: len(chain) // 2 + 3]:
        k = int(used[u].sum())
        c = s[u, 1:k, 0] - s[u, :k - 1, 1]
        comp.append(float(np.median(c)))
    res[name] = {
        'span_cycles': span,
        'resident_strips_over_time': resident,
        'waiting_strips_over_time': waiting,
        'chain_strips': len(chain),
        'chain_start_lag_median': float(np.median(np.diff(starts))),
        'chain_first_start': int(starts[0] - t_min),
        'chain_last_end': int(max(last[u] for u in chain) - t_min),
        'chain_mid_comp_per_block_median': comp,
        'chain_mid_wait_per_block_median': [float(np.median(wait[u, 3:int(used[u].sum()) - 2]))
                                            for u in chain[len(chain) // 2: len(chain) // 2 + 3]],
    }
os.makedirs(os.path.dirname(out_path), exist_ok=True)
with open(out_path, 'w') as f:
    json.dump(res, f, indent=1)
print(json.dumps({k: (v if not isinstance(v, dict) else {kk: vv for kk, vv in v.items() if 'over_time' not in kk})
                  for k, v in res.items()}, indent=1))
