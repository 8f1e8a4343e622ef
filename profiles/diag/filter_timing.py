"""profiles/diag/filter_timing.py -- where the consensus-distance filter's
time goes when the consensuses are long (C4 'all': 24 consensuses up to
SARS-CoV-2's 30 kb): the K x K Gotoh batch on the device, the relevant-seed
extraction, and the K x K edit distances on the host, against the one
device batch the filter now makes of all three (device_batch_ms, checked
equal).  Consensuses are the seeds with
10 % substitutions (the bench's sample genomes).
    python3 profiles/diag/filter_timing.py [repeats]"""
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [REPO, os.path.join(REPO, 'micall-lite_amd')]

from micall_amd import _native, projects  # noqa: E402
from micall_amd.consensus import (FILTER_GEP, FILTER_GOP, HYPHY_NUC, HYPHY_NUC_ALPHABET,  # noqa: E402
                                  clean_sequence, extract_relevant_seed)

NAMES = ['ERCC-00002-seed', 'ERCC-00003-seed', 'ERCC-00007-seed', 'ERCC-00014-seed', 'ERCC-00017-seed',
         'ERCC-00025-seed', 'ERCC-00033-seed', 'ERCC-00099-seed', 'HCV-1a', 'HCV-1b', 'HCV-2c', 'HCV-3i',
         'HCV-4b', 'HCV-5a', 'HCV-6u', 'HCV-7a', 'HIV1B-env-seed', 'HIV1B-gag-seed', 'HIV1B-nef-seed',
         'HIV1B-pol-seed', 'HIV1B-vif-seed', 'HIV1B-vpr-seed', 'HLA-B-seed', 'SARS-CoV-2']
reps = int(sys.argv[1]) if len(sys.argv) > 1 else 3
seeds = projects.load_default().seed_sequences()
rng = np.random.default_rng(1)
cons = {}
for n in NAMES:
    s = np.frombuffer(seeds[n].encode(), dtype=np.uint8).copy()
    sub = rng.random(len(s)) < 0.1
    s[sub] = np.frombuffer(b'ACGT', dtype=np.uint8)[rng.integers(0, 4, int(sub.sum()))]
    cons[n] = s.tobytes().decode()
ctx = _native.Context(0)
jobs = [(n, s) for n in NAMES for s in NAMES]
for rep in range(reps):
    t0 = time.perf_counter()
    inputs = [(clean_sequence(seeds[s]), clean_sequence(cons[n])) for n, s in jobs]
    t1 = time.perf_counter()
    aligned = ctx.gotoh_align_many(inputs, FILTER_GOP, FILTER_GEP, True, HYPHY_NUC_ALPHABET, HYPHY_NUC)
    t2 = time.perf_counter()
    lev_in = [(extract_relevant_seed(a_c, a_s), cons[n]) for (n, _s), (a_s, a_c, _sc) in zip(jobs, aligned)]
    t3 = time.perf_counter()
    d = _native.levenshtein_many(lev_in)
    t4 = time.perf_counter()
    # consensus.filter_conseqs' two phases: own seed + nearest bound, then
    # the others whose bound does not exceed the nearest distance found
    bound = [abs(len(rs) - len(c)) for rs, c in lev_in]
    first = {}
    for k, (n, s) in enumerate(jobs):
        if s != n and (n not in first or bound[k] < bound[first[n]]):
            first[n] = k
    todo = [k for k, (n, s) in enumerate(jobs) if s == n or first.get(n) == k]
    dist = dict(zip(todo, _native.levenshtein_many([lev_in[k] for k in todo])))
    t5 = time.perf_counter()
    near = {jobs[k][0]: dist[k] for k in todo if jobs[k][1] != jobs[k][0]}
    rest = [k for k, (n, s) in enumerate(jobs) if k not in dist and bound[k] <= near[n]]
    dist.update(zip(rest, _native.levenshtein_many([lev_in[k] for k in rest])))
    t6 = time.perf_counter()
    # the filter's own call: alignments, relevant seeds and distances in one
    # device batch (mh_gotoh_distance_batch)
    dd = ctx.gotoh_distance_many([(a, b, cons[n]) for (a, b), (n, _s) in zip(inputs, jobs)],
                                 FILTER_GOP, FILTER_GEP, True, HYPHY_NUC_ALPHABET, HYPHY_NUC)
    t7 = time.perf_counter()
    assert dd == d, 'device distances differ from the host ones'
    print(json.dumps({'rep': rep, 'pairs': len(jobs), 'device_batch_ms': round(1e3 * (t7 - t6), 1),
                      'gotoh_cells_G': round(sum(len(a) * len(b) for a, b in inputs) / 1e9, 2),
                      'lev_cells_G': round(sum(len(a) * len(b) for a, b in lev_in) / 1e9, 2),
                      'clean_ms': round(1e3 * (t1 - t0), 1), 'gotoh_ms': round(1e3 * (t2 - t1), 1),
                      'extract_ms': round(1e3 * (t3 - t2), 1), 'lev_ms': round(1e3 * (t4 - t3), 1),
                      'lev_pruned_ms': [round(1e3 * (t5 - t4), 1), round(1e3 * (t6 - t5), 1)],
                      'lev_pruned_pairs': [len(todo), len(rest)],
                      'dist_sum': int(sum(d))}), flush=True)
# what exact length bounds could skip (d >= len(relevant) - len(seed) before
# the alignment, d >= |len(relevant seed) - len(relevant)| after it): pairs
# whose bound exceeds the name's nearest other seed's distance
best = {}
for (n, s), dist in zip(jobs, d):
    if s != n:
        best[n] = min(best.get(n, 1 << 60), dist)
pre = [(n, s) for (n, s), (a, b) in zip(jobs, inputs) if s != n and len(b) - len(a) > best[n]]
post = [(n, s) for (n, s), (rs, c) in zip(jobs, lev_in) if s != n and abs(len(rs) - len(c)) > best[n]]
cells = {(n, s): len(a) * len(b) for (n, s), (a, b) in zip(jobs, inputs)}
lcells = {(n, s): len(a) * len(b) for (n, s), (a, b) in zip(jobs, lev_in)}
print(json.dumps({'prune_before_alignment': len(pre),
                  'gotoh_cells_G_skipped': round(sum(cells[k] for k in pre) / 1e9, 2),
                  'lev_cells_G_skipped_with_it': round(sum(lcells[k] for k in pre) / 1e9, 2),
                  'prune_after_alignment': len(post),
                  'lev_cells_G_skipped': round(sum(lcells[k] for k in post) / 1e9, 2)}), flush=True)
ctx.close()
