"""profiles/diag/filter_prune_eval.py -- what an exact lower bound prunes
from the consensus-distance filter's K x K batch (CPU, oracle only).

The filter (remap.py:228-268) needs, per consensus i, d(i, i) and the least
d(i, j) over the other seeds j (its first arg-min in name order), where
d(i, j) = Levenshtein(relevant seed of the Gotoh alignment of seed j
against the relevant consensus i, relevant consensus i).  The relevant
seed is a substring of seed j, so d(i, j) >= LB(i, j) = the least edit
distance between relevant consensus i and any substring of seed j
(og_levenshtein_infix).  Phase B computes d(i, i) and d(i, j*) for
j* = argmin LB; phase C every other j with LB(i, j) <= min d found.
Consensuses: the seeds with 10 % substitutions (as filter_timing.py).
Prints the cells (m x n) each phase aligns against the full batch, and
checks the pruned decisions against all K x K distances.
Needs profiles/r06/diag/filter_bound_rejected.patch applied (the oracle's
og_levenshtein_infix); the pruning was measured slower on the device and
not kept ("Round 6: the filter batch").
    python3 profiles/diag/filter_prune_eval.py [threads]"""
import json
import os
import sys
import time
from concurrent.futures import ThreadPoolExecutor

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(REPO, 'oracle'), REPO, os.path.join(REPO, 'micall-lite_amd')]

import oracle  # noqa: E402
from cpu_e2e import HYPHY_NUC  # noqa: E402
from micall_amd import projects  # noqa: E402

NAMES = ['ERCC-00002-seed', 'ERCC-00003-seed', 'ERCC-00007-seed', 'ERCC-00014-seed', 'ERCC-00017-seed',
         'ERCC-00025-seed', 'ERCC-00033-seed', 'ERCC-00099-seed', 'HCV-1a', 'HCV-1b', 'HCV-2c', 'HCV-3i',
         'HCV-4b', 'HCV-5a', 'HCV-6u', 'HCV-7a', 'HIV1B-env-seed', 'HIV1B-gag-seed', 'HIV1B-nef-seed',
         'HIV1B-pol-seed', 'HIV1B-vif-seed', 'HIV1B-vpr-seed', 'HLA-B-seed', 'SARS-CoV-2']
threads = int(sys.argv[1]) if len(sys.argv) > 1 else 8
matrix, alphabet = HYPHY_NUC
seeds = projects.load_default().seed_sequences()
rng = np.random.default_rng(1)
rel = {}
for n in NAMES:
    s = np.frombuffer(seeds[n].encode(), dtype=np.uint8).copy()
    sub = rng.random(len(s)) < 0.1
    s[sub] = np.frombuffer(b'ACGT', dtype=np.uint8)[rng.integers(0, 4, int(sub.sum()))]
    rel[n] = s.tobytes().decode()
clean = {n: oracle.clean_sequence(seeds[n], alphabet) for n in NAMES}
pairs = [(i, j) for i in NAMES for j in NAMES]


def dist(p):
    i, j = p
    a_seed, a_con, _ = oracle.gotoh_align(clean[j], oracle.clean_sequence(rel[i], alphabet), 15, 3, True,
                                          alphabet, matrix)
    return oracle.levenshtein(oracle.extract_relevant_seed(a_con, a_seed), rel[i])


def cells(ps):
    return sum(len(rel[i]) * len(seeds[j]) for i, j in ps)


t0 = time.time()
big = sorted(pairs, key=lambda p: -len(rel[p[0]]) * len(seeds[p[1]]))
with ThreadPoolExecutor(threads) as pool:
    lb = dict(zip(big, pool.map(lambda p: oracle.levenshtein_infix(rel[p[0]], clean[p[1]]), big)))
    t1 = time.time()
    d = dict(zip(big, pool.map(dist, big)))
t2 = time.time()
assert all(d[p] >= lb[p] for p in pairs), 'bound violated'
# phases
phase_b = []
for i in NAMES:
    others = [j for j in NAMES if j != i]
    jstar = min(others, key=lambda j: (lb[(i, j)], NAMES.index(j)))
    phase_b += [(i, i), (i, jstar)]
done = set(phase_b)
phase_c = []
for i in NAMES:
    t = min(d[(i, j)] for j in NAMES if j != i and (i, j) in done)
    phase_c += [(i, j) for j in NAMES if j != i and (i, j) not in done and lb[(i, j)] <= t]
done |= set(phase_c)
ok = True
for i in NAMES:
    full = [(j, d[(i, j)]) for j in NAMES if j != i]
    od = min(x for _, x in full)
    os_ = next(j for j, x in full if x == od)
    pr = [(j, d[(i, j)]) for j in NAMES if j != i and (i, j) in done]
    pd = min(x for _, x in pr)
    ps = next(j for j, x in pr if x == pd)
    ok &= (od, os_) == (pd, ps)
out = {'lb_seconds': round(t1 - t0, 1), 'align_seconds': round(t2 - t1, 1),
       'full_pairs': len(pairs), 'full_cells': cells(pairs),
       'phase_b_pairs': len(phase_b), 'phase_b_cells': cells(phase_b),
       'phase_c_pairs': len(phase_c), 'phase_c_cells': cells(phase_c),
       'phase_c': phase_c, 'pruned_equals_full': ok,
       'per_consensus': {i: {'seed_dist': d[(i, i)], 'lb_self': lb[(i, i)],
                             'other': min((d[(i, j)], j) for j in NAMES if j != i),
                             'lb_min_other': min((lb[(i, j)], j) for j in NAMES if j != i)} for i in NAMES}}
print(json.dumps(out, indent=1))
