"""profiles/diag/filter_phases.py -- the consensus-distance filter's device
time by phase at C4-all size (24 consensuses up to SARS-CoV-2's 30 kb: the
seeds with 10 % substitutions, as filter_timing.py): the full K x K batch
against the pruned filter's bound batch, its first (own + least-bound
seed) and second (bound <= least distance) alignment batches; the pruned
decisions checked equal to the full batch's.
The pruned filter was measured slower than the full batch and not kept:
main() needs profiles/r06/diag/filter_bound_rejected.patch applied (the
bound batch, ctx.lev_bound_many); the consensuses, kern() and the context
are imported by filter_chain.py and filter_profile_lds.py.
    python3 profiles/diag/filter_phases.py [repeats]"""
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [REPO, os.path.join(REPO, 'micall-lite_amd')]

from micall_amd import _native, projects  # noqa: E402
from micall_amd.consensus import (FILTER_GEP, FILTER_GOP, HYPHY_NUC, HYPHY_NUC_ALPHABET,  # noqa: E402
                                  clean_sequence)

NAMES = ['ERCC-00002-seed', 'ERCC-00003-seed', 'ERCC-00007-seed', 'ERCC-00014-seed', 'ERCC-00017-seed',
         'ERCC-00025-seed', 'ERCC-00033-seed', 'ERCC-00099-seed', 'HCV-1a', 'HCV-1b', 'HCV-2c', 'HCV-3i',
         'HCV-4b', 'HCV-5a', 'HCV-6u', 'HCV-7a', 'HIV1B-env-seed', 'HIV1B-gag-seed', 'HIV1B-nef-seed',
         'HIV1B-pol-seed', 'HIV1B-vif-seed', 'HIV1B-vpr-seed', 'HLA-B-seed', 'SARS-CoV-2']
reps = int(sys.argv[1]) if len(sys.argv) > 1 else 3
seeds = projects.load_default().seed_sequences()
rng = np.random.default_rng(1)
rel = {}
for n in NAMES:
    s = np.frombuffer(seeds[n].encode(), dtype=np.uint8).copy()
    sub = rng.random(len(s)) < 0.1
    s[sub] = np.frombuffer(b'ACGT', dtype=np.uint8)[rng.integers(0, 4, int(sub.sum()))]
    rel[n] = s.tobytes().decode()
clean = {n: clean_sequence(seeds[n]) for n in NAMES}
crel = {n: clean_sequence(rel[n]) for n in NAMES}
ctx = _native.Context(0)


def measure(jobs):
    return dict(zip(jobs, ctx.gotoh_distance_many([(clean[s], crel[n], rel[n]) for n, s in jobs],
                                                  FILTER_GOP, FILTER_GEP, True, HYPHY_NUC_ALPHABET,
                                                  HYPHY_NUC)))


KERNELS = ('k_gotoh_fwd', 'k_gotoh_bwd', 'k_gotoh', 'k_lev', 'k_lev_bound')


def kern():
    """device ms per kernel since the last call (HIP events), then reset"""
    out = {k: round(ctx.profile_get(k)[0], 2) for k in KERNELS}
    ctx.profile(True)
    return {k: v for k, v in out.items() if v}


def cells(jobs):
    return sum(len(rel[n]) * len(seeds[s]) for n, s in jobs)


def main():
  runs = []
  ctx.profile(True)
  for rep in range(reps):
      r = {}
      full = [(n, s) for n in NAMES for s in NAMES]
      t = time.perf_counter()
      dfull = measure(full)
      r['full_ms'] = (time.perf_counter() - t) * 1e3
      r['full_kernels'] = kern()
      pairs = [(n, s) for n in NAMES for s in NAMES if s != n]
      t = time.perf_counter()
      bound = dict(zip(pairs, ctx.lev_bound_many([(rel[n], clean[s]) for n, s in pairs], HYPHY_NUC_ALPHABET)))
      r['bound_ms'] = (time.perf_counter() - t) * 1e3
      r['bound_kernels'] = kern()
      first = []
      for n in NAMES:
          first += [(n, n), min(((n, s) for s in NAMES if s != n), key=bound.__getitem__)]
      t = time.perf_counter()
      dist = measure(first)
      r['first_ms'] = (time.perf_counter() - t) * 1e3
      r['first_kernels'] = kern()
      rest = []
      for n in NAMES:
          least = min(dist[(n, s)] for s in NAMES if s != n and (n, s) in dist)
          rest += [(n, s) for s in NAMES if s != n and (n, s) not in dist and bound[(n, s)] <= least]
      t = time.perf_counter()
      dist.update(measure(rest) if rest else {})
      r['second_ms'] = (time.perf_counter() - t) * 1e3
      r['second_kernels'] = kern()
      r.update(first_pairs=len(first), first_cells=cells(first), second_pairs=len(rest), second_cells=cells(rest),
               full_cells=cells(full))
      ok = all(dfull[p] >= bound[p] for p in pairs)
      for n in NAMES:
          f = min((dfull[(n, s)], NAMES.index(s)) for s in NAMES if s != n)
          p = min((dist[(n, s)], NAMES.index(s)) for s in NAMES if s != n and (n, s) in dist)
          ok &= f == p and dfull[(n, n)] == dist[(n, n)]
      r['pruned_equals_full'] = bool(ok)
      runs.append({k: round(v, 2) if isinstance(v, float) else v for k, v in r.items()})
      print(json.dumps(runs[-1]), flush=True)


if __name__ == '__main__':
    main()
