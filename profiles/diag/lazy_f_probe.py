"""Diagnostics (CPU): how often could a lazy deletion move skip k_dp's
prefix-max scan exactly?  Builds the oracle mapper with -DOG_ROW_PROBE and
lazy_f_probe.c into _ab/lazyf/liboracle.so, maps the first pairs of the
bench's own input (C2: 2x251 pol pairs; C5: unpaired 1x300) in both modes,
and prints the per-row counts of lazy_f_probe.c as JSON.

    python profiles/diag/lazy_f_probe.py [pairs]
"""
import ctypes
import json
import os
import subprocess
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [REPO, os.path.join(REPO, 'oracle'), os.path.join(REPO, 'micall-lite_amd')]
OUT = os.path.join(REPO, '_ab', 'lazyf', 'liboracle.so')
KEYS = ['rows', 'mono', 'fwin', 'gate1', 'gate1_bad', 'fb_live', 'lanes', 'lanes_fwin']


def build():
    os.makedirs(os.path.dirname(OUT), exist_ok=True)
    src = [os.path.join(REPO, 'oracle', f) for f in ('og_gotoh.c', 'og_mapper.c', 'og_pileup.c')]
    subprocess.run(['gcc', '-O2', '-fPIC', '-fopenmp', '-shared', '-DOG_ROW_PROBE', '-o', OUT] + src +
                   [os.path.join(REPO, 'profiles', 'diag', 'lazy_f_probe.c'), '-lm'], check=True)


def main():
    pairs = int(sys.argv[1]) if len(sys.argv) > 1 else 20000
    build()
    import oracle
    oracle.LIB_PATH = OUT
    L = oracle.lib()
    L.og_row_probe_get.argtypes = [ctypes.POINTER(ctypes.c_uint64)]
    import bench
    import cpu_pipeline
    from micall_amd import projects
    seeds = projects.load_default().seed_sequences()
    res = {}
    for shape, kw in (('c2_2x251', dict(read_len=251, paired=True)),
                      ('c5_1x300', dict(read_len=300, paired=False))):
        reads, quals = bench.make_reads(pairs, block=0, **kw)
        for mode, refs in (('e2e_74_seeds', list(seeds.values())),
                           ('local_pol', [seeds['HIV1B-pol-seed']])):
            L.og_row_probe_reset()
            cpu_pipeline.map_arrays(refs, oracle.E2E if mode.startswith('e2e') else oracle.LOCAL,
                                    reads, quals, kw['paired'], os.cpu_count())
            out = (ctypes.c_uint64 * 8)()
            L.og_row_probe_get(out)
            c = dict(zip(KEYS, [int(v) for v in out]))
            r = max(c['rows'], 1)
            c['frac'] = {k: round(c[k] / r, 4) for k in ('mono', 'fwin', 'gate1', 'gate1_bad', 'fb_live')}
            c['frac']['lanes_fwin'] = round(c['lanes_fwin'] / max(c['lanes'], 1), 4)
            res['{}/{}'.format(shape, mode)] = c
            print(shape, mode, json.dumps(c), flush=True)
    with open(os.path.join(REPO, 'profiles', 'diag', 'lazy_f_probe.json'), 'w') as f:
        json.dump({'pairs': pairs, 'results': res}, f, indent=1)


if __name__ == '__main__':
    main()
