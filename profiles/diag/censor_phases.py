"""profiles/diag/censor_phases.py -- the censor drop-in's phases on the C2
R1 file (single gzip member, as bcl2fastq writes it): staging (mmap +
inflate), mh_censor_staged (split, k_censor, rewrite + deflate), the write.
    python3 profiles/diag/censor_phases.py [pairs]"""
import gzip
import json
import os
import sys
import tempfile
import time

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [REPO, os.path.join(REPO, 'micall-lite_amd')]

import bench  # noqa: E402
from micall_amd import _native, projects, synth  # noqa: E402

pairs = int(sys.argv[1]) if len(sys.argv) > 1 else 1000000
pol = projects.load_default().seed_sequences()['HIV1B-pol-seed']
d = synth.make_pairs(pairs, genomes={'HIV1B-pol-seed': pol}, genome_seed=bench.SEED,
                     read_seed=bench.SEED, block=0, read_len=bench.READ_LEN)
raw1 = bench._fastq_text(d['r1'], d['q1'], 1)
gz1 = gzip.compress(raw1, compresslevel=1)
bad = [(str(1101 + t), c) for t in range(8) for c in range(5, 250, 50)]
ctx = _native.Context(0)
with tempfile.TemporaryDirectory(dir='/tmp') as tmp:
    p = os.path.join(tmp, 'R1.fastq.gz')
    with open(p, 'wb') as f:
        f.write(gz1)
    for rep in range(3):
        with open(p, 'rb') as src, open(os.path.join(tmp, 'out.gz'), 'wb') as dst:
            t0 = time.perf_counter()
            fq = _native.Fastq(fd=src.fileno())
            t1 = time.perf_counter()
            n, bc, ss = ctx.censor_staged(fq, bad, True)
            t2 = time.perf_counter()
            fq.close()
            ctx.censor_write(dst.fileno(), 0)
            t3 = time.perf_counter()
        print(json.dumps({'rep': rep, 'stage_s': round(t1 - t0, 4), 'info': fq.info if hasattr(fq, 'info') else None,
                          'censor_s': round(t2 - t1, 4), 'write_s': round(t3 - t2, 4),
                          'lib_ms': [round(x, 1) for x in ctx.censor_timing()], 'out_bytes': n}), flush=True)
ctx.close()
