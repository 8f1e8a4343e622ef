"""profiles/diag/ingest_phases.py -- the host phases of the FASTQ ingest and
of the CSV writing, repeated, on the GPU box (mh_phase_times):
    python3 profiles/diag/ingest_phases.py [pairs] [repeats]
Writes the C2 input as 64-member gzip FASTQ, then loads it `repeats` times
on one context and formats + writes prelim.csv-style rows each time."""
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
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 3
with tempfile.TemporaryDirectory(dir='/tmp') as d:
    r1, r2 = os.path.join(d, 'R1.fastq.gz'), os.path.join(d, 'R2.fastq.gz')
    p = synth.make_pairs(pairs, genomes=bench.bench_genomes('pol'), genome_seed=bench.SEED,
                         read_seed=bench.SEED, block=0)
    bench.write_fastq_gz(p, r1, r2)
    del p
    seeds = projects.load_default().seed_sequences()
    ctx = _native.Context(0)
    ctx.index_build(list(seeds), list(seeds.values()), 22)
    for rep in range(reps):
        ctx.phase_times(reset=True)
        t = time.perf_counter()
        ctx.reads_load_fastq(r1, r2)
        load_s = time.perf_counter() - t
        ctx.map(_native.params(_native.E2E))
        out = os.path.join(d, 'rows.csv')
        t = time.perf_counter()
        with open(out, 'w') as f:
            lens = ctx.format_segments(1, None, [0, ctx.reads_count()[0]])
            t1 = time.perf_counter()
            ctx.write_segments(f.fileno(), [0])
        t2 = time.perf_counter()
        os.remove(out)
        ph = ctx.phase_times(reset=True)
        print(json.dumps({'rep': rep, 'load_s': round(load_s, 4), 'format_s': round(t1 - t, 4),
                          'write_s': round(t2 - t1, 4), 'bytes': int(lens.sum()),
                          'lib_ms': {k: round(v, 1) for k, v in ph.items()}}))
    ctx.close()
