#!/usr/bin/env python3
"""
profiles/reference_cpu.py -- times the STOCK reference pipeline on the CPU
(dev container only: needs /root/reference; never runs on the GPU box).

The reference's prelim_map() + remap() (micall/core, imported through
tests/golden/refharness.py) run file to file exactly as bin/micall:142-169
calls them, with nthreads = every CPU of this container.  bowtie2 is absent
from the image, so oracle/shim_bin/bowtie2 stands in for it:
the CPU oracle mapper (og_map, C + OpenMP over all cores) behind bowtie2's
command line, SAM text over a pipe.  Everything else -- the per-line SAM
loops, the pileup (sam_to_conseqs with its multiprocessing pool), the
consensus and the loop control -- is the reference's own Python.

Inputs: BASELINE config C1 (examples/HIV1C-pol, 9,600 pairs) and a sample of
config C2 (the bench generator's first pairs, gzip FASTQ).

    python profiles/reference_cpu.py [c2_pairs] > profiles/r02/reference_cpu.json
"""
import json
import os
import sys
import tempfile
import time

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
for p in (os.path.join(REPO, 'tests', 'golden'), os.path.join(REPO, 'oracle'),
          os.path.join(REPO, 'micall-lite_amd'), REPO):
    sys.path.insert(0, p)

import refharness  # noqa: E402


def run(r1, r2, nthreads):
    refharness.setup()
    from micall.core.prelim_map import prelim_map
    from micall.core.remap import remap
    shim = os.path.join(REPO, 'oracle', 'shim_bin')
    work = tempfile.mkdtemp(prefix='refcpu_')
    cwd = os.getcwd()
    os.chdir(work)
    try:
        t0 = time.perf_counter()
        with open('prelim.csv', 'w') as h:
            prelim_map(r1, r2, h, bt2_path=os.path.join(shim, 'bowtie2'),
                       bt2build_path=os.path.join(shim, 'bowtie2-build-s'), nthreads=nthreads,
                       gzip=True, work_path=work)
        t1 = time.perf_counter()
        with open('prelim.csv') as pre, open('remap.csv', 'w') as out, \
                open('remap_counts.csv', 'w') as counts:
            remap(r1, r2, pre, out, counts, work_path=work, bt2_path=os.path.join(shim, 'bowtie2'),
                  bt2build_path=os.path.join(shim, 'bowtie2-build-s'), nthreads=nthreads,
                  gzip=True)
        t2 = time.perf_counter()
        with open('remap_counts.csv') as f:
            passes = sum(1 for line in f if line.startswith('remap-') and
                         not line.startswith('remap-final'))
        return dict(prelim_map_s=round(t1 - t0, 2), remap_s=round(t2 - t1, 2),
                    seconds=round(t2 - t0, 2), remap_rows_passes=passes)
    finally:
        os.chdir(cwd)
        import shutil
        shutil.rmtree(work, ignore_errors=True)


def main():
    import bench
    c2_pairs = int(sys.argv[1]) if len(sys.argv) > 1 else 20000
    threads = len(os.sched_getaffinity(0))
    out = {'host': {'cpus': threads, 'nproc': os.cpu_count()},
           'mapper': 'oracle/shim_bin/bowtie2 (og_map, OpenMP) standing in for bowtie2 2.2.8',
           'runs': {}}
    ex = os.path.join(refharness.REF, 'examples', 'HIV1C-pol_S1_L001_R{}_001.fastq.gz')
    res = run(ex.format(1), ex.format(2), threads)
    res.update(pairs=9600, reads_per_s=round(2 * 9600 / res['seconds'], 1))
    out['runs']['C1 examples/HIV1C-pol'] = res
    from micall_amd import synth
    work = tempfile.mkdtemp(prefix='refcpu_in_')
    pairs = synth.make_pairs(c2_pairs, genomes=bench.bench_genomes('pol'), genome_seed=bench.SEED,
                             read_seed=bench.SEED, block=0)
    r1, r2 = os.path.join(work, 'R1.fastq.gz'), os.path.join(work, 'R2.fastq.gz')
    bench.write_fastq_gz(pairs, r1, r2, threads=threads)
    res = run(r1, r2, threads)
    res.update(pairs=c2_pairs, reads_per_s=round(2 * c2_pairs / res['seconds'], 1))
    out['runs']['C2 sample'] = res
    for p in (r1, r2):
        os.remove(p)
    os.rmdir(work)
    print(json.dumps(out, indent=1))


if __name__ == '__main__':
    main()
