#!/usr/bin/env python3
"""
bench.py -- MiCall-Lite iterative-remap hot path on MI355X.

One step = one pass of the hot path over one batch of synthetic input already
resident in HBM (BASELINE.json configs[1], "C2"): prelim_map's end-to-end
mapping of every read pair against all 74 seed references, seed selection,
the prelim consensus (device pileup), ONE remap iteration (--local mapping
against the consensus, device pileup, consensus + distance filter).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--pairs P]

N > 1 is launched by torch.distributed.run, one rank per GPU; every rank holds
its own block of P pairs (weak scaling), per-reference tallies and the dense
pileup counters are all-reduced over RCCL between passes.  Rank 0 prints one
JSON line.  value = reads/s over the whole job (2 reads per pair).
"""
import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
for _p in (os.path.join(REPO, 'micall-lite_amd'), os.path.join(REPO, 'oracle')):
    if _p not in sys.path:
        sys.path.insert(0, _p)

import numpy as np  # noqa: E402

METRIC = 'paired 2×251 nt reads/sec mapped+realigned; fraction of HBM roofline'
HBM_PEAK_GBS = 8000.0      # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
SEED = 20261015
READ_LEN = 251


def algo_bytes_per_pair(L=READ_LEN):
    """2-bit bases + N mask + qualities for both mates + two
    32-byte alignment records, per pair per mapping pass (756 B at L=251)."""
    return 2 * -(-L // 4) + 2 * -(-L // 8) + 2 * L + 64


def bench_genomes(which='pol', read_len=READ_LEN):
    """Seeds the synthetic sample genomes derive from: 'pol' (C2/C3/C5),
    'hiv' (C4: the HIV-1 seeds that hold a fragment of >= 260 nt; vpu, 246 nt,
    is shorter than a read) or 'all' (C4's other reading: every seed region of
    the project file long enough for a fragment)."""
    from micall_amd import projects
    seeds = projects.load_default().seed_sequences()
    if which == 'pol':
        return {'HIV1B-pol-seed': seeds['HIV1B-pol-seed']}
    if which == 'all':   # SURVEY.md 8(d) C4, the all-seed-regions reading
        return {k: v for k, v in seeds.items() if len(v) >= max(260, read_len + 9)}
    return {k: v for k, v in seeds.items() if k.startswith('HIV') and len(v) >= max(260, read_len + 9)}


def make_reads(pairs, block, read_len=READ_LEN, paired=True, genomes='pol'):
    from micall_amd import synth
    d = synth.make_pairs(pairs, genomes=bench_genomes(genomes, read_len), genome_seed=SEED,
                         read_seed=SEED, block=block, read_len=read_len, paired=paired)
    if not paired:
        return d['r1'], d['q1']
    reads = np.stack([d['r1'], d['r2']], axis=1).reshape(2 * pairs, read_len)
    quals = np.stack([d['q1'], d['q2']], axis=1).reshape(2 * pairs, read_len)
    return reads, quals


def cgroup_throttle():
    """(nr_throttled, throttled_usec / 1e3) of this cgroup's CPU quota so
    far, or None: a bench leg reports the difference, the periods in which
    its threads stood still because the cgroup had used up its quota (the
    kernel's throttled time is summed over CPUs, so it can exceed the wall
    time of the leg)."""
    try:
        with open('/sys/fs/cgroup/cpu.stat') as f:
            kv = dict(line.split() for line in f if line.strip())
        return int(kv['nr_throttled']), int(kv['throttled_usec']) / 1e3
    except (OSError, ValueError, KeyError):
        return None


def throttle_since(before):
    after = cgroup_throttle()
    if before is None or after is None:
        return None
    return {'periods': after[0] - before[0], 'cpu_ms': round(after[1] - before[1], 1)}


def host_cpus():
    """The host CPUs as this process sees them: every CPU it may run on
    (sched_getaffinity: all host cores, 256 on the GPU box), the launcher's
    OMP_NUM_THREADS (the box's CPU share, 16) and the cgroup CPU quota."""
    affinity = len(os.sched_getaffinity(0))
    omp = os.environ.get('OMP_NUM_THREADS')
    share = min(affinity, int(omp)) if omp and omp.isdigit() and int(omp) > 0 else affinity
    quota = None
    try:
        with open('/sys/fs/cgroup/cpu.max') as f:
            q, period = f.read().split()
            quota = None if q == 'max' else round(int(q) / int(period), 2)
    except (OSError, ValueError):
        pass
    return {'sched_getaffinity': affinity, 'nproc': os.cpu_count(), 'OMP_NUM_THREADS': omp,
            'share_threads': share, 'cgroup_cpu_quota': quota}


def _oracle_step(reads, quals, paired, threads, iterations=1, forced=False):
    """One run of the CPU oracle's step (cpu_pipeline.timed_step) on the
    given units: (seconds, the prepared reads with .result)."""
    import cpu_pipeline
    from micall_amd import projects
    cfg = projects.load_default()
    seed_set = cfg.seed_sequences()
    groups = {k: cfg.getSeedGroup(k) for k in seed_set}
    prep = cpu_pipeline.Prepared.from_arrays(reads, quals, paired)
    _, secs = cpu_pipeline.timed_step(seed_set, cfg.all_region_sequences(), groups, prep, threads,
                                      max_iterations=iterations,
                                      min_iterations=iterations if forced else None)
    return secs, prep


def cpu_baseline(reads, quals, paired=True, iterations=1, forced=False, workload='2x251 pol'):
    """The CPU oracle's step (C restatement: og_map + og_rows_from_alns +
    og_pileup_mt, OpenMP over read pairs; O(reference length) consensus in
    Python; the consensus-distance filter's K x K og_gotoh_align +
    og_levenshtein on host threads) on a bounded sample of the same workload
    -- the first units of the bench's own input -- on every host core
    (sched_getaffinity) and again on the box's CPU share (OMP_NUM_THREADS).
    The reads are packed before the clock starts, so the timed region holds
    no per-read Python: the device-resident step's CPU equivalent.  Returns
    (baseline dict, the oracle's records and consensus of the last run for
    the parity leg)."""
    units = reads.shape[0] // 2 if paired else reads.shape[0]
    per_unit = 2 if paired else 1
    cpus = host_cpus()
    runs = {}
    prep = None
    for threads in sorted({cpus['sched_getaffinity'], cpus['share_threads']}, reverse=True):
        secs, prep = _oracle_step(reads, quals, paired, threads, iterations, forced)
        runs[threads] = secs
    allc, share = cpus['sched_getaffinity'], cpus['share_threads']
    best = min(runs, key=runs.get)   # the faster of the two is the baseline
    passes = len(prep.result['passes'])
    return {'value': round(per_unit * units / runs[best], 1), 'unit': 'reads/s', 'cores': best,
            'kind': 'port', 'host_cpus': cpus,
            'runs': {str(t): {'seconds': round(s, 3), 'value': round(per_unit * units / s, 1)}
                     for t, s in sorted(runs.items())},
            'sample': 'the first {} {} of the bench input ({}): prelim e2e pass over 74 seeds + '
                      '{} local remap pass(es) with pileup, consensus and the consensus-distance '
                      'filter, oracle C restatement (og_map, og_pileup_mt, og_gotoh_align, '
                      'og_levenshtein) with OpenMP / threads over units, timed on all {} host '
                      'cores ({:.1f} s) and on the {}-thread CPU share ({:.1f} s); value is the '
                      'faster; reads packed before timing'.format(
                          units, 'pairs' if paired else 'reads', workload, passes, allc, runs[allc],
                          share, runs[share])}, prep.result


def record_mismatches(dev, ref):
    """Indices of the records that differ between two arrays of alignment
    records (every field, and the CIGAR words up to n_cigar)."""
    from micall_amd import _native
    assert len(dev) == len(ref), (len(dev), len(ref))
    same = np.ones(len(ref), dtype=bool)
    for f in _native.ALN_FIELDS:
        same &= dev[f] == ref[f]
    live = np.arange(ref['cigar'].shape[1])[None, :] < ref['n_cigar'][:, None]
    same &= np.all((dev['cigar'] == ref['cigar']) | ~live, axis=1)
    return np.flatnonzero(~same)


def parity_check(ctx, pipe, sample, paired, baseline_result=None, device_index=0, iterations=1,
                 forced=False):
    """Parity at configuration size (untimed, after the timed steps): the
    device's alignment records of the bench's own run for its first units
    against the CPU oracle's (og_map) on the same reads, byte for byte.
    A record depends on its read (pair) and the references only, so the
    first units of the 1M-pair run must equal the oracle's on those units.

      prelim   an end-to-end pass over the 74 seeds on the resident reads
               (what every step's prelim pass computes);
      remap    the last step's --local pass, against the consensus set it
               mapped to (pipe.mapped_to), vs og_map against the same set;
      consensus  the sample alone through the device pipeline on a new
               context, with the bench's iteration settings: its prelim
               consensus, every pass's kept set after the consensus-distance
               filter, and the final consensus against the oracle step's
               (cpu_pipeline.timed_step; the CPU baseline's run of the same
               sample when there was one, else one untimed run here).

    Consumers of these records in the reference: remap.py:474-541 (seed
    selection and the consensus), prelim_map.py:134-151 (prelim.csv)."""
    import cpu_pipeline
    import oracle
    from micall_amd import _native
    from micall_amd.pipeline import RemapPipeline
    t0 = time.perf_counter()
    reads, quals = sample
    n = reads.shape[0]
    threads = host_cpus()['share_threads']
    out = {'units_checked': n // 2 if paired else n, 'reads_checked': n,
           'unit': 'pairs' if paired else 'reads'}
    # the last step's remap pass: its records are still the context's
    mapped_to = dict(pipe.mapped_to or {})
    if mapped_to:
        dev = ctx.fetch(0, n)
        ref = cpu_pipeline.map_arrays(list(mapped_to.values()), oracle.LOCAL, reads, quals, paired,
                                      threads)
        bad = record_mismatches(dev, ref)
        out['remap'] = {'references': list(mapped_to), 'record_mismatches': int(len(bad)),
                        'first_mismatches': bad[:8].tolist(),
                        'mapped_reads': int(((ref['flag'] & 4) == 0).sum())}
        del dev, ref
    names = list(pipe.seed_set)
    ctx.index_build(names, [pipe.seed_set[k] for k in names], 22)
    ctx.map(pipe._params(_native.E2E))
    dev = ctx.fetch(0, n)
    if baseline_result is not None and baseline_result['prelim_names'] == names:
        ref = baseline_result['prelim']
    else:
        ref = cpu_pipeline.map_arrays([pipe.seed_set[k] for k in names], oracle.E2E, reads, quals,
                                      paired, threads)
    bad = record_mismatches(dev, ref)
    out['prelim'] = {'record_mismatches': int(len(bad)), 'first_mismatches': bad[:8].tolist(),
                     'mapped_reads': int(((ref['flag'] & 4) == 0).sum())}
    del dev, ref
    if baseline_result is None:
        t1 = time.perf_counter()
        baseline_result = _oracle_step(reads, quals, paired, threads, iterations, forced)[1].result
        out['oracle_step_seconds'] = round(time.perf_counter() - t1, 2)
    if baseline_result is not None:
        c2 = _native.Context(device_index)
        try:
            c2.reads_load_fixed(reads, quals, paired)
            p2 = RemapPipeline(c2)
            units = n // 2 if paired else n
            final, _counts, _unm = p2.run(2.0 * units, max_iterations=iterations,
                                          min_iterations=iterations if forced else None)
            cpu_passes = baseline_result.get('passes', [])
            first = p2.first_mapped_to or {}
            out['consensus'] = {
                'prelim_equal': (first == baseline_result['prelim_conseqs'] and
                                 list(first) == list(baseline_result['prelim_conseqs'])),
                'passes': len(p2.log),
                'passes_equal': (len(p2.log) == len(cpu_passes) and
                                 all(sorted(a['conseqs']) == b['kept'] for a, b in zip(p2.log, cpu_passes))),
                'kept_per_pass': [sorted(a['conseqs']) for a in p2.log],
                'unfiltered_per_pass': [b['unfiltered'] for b in cpu_passes],
                'final_equal': final == baseline_result['conseqs'],
                'references': sorted(final)}
            if (out['consensus']['prelim_equal'] and out['consensus']['passes_equal'] and
                    list(p2.mapped_to or {}) == baseline_result['remap_names'] and
                    baseline_result['remap'] is not None):
                bad = record_mismatches(c2.fetch(), baseline_result['remap'])
                out['consensus']['sample_remap_record_mismatches'] = int(len(bad))
        finally:
            c2.close()
    out['record_mismatches'] = out['prelim']['record_mismatches'] + \
        out.get('remap', {}).get('record_mismatches', 0)
    out['pairs_checked'] = out['units_checked'] if paired else None
    out['consensus_equal'] = (out['consensus']['prelim_equal'] and out['consensus']['passes_equal'] and
                              out['consensus']['final_equal'] if 'consensus' in out else None)
    out['seconds'] = round(time.perf_counter() - t0, 2)
    out['oracle_threads'] = threads
    return out


def parity_full(ctx, pipe, reads, quals, paired, chunk_units, log=sys.stderr):
    """Whole-input parity (untimed): every record of every mapping pass of
    the last step -- the prelim end-to-end pass over the 74 seeds and each
    --local pass against the consensus set it mapped to (pipe.pass_refs) --
    against og_map on the same reads, in chunks of chunk_units units so the
    oracle's buffers stay bounded (records depend only on their read pair
    and the references).  Each pass is mapped again on the device over the
    whole resident input (the step's own computation, deterministic) and
    fetched chunk by chunk.  Reference loop: remap.py:544-606."""
    import cpu_pipeline
    import oracle
    from micall_amd import _native
    threads = host_cpus()['share_threads']
    per = 2 if paired else 1
    n = reads.shape[0]
    step = chunk_units * per
    passes = [('prelim', oracle.E2E, dict(pipe.seed_set))] + \
             [('remap-%d' % (i + 1), oracle.LOCAL, refs) for i, refs in enumerate(pipe.pass_refs)]
    out = {'units_checked': n // per, 'unit': 'pairs' if paired else 'reads', 'chunk_units': chunk_units,
           'oracle_threads': threads, 'passes': []}
    t0 = time.perf_counter()
    for name, mode, refs in passes:
        names = list(refs)
        ctx.index_build(names, [refs[k] for k in names], oracle.seed_len(mode))
        ctx.map(pipe._params(_native.E2E if mode == oracle.E2E else _native.LOCAL))
        bad_total, first_bad, mapped = 0, [], 0
        for a in range(0, n, step):
            b = min(n, a + step)
            dev = ctx.fetch(a, b - a)
            ref = cpu_pipeline.map_arrays([refs[k] for k in names], mode, reads[a:b], quals[a:b], paired,
                                          threads)
            bad = record_mismatches(dev, ref)
            bad_total += len(bad)
            first_bad += (bad[:4] + a).tolist() if len(first_bad) < 8 else []
            mapped += int(((ref['flag'] & 4) == 0).sum())
            del dev, ref
            print('parity_full {} reads {}..{}: {} mismatches ({:.0f} s)'.format(
                name, a, b, len(bad), time.perf_counter() - t0), file=log, flush=True)
        out['passes'].append({'pass': name, 'references': len(names), 'reads': n,
                              'record_mismatches': int(bad_total), 'first_mismatches': first_bad[:8],
                              'mapped_reads': mapped})
    out['record_mismatches'] = sum(p['record_mismatches'] for p in out['passes'])
    out['seconds'] = round(time.perf_counter() - t0, 1)
    return out


def cpu_end_to_end(sample_pairs, workdir):
    """The reference's file-to-file path on the CPU (oracle/cpu_e2e.py: its
    prelim_map() + remap() structure -- FASTQ parsed every pass, SAM text,
    prelim.csv through csv.DictWriter / DictReader, sam_to_conseqs, the
    stopping rules, the splitter -- with the oracle C mapper where bowtie2 -p
    N stood), on a bounded sample of the C2 input written as gzip FASTQ,
    timed on every host core (sched_getaffinity) and on the launcher's CPU
    share (OMP_NUM_THREADS); the faster is the baseline, as in cpu_baseline.
    Byte-equal to the reference on the golden cases (tests/test_cpu_e2e.py)."""
    import cpu_e2e
    from micall_amd import projects, synth
    cfg = projects.load_default()
    seeds = cfg.seed_sequences()
    r1 = os.path.join(workdir, 'cpu_R1.fastq.gz')
    r2 = os.path.join(workdir, 'cpu_R2.fastq.gz')
    pairs = synth.make_pairs(sample_pairs, genomes=bench_genomes('pol'), genome_seed=SEED,
                             read_seed=SEED, block=0)
    write_fastq_gz(pairs, r1, r2)
    del pairs
    cpus = host_cpus()
    paths = {k: os.path.join(workdir, 'cpu_' + k) for k in ('prelim.csv', 'remap.csv', 'counts.csv',
                                                           'conseq.csv', 'u1.fastq', 'u2.fastq')}
    runs = {}
    for threads in sorted({cpus['sched_getaffinity'], cpus['share_threads']}, reverse=True):
        t0 = time.perf_counter()
        with open(paths['prelim.csv'], 'w') as f:
            cpu_e2e.prelim_map(r1, r2, f, seeds, threads)
        t1 = time.perf_counter()
        with open(paths['prelim.csv']) as pre, open(paths['remap.csv'], 'w') as out, \
                open(paths['counts.csv'], 'w') as counts, open(paths['conseq.csv'], 'w') as conseq, \
                open(paths['u1.fastq'], 'w+') as u1, open(paths['u2.fastq'], 'w+') as u2:
            cpu_e2e.remap(r1, r2, pre, out, counts, conseq, u1, u2, cfg.all_region_sequences(),
                          {k: cfg.getSeedGroup(k) for k in seeds}, workdir, threads)
        t2 = time.perf_counter()
        runs[threads] = (t2 - t0, t1 - t0, t2 - t1)
    for p in list(paths.values()) + [r1, r2]:
        os.remove(p)
    best = min(runs, key=lambda t: runs[t][0])
    secs, pre_s, rem_s = runs[best]
    return {'value': round(2 * sample_pairs / secs, 1), 'unit': 'reads/s', 'cores': best,
            'kind': 'port', 'seconds': round(secs, 3), 'prelim_map_s': round(pre_s, 3),
            'remap_s': round(rem_s, 3), 'host_cpus': cpus,
            'runs': {str(t): {'seconds': round(v[0], 3), 'value': round(2 * sample_pairs / v[0], 1)}
                     for t, v in sorted(runs.items())},
            'sample': '{} pairs of the C2 input as gzip FASTQ, file to file (prelim.csv, remap.csv, '
                      'remap_counts.csv, remap_conseq.csv, unmapped FASTQs): the reference\'s '
                      'prelim_map() + remap() structure restated in oracle/cpu_e2e.py with the '
                      'oracle C mapper, timed on {} threads; value is the fastest'.format(
                          sample_pairs, ' and '.join(str(t) for t in sorted(runs)))}


class PhaseClock:
    """Wall time per phase of the drop-ins' file-to-file path, without added
    synchronisation: the Python calls below are wrapped with perf_counter
    (each device call they make ends in its own stream sync), and the
    library's own host phases (inflate, parse, upload, format, write) come
    from mh_phase_times.  'other' is what the named phases leave of the
    total (Python glue, the splitter, remap_counts, file opens)."""

    def __init__(self):
        self.acc = {}
        self._undo = []

    def _wrap(self, owner, name, label_of):
        fn = getattr(owner, name)
        acc = self.acc

        def timed(*a, **kw):
            t = time.perf_counter()
            try:
                return fn(*a, **kw)
            finally:
                label = label_of(a, kw)
                acc[label] = acc.get(label, 0.0) + time.perf_counter() - t
        setattr(owner, name, timed)
        self._undo.append((owner, name, fn))

    def __enter__(self):
        from micall_amd import _native, pipeline, session
        self._wrap(_native.Context, 'index_build',
                   lambda a, kw: 'index_build_' + ('seeds' if len(a[1]) > 10 else 'consensus'))
        self._wrap(_native.Context, 'map',
                   lambda a, kw: 'map_prelim' if a[1].mode == _native.E2E else 'map_remap')
        self._wrap(pipeline.RemapPipeline, 'prelim_conseqs', lambda a, kw: 'pileup_consensus')
        self._wrap(pipeline.RemapPipeline, 'build_conseqs_filtered', lambda a, kw: 'pileup_consensus')
        self._wrap(session, 'prelim_resident', lambda a, kw: 'prelim_csv_check')
        self._wrap(_native.Context, 'map_counts', lambda a, kw: 'tallies')
        return self

    def __exit__(self, *exc):
        for owner, name, fn in reversed(self._undo):
            setattr(owner, name, fn)
        return False


class Job:
    """This process's place in the bench job and the collectives the
    file-to-file legs use: rank, world, and a barrier / gathers over the
    initialised torch.distributed group (through the drop-ins' own
    pipeline.Shard, so the legs run the sharded code paths a torchrun'd
    bin/micall runs).  world == 1 without a group."""

    def __init__(self, shard=None):
        import torch.distributed as dist
        from micall_amd import session
        if shard is None and dist.is_available() and dist.is_initialized():
            shard = session.shard()
        self.shard = shard
        self.rank = self.shard.rank if self.shard else 0
        self.world = self.shard.world if self.shard else 1

    def barrier(self):
        if self.shard:
            self.shard.barrier()

    def gather(self, values):
        """int64 values of every rank: array [world, len(values)]."""
        if not self.shard:
            return np.asarray([values], dtype=np.int64)
        return self.shard._gather_sizes(values)

    def max_seconds(self, secs):
        """max over ranks of a duration (microsecond resolution)."""
        return float(self.gather([int(round(secs * 1e6))])[:, 0].max()) / 1e6

    def per_rank_seconds(self, secs):
        return [round(float(x) / 1e6, 4) for x in self.gather([int(round(secs * 1e6))])[:, 0]]

    def shared_dir(self, prefix):
        """A fresh directory every rank of the job uses (rank 0 makes it)."""
        import tempfile
        path = tempfile.mkdtemp(prefix=prefix).encode() if self.rank == 0 else b''
        if self.shard:
            path = self.shard.all_gather_bytes(path)[0]
        return path.decode()


def _fastq_records(pairs, mate):
    from micall_amd import synth
    r, q = pairs['r%d' % mate], pairs['q%d' % mate]
    return [b'%s\n%s\n+\n%s\n' % (synth.read_name(pairs['block'], i, mate).encode(), r[i].tobytes(),
                                  q[i].tobytes()) for i in range(pairs['n'])]


def write_fastq_gz(pairs, path1, path2, threads=16, single=False, job=None):
    """The pairs as gzip FASTQ files.  One process: independent gzip members
    compressed on `threads` threads (a multi-member file is one valid gzip
    stream), or with single=True one gzip member, as bcl2fastq writes it
    (one deflate stream over the whole text).

    Under a job of W ranks each rank passes its own block of pairs and the
    file holds the blocks in rank order: its members (many), or (single)
    one gzip member whose deflate stream each rank writes for its block --
    one stream per rank, primed with the last 32 KiB of the block before
    (so back-references cross the rank boundaries, as pigz writes a single
    member) and ended with a sync flush -- between rank 0's gzip header and
    a trailer carrying the CRC-32 and size of the whole text.  Every rank
    pwrites its bytes at offsets all-gathered from the sizes."""
    import zlib
    from concurrent.futures import ThreadPoolExecutor
    from micall_amd import _native
    world = job.world if job else 1
    rank = job.rank if job else 0

    def member(chunk):
        c = zlib.compressobj(1, zlib.DEFLATED, 31)
        return c.compress(chunk) + c.flush()
    for mate, path in ((1, path1), (2, path2)):
        recs = _fastq_records(pairs, mate)
        if not single:
            step = -(-len(recs) // (threads * 4))
            chunks = [b''.join(recs[k:k + step]) for k in range(0, len(recs), step)]
            del recs
            with ThreadPoolExecutor(threads) as ex:
                blob = b''.join(ex.map(member, chunks))
            head, tail = b'', b''
        elif world == 1:
            blob = member(b''.join(recs))
            del recs
            head, tail = b'', b''
        else:
            text = b''.join(recs)
            del recs
            before = job.shard.all_gather_bytes(text[-32768:])
            zdict = before[rank - 1] if rank > 0 else None
            c = (zlib.compressobj(1, zlib.DEFLATED, -15, zdict=zdict) if zdict else
                 zlib.compressobj(1, zlib.DEFLATED, -15))
            blob = c.compress(text) + c.flush(zlib.Z_FINISH if rank == world - 1 else zlib.Z_SYNC_FLUSH)
            facts = job.gather([zlib.crc32(text), len(text)])
            del text
            crc = 0
            for k in range(world):
                crc = _native.crc32_combine(crc, int(facts[k, 0]), int(facts[k, 1]))
            size = int(facts[:, 1].sum())
            head = b'\x1f\x8b\x08\x00\x00\x00\x00\x00\x00\x03' if rank == 0 else b''
            tail = (crc.to_bytes(4, 'little') + (size & 0xffffffff).to_bytes(4, 'little')
                    if rank == world - 1 else b'')
        data = head + blob + tail
        if world == 1:
            with open(path, 'wb') as f:
                f.write(data)
            continue
        lens = job.gather([len(data)])[:, 0]
        if rank == 0:
            with open(path, 'wb') as f:
                f.truncate(int(lens.sum()))
        job.barrier()
        fd = os.open(path, os.O_WRONLY)
        try:
            at, mv = int(lens[:rank].sum()), memoryview(data)
            while len(mv):
                n = os.pwrite(fd, mv, at)
                at += n
                mv = mv[n:]
        finally:
            os.close(fd)
        job.barrier()


def end_to_end(n_pairs, workdir, single_member=False, job=None):
    """The file-to-file path bin/micall runs (prelim_map() then remap(), the
    drop-ins) on the C2 input written as gzip FASTQ: ingest (gunzip + parse
    + H2D + 2-bit packing), the cold 74-seed index, the prelim pass and
    prelim.csv text, remap's prelim.csv parse, one remap pass, remap.csv
    text.  A new device context is used, so nothing is cached from the
    device-resident bench.

    Under a job of W ranks (torchrun) the files hold every rank's block of
    n_pairs pairs (written untimed, in rank order) and every rank calls the
    drop-ins with the same paths, as a torchrun'd bin/micall does: each
    reads its share of the FASTQ, maps its block and writes its own rows;
    the time is the max over ranks.  Returns the result dict (reads/s over
    the whole job, seconds per part)."""
    import io
    from micall_amd import _native, prelim_map, remap, session, sharded_io, synth
    world = job.world if job else 1
    rank = job.rank if job else 0
    r1 = os.path.join(workdir, 'R1.fastq.gz')
    r2 = os.path.join(workdir, 'R2.fastq.gz')
    pairs = synth.make_pairs(n_pairs, genomes=bench_genomes('pol'), genome_seed=SEED,
                             read_seed=SEED, block=rank)
    t_write = time.perf_counter()
    write_fastq_gz(pairs, r1, r2, single=single_member, job=job)
    t_write = time.perf_counter() - t_write
    del pairs
    sizes = os.path.getsize(r1) + os.path.getsize(r2)
    # cold index build alone, on its own context
    from micall_amd import projects
    seeds = projects.load_default().seed_sequences()
    probe = _native.Context(session._device_index())
    probe.sync()
    t = time.perf_counter()
    probe.index_build(list(seeds), list(seeds.values()), 22)
    probe.sync()
    index_cold_ms = 1e3 * (time.perf_counter() - t)
    probe.close()
    session.reset()
    sharded_io.reset_stats()
    prelim_path = os.path.join(workdir, 'prelim.csv')
    remap_path = os.path.join(workdir, 'remap.csv')
    thr0 = cgroup_throttle()
    if job:
        job.barrier()
    with PhaseClock() as clock:
        t0 = time.perf_counter()
        with open(prelim_path, 'w') as f:
            prelim_map.prelim_map(r1, r2, f, gzip=True)
        t1 = time.perf_counter()
        lib_pre = session.context().phase_times(reset=True)
        with open(prelim_path) as pre, open(remap_path, 'w') as out:
            counts = io.StringIO()
            remap.remap(r1, r2, pre, out, counts, gzip=True)
        t2 = time.perf_counter()
    lib_rem = session.context().phase_times(reset=True)
    session.context().sync()
    io_stats = dict(sharded_io.IO_STATS)
    if job:
        job.barrier()
        secs = job.max_seconds(t2 - t0)
        per_rank = job.per_rank_seconds(t2 - t0)
        pre_s = job.max_seconds(t1 - t0)
        rem_s = job.max_seconds(t2 - t1)
        rank_io = job.gather([io_stats['fastq_file_bytes'], io_stats['fastq_text_bytes'],
                              io_stats['written_bytes']])
    else:
        secs, per_rank, pre_s, rem_s, rank_io = t2 - t0, None, t1 - t0, t2 - t1, None
    ph = {k: v for k, v in clock.acc.items()}
    phases = {'inflate': lib_pre['inflate'] / 1e3, 'parse': lib_pre['parse'] / 1e3,
              'upload_pack': lib_pre['upload'] / 1e3,
              'index_build_seeds': ph.get('index_build_seeds', 0.0),
              'map_prelim': ph.get('map_prelim', 0.0),
              'prelim_csv_format': lib_pre['format'] / 1e3, 'prelim_csv_write': lib_pre['write'] / 1e3,
              'prelim_csv_check': ph.get('prelim_csv_check', 0.0),
              'tallies': ph.get('tallies', 0.0),
              'pileup_consensus': ph.get('pileup_consensus', 0.0),
              'index_build_consensus': ph.get('index_build_consensus', 0.0),
              'map_remap': ph.get('map_remap', 0.0),
              'remap_csv_format': lib_rem['format'] / 1e3, 'remap_csv_write': lib_rem['write'] / 1e3}
    phases['other'] = (t2 - t0) - sum(phases.values())
    layout = ('one gzip member per file' + (' (one deflate stream per rank block, primed with the '
                                            'block before\'s last 32 KiB)' if world > 1 else '')
              if single_member else 'many members ({} per file)'.format(64 * world))
    out = {'value': round(2 * n_pairs * world / secs, 1), 'unit': 'reads/s', 'n_gpus': world,
           'seconds': round(secs, 3), 'prelim_map_s': round(pre_s, 3),
           'remap_s': round(rem_s, 3), 'index_build_cold_ms': round(index_cold_ms, 2),
           'cgroup_throttled': throttle_since(thr0),
           'phases_s': {k: round(v, 4) for k, v in phases.items()},
           'prelim_source': session.stats.get('prelim_source'),
           'fastq_gz_bytes': sizes, 'fastq_gz_members': layout,
           'fastq_write_untimed_s': round(t_write, 2),
           'prelim_csv_bytes': os.path.getsize(prelim_path),
           'remap_csv_bytes': os.path.getsize(remap_path),
           'remap_counts': counts.getvalue().strip().split('\n')[-3:],
           'what': 'prelim_map() + remap() drop-ins file to file on {} pairs of gzip FASTQ '
                   '(C2 input{}): ingest, cold 74-seed index, prelim pass, prelim.csv write, '
                   'remap pass(es) by the reference\'s stopping rules, remap.csv write; '
                   'new device context'.format(n_pairs * world,
                                               '' if world == 1 else ', {} pairs per rank'.format(n_pairs))}
    if job and world > 1:
        out['per_rank_seconds'] = per_rank
        out['per_rank_io'] = {'fastq_file_bytes': rank_io[:, 0].tolist(),
                              'fastq_text_bytes': rank_io[:, 1].tolist(),
                              'written_bytes': rank_io[:, 2].tolist(),
                              'fastq_mode': io_stats['fastq_mode']}
        out['phases_s_rank0'] = out.pop('phases_s')
    session.reset()
    if job:
        job.barrier()
    if rank == 0:
        for p in (r1, r2, prelim_path, remap_path):
            os.remove(p)
    return out


KERNEL_SOURCES = ('micall-lite_amd/csrc/mh_map.hip', 'micall-lite_amd/csrc/mh_pileup.hip',
                  'micall-lite_amd/csrc/mh_internal.h', 'micall-lite_amd/csrc/Makefile')


def kernel_source_sha():
    """Fingerprint of the mapping / pileup kernels' sources (the files the
    committed PMC and SQ summaries were measured on must hash the same)."""
    import hashlib
    h = hashlib.sha256()
    for rel in KERNEL_SOURCES:
        with open(os.path.join(REPO, rel), 'rb') as f:
            h.update(rel.encode() + b'\0' + f.read())
    return h.hexdigest()[:16]


def matching_profile(name):
    """The committed profile summary `name` (profiles/rNN/c2*/name, newest
    round first) that was measured on these kernel sources
    (kernel_source_sha), or None: a summary of another build is never
    divided by this run's launch times."""
    base = os.path.join(REPO, 'profiles')
    try:
        rounds = sorted((d for d in os.listdir(base) if len(d) == 3 and d[0] == 'r' and d[1:].isdigit()),
                        reverse=True)
    except OSError:
        return None
    sha = kernel_source_sha()
    for d in rounds:
        for sub in sorted((x for x in os.listdir(os.path.join(base, d)) if x.startswith('c2')), reverse=True):
            path = os.path.join(base, d, sub, name)
            try:
                with open(path) as f:
                    if json.load(f).get('kernel_source_sha') == sha:
                        return path
            except (OSError, ValueError):
                continue
    return None


def read_pmc_traffic(kernel, pairs, stage='remap'):
    """Per-launch HBM bytes of `kernel` from the committed rocprofv3 PMC
    summary of this stage (separate --pmc passes, FETCH_SIZE doubled per the
    gfx950 rule; profiles/collect_pmc_stages.sh), when it was measured on the
    same per-GPU pair count; the remap stage's summary must also carry these
    kernel sources' fingerprint (matching_profile)."""
    if stage == 'remap':
        path = matching_profile('pmc_traffic.json')
        if path is None:
            return None
    else:
        path = os.path.join(REPO, 'profiles', 'pmc_traffic_{}.json'.format(stage))
    try:
        with open(path) as f:
            d = json.load(f)
        k = d['kernels'][kernel]
        if int(d.get('pairs', -1)) != pairs:
            return None
        return k['hbm_bytes_per_launch']
    except (OSError, KeyError, ValueError):
        return None


VALU_ISSUE_CYCLES = 2      # MI355X_MICROARCH.md: a wave64 VALU instruction issues over 2 cycles


def read_valu_issue(kernel, pairs, avg_launch_ms):
    """Issue-side roofline of `kernel` (it is bound by integer VALU issue and
    its dependency chain, not HBM): VALU wave-instructions per launch from the
    committed SQ_INSTS_VALU pass (profiles/rNN/c2*/sq_issue.json measured on
    these kernel sources, matching_profile; same per-GPU pair count; the mate-rescue DP launch, the one after k_rescue, is
    left out), over this run's average launch time, against 1024 SIMDs x the
    measured clock / VALU_ISSUE_CYCLES."""
    path = matching_profile('sq_issue.json')
    if path is None:
        return None
    try:
        with open(path) as f:
            every = json.load(f)['dispatches']
        d = [x for k, x in enumerate(every) if x['kernel'] == kernel and
             not (k and every[k - 1]['kernel'] == 'k_rescue')]
        if not d or pairs != 1000000 or avg_launch_ms <= 0:
            return None
        insts = sum(x['valu_insts'] for x in d) / len(d)
        clk = sum(x['clock_ghz'] for x in d) / len(d)
        achieved = insts / (avg_launch_ms / 1e3) / 1e9
        peak = 1024 * clk / VALU_ISSUE_CYCLES
        return {'unit': 'G wave-instr/s', 'valu_insts_per_launch': insts, 'achieved': round(achieved, 1),
                'peak': round(peak, 1), 'frac': round(achieved / peak, 4), 'clock_ghz': round(clk, 3),
                'source': os.path.relpath(path, REPO) + ' (SQ_INSTS_VALU, GRBM_GUI_ACTIVE)'}
    except (OSError, KeyError, ValueError):
        return None


def instrument(pipe, ctx, stages):
    """Wrap the pipeline's stages and the context's calls with synchronised
    wall-clock timers (diagnostics only: it serialises host and device)."""
    def wrap(obj, name, label):
        fn = getattr(obj, name)

        def timed(*a, **kw):
            ctx.sync()
            t = time.perf_counter()
            r = fn(*a, **kw)
            ctx.sync()
            acc = stages.setdefault(label, [0.0, 0])
            acc[0] += time.perf_counter() - t
            acc[1] += 1
            if name == 'map':
                stages.setdefault('_map_stats', []).append(ctx.map_stats())
            return r
        setattr(obj, name, timed)

    for name in ('index_build', 'map', 'map_counts', 'pileup', 'pileup_fetch'):
        wrap(ctx, name, 'ctx.' + name)
    for name in ('prelim', 'prelim_conseqs', 'map_to_reference', 'build_conseqs_filtered'):
        wrap(pipe, name, 'pipe.' + name)
    from micall_amd import pipeline as pl
    for name in ('counts_to_conseqs', 'filter_conseqs'):
        fn = getattr(pl, name)

        def timed(*a, _fn=fn, _label='host.' + name, **kw):
            t = time.perf_counter()
            r = _fn(*a, **kw)
            acc = stages.setdefault(_label, [0.0, 0])
            acc[0] += time.perf_counter() - t
            acc[1] += 1
            return r
        setattr(pl, name, timed)


def s2a_algo_bytes(text_rows, res_pairs, body_bytes):
    """k_s2a_merge's algorithmic bytes: read seq + qual of every mate of a
    merged pair, write the merged body, 16 B of results and 16 B of hashes
    per pair."""
    return text_rows + body_bytes + 32 * res_pairs


def bench_sam2aln(args):
    """sam2aln (micall_amd.sam2aln, mh_sam2aln_csv) over remap.csv text of
    one C2 remap pass: host CSV parse + upload + device merge/group + fetch,
    then the three CSV outputs."""
    import torch
    from micall_amd import _native
    from micall_amd.pipeline import RemapPipeline
    import og_sam2aln
    ctx = _native.Context(0)
    reads, quals = make_reads(args.pairs, block=0)
    ctx.reads_load_fixed(reads, quals, True)
    del reads, quals
    ctx.set_names(['M00000:1:000000000-AAAAA:1:1101:{}:{}'.format(1000 + i // 1000000,
                                                                         1000 + i % 1000000)
                         for i in range(args.pairs) for _ in (0, 1)])
    pipe = RemapPipeline(ctx)
    pipe.run(2.0 * args.pairs, max_iterations=1)
    text = ('qname,flag,rname,pos,mapq,cigar,rnext,pnext,tlen,seq,qual\n' +
            ctx.format_rows(1, 0, 2 * args.pairs)).encode()
    for _ in range(args.warmup):
        ctx.sam2aln_csv(text)
    torch.cuda.synchronize()
    ctx.profile(True)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        ctx.sam2aln_csv(text)
    elapsed = time.perf_counter() - t0
    kern = {k: ctx.profile_get(k) for k in ('k_s2a_merge', 'k_s2a_group')}
    t1 = time.perf_counter()
    outs = {w: ctx.sam2aln_output(w) for w in ('aligned', 'insert', 'failed')}
    t_out = time.perf_counter() - t1
    host_ms = ctx.sam2aln_timing()
    st = ctx.sam2aln_stats()
    merge_ms, merge_n = kern['k_s2a_merge']
    avg_s = merge_ms / 1e3 / max(merge_n, 1)
    # algorithmic bytes: every merged mate's seq + qual, the merged bodies
    body = sum(int(line.rsplit(',', 1)[1].__len__()) * int(line.split(',')[3])
               for line in outs['aligned'].splitlines()[1:])
    mate_bytes = 2 * 2 * READ_LEN * st[1]
    algo = s2a_algo_bytes(mate_bytes, st[1], body)
    achieved = algo / avg_s / 1e9 if avg_s > 0 else 0.0
    sample = min(20000, args.pairs)
    lines = text.decode().split('\n', 2 * sample + 1)
    stext = '\n'.join(lines[:2 * sample + 1]) + '\n'
    t2 = time.perf_counter()
    og_sam2aln.sam2aln(stext)
    cpu_s = time.perf_counter() - t2
    dev_ms = sum(v[0] for v in kern.values()) / args.steps
    out = {
        'metric': 'sam2aln read pairs/sec (remap.csv -> aligned/insert/failed)',
        'value': round(st[0] * args.steps / elapsed, 1), 'unit': 'pairs/s', 'n_gpus': 1,
        'steps': args.steps, 'warmup': args.warmup,
        'ms_per_step': round(1e3 * elapsed / args.steps, 3), 'higher_is_better': True,
        'scaling': 'weak', 'vs_baseline': None, 'dtype': 'u8', 'data': 'synthetic',
        'config': {'workload': 'sam2aln over the remap.csv of one C2 remap pass (1M pairs '
                               'of synthetic 2x251 HIV-1 pol reads), q-cutoff 15',
                   'pairs': st[0], 'merged': st[1], 'distinct': st[2], 'failed': st[3],
                   'csv_bytes': len(text)},
        'device_ms_per_step': round(dev_ms, 3),
        'device_pairs_per_s': round(st[0] / (dev_ms / 1e3), 1) if dev_ms > 0 else None,
        'output_format_ms': round(1e3 * t_out, 1),
        'host_ms_last_step': {'parse': round(host_ms[0], 1), 'device_call': round(host_ms[1], 1),
                              'format_aligned': round(host_ms[2], 1),
                              'format_insert': round(host_ms[3], 1),
                              'format_failed': round(host_ms[4], 1)},
        'roofline': {'kernel': 'k_s2a_merge', 'bound': 'hbm', 'achieved': round(achieved, 3),
                     'peak': HBM_PEAK_GBS, 'unit': 'GB/s', 'frac': round(achieved / HBM_PEAK_GBS, 6),
                     'traffic': read_pmc_traffic('k_s2a_merge', args.pairs, 'sam2aln'), 'algo_bytes_per_launch': algo,
                     'avg_launch_ms': round(1e3 * avg_s, 4), 'launches': merge_n},
        'kernels_ms_per_step': {k: round(v[0] / args.steps, 3) for k, v in kern.items()},
        'cpu_baseline': {'value': round(sample / cpu_s, 1), 'unit': 'pairs/s', 'cores': 1,
                         'kind': 'port',
                         'sample': 'first {} pairs of the same remap.csv through the pure-Python '
                                   'restatement oracle/og_sam2aln.py, {:.1f} s'.format(sample, cpu_s)},
    }
    print(json.dumps(out))
    ctx.close()


def _fastq_text(reads, quals, mate, tiles=8):
    """FASTQ text of one mate's reads with Illumina headers over `tiles` tiles."""
    n = reads.shape[0]
    out = []
    for i in range(n):
        out.append('@M00000:1:000000000-AAAAA:1:{}:{}:{} {}:N:0:1\n{}\n+\n{}\n'.format(
            1101 + i % tiles, 1000 + i // 1000, 1000 + i % 1000, mate,
            reads[i].tobytes().decode(), quals[i].tobytes().decode()))
    return ''.join(out).encode()


def bench_censor(args):
    """censor_fastq.censor (mh_censor_fastq) of the C2 R1 file (gzip in and
    out) with ~2 % bad (tile, cycle) pairs (BASELINE config C5's censor
    shape), and the FASTQ ingest of the pair (mh_reads_load_fastq)."""
    import gzip
    import random
    import tempfile
    import og_censor
    from micall_amd import _native, synth, projects
    pol = projects.load_default().seed_sequences()['HIV1B-pol-seed']
    d = synth.make_pairs(args.pairs, genomes={'HIV1B-pol-seed': pol}, genome_seed=SEED,
                         read_seed=SEED, block=0, read_len=READ_LEN)
    raw1 = _fastq_text(d['r1'], d['q1'], 1)
    raw2 = _fastq_text(d['r2'], d['q2'], 2)
    gz1 = gzip.compress(raw1, compresslevel=1)
    gz2 = gzip.compress(raw2, compresslevel=1)
    rng = random.Random(SEED)
    bad = sorted({(str(1101 + t), c) for t in range(8) for c in range(1, READ_LEN + 1)
                  if rng.random() < 0.02})
    from micall_amd import censor_fastq, session
    tmp = tempfile.mkdtemp(prefix='bench_fq_')
    p1, p2 = os.path.join(tmp, 'R1.fastq.gz'), os.path.join(tmp, 'R2.fastq.gz')
    with open(p1, 'wb') as f:
        f.write(gz1)
    with open(p2, 'wb') as f:
        f.write(gz2)
    pout = os.path.join(tmp, 'R1.censor.fastq.gz')
    rows = [{'tile': t, 'cycle': str(c)} for t, c in bad]

    def censor_file():
        # the drop-in as bin/micall calls it: file handles in and out
        with open(p1, 'rb') as src, open(pout, 'wb') as dst:
            censor_fastq.censor(src, iter(rows), dst, use_gzip=True)

    ctx = session.context()
    for _ in range(args.warmup):
        censor_file()
    ctx.profile(True)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        censor_file()
    elapsed = time.perf_counter() - t0
    host_ms = ctx.censor_timing()
    k_ms, k_n = ctx.profile_get('k_censor')
    # the in-memory entry (bytes in, bytes out: mh_censor_fastq) for comparison
    t3 = time.perf_counter()
    out, n_bases, total = ctx.censor_fastq(gz1, bad, True, True)
    mem_s = time.perf_counter() - t3
    # k_censor runs once per inflated piece (~32 MB of FASTQ): account per
    # file.  Algorithmic bytes: read and write every base and quality byte
    # once (the kernel censors in place), 16 B of spans per record.
    step_s = k_ms / 1e3 / max(args.steps, 1)
    algo = 2 * 2 * READ_LEN * args.pairs + 16 * args.pairs
    achieved = algo / step_s / 1e9 if step_s > 0 else 0.0
    pmc = read_pmc_traffic('k_censor', args.pairs, 'censor')
    try:
        with open(os.path.join(REPO, 'profiles', 'pmc_traffic_censor.json')) as f:
            pmc_launches = json.load(f)['kernels']['k_censor']['launches']
    except (OSError, KeyError, ValueError):
        pmc_launches = 1
    # FASTQ ingest of the pair (what prelim_map does first)
    t1 = time.perf_counter()
    ctx.reads_load_fastq(p1, p2)
    ingest_s = time.perf_counter() - t1
    import shutil
    shutil.rmtree(tmp, ignore_errors=True)
    sample = min(20000, args.pairs)
    stext = b'\n'.join(raw1.split(b'\n', 4 * sample)[:4 * sample]) + b'\n'
    t2 = time.perf_counter()
    og_censor.censor_bytes(stext, set(bad))
    cpu_s = time.perf_counter() - t2
    res = {
        'metric': 'censor reads/sec (FASTQ.gz in -> censored FASTQ.gz out)',
        'value': round(args.pairs * args.steps / elapsed, 1), 'unit': 'reads/s', 'n_gpus': 1,
        'steps': args.steps, 'warmup': args.warmup,
        'ms_per_step': round(1e3 * elapsed / args.steps, 3), 'higher_is_better': True,
        'scaling': 'weak', 'vs_baseline': None, 'dtype': 'u8', 'data': 'synthetic',
        'config': {'workload': 'censor of the C2 R1 file (1M synthetic 2x251 reads over 8 tiles, '
                               'gzip level 1 in, level 1 out), 2 % bad tile-cycles',
                   'reads': args.pairs, 'bad_cycles': len(bad), 'fastq_bytes': len(raw1),
                   'gz_bytes': len(gz1)},
        'host_ms_last_step': {'gunzip_split': round(host_ms[0], 1),
                              'device_call': round(host_ms[1], 1),
                              'rewrite_gzip': round(host_ms[2], 1)},
        'what': 'censor_fastq.censor() drop-in, file to file (single-member gzip R1 in, gzip out '
                'written with pwrite); in_memory_s: mh_censor_fastq on the same bytes in memory',
        'in_memory_s': round(mem_s, 3),
        'ingest_pair_s': round(ingest_s, 3),
        'ingest_reads_per_s': round(2 * args.pairs / ingest_s, 1),
        'roofline': {'kernel': 'k_censor', 'bound': 'hbm', 'achieved': round(achieved, 3),
                     'peak': HBM_PEAK_GBS, 'unit': 'GB/s', 'frac': round(achieved / HBM_PEAK_GBS, 6),
                     'traffic': None if pmc is None else pmc * pmc_launches,
                     'per': 'file (all pieces of one step)', 'algo_bytes': algo,
                     'kernel_ms_per_file': round(1e3 * step_s, 4), 'launches': k_n},
        'cpu_baseline': {'value': round(sample / cpu_s, 1), 'unit': 'reads/s', 'cores': 1,
                         'kind': 'port',
                         'sample': 'first {} reads of the same R1 (plain text) through the '
                                   'pure-Python restatement oracle/og_censor.py, {:.1f} s'.format(
                                       sample, cpu_s)},
    }
    print(json.dumps(res))
    ctx.close()


def bench_aln2counts(args):
    """aln2counts (micall_amd.aln2counts: mh_a2c_load_csv + k_a2c_count, the
    coordinate mapping with k_gotoh, mh_a2c_inserts, the CSV reports) over
    the aligned.csv that sam2aln makes from one C2 remap pass."""
    import io
    import tempfile
    import torch
    from micall_amd import session
    from micall_amd import aln2counts as a2c
    from micall_amd.pipeline import RemapPipeline
    import og_aln2counts
    ctx = session.context()
    reads, quals = make_reads(args.pairs, block=0)
    ctx.reads_load_fixed(reads, quals, True)
    del reads, quals
    ctx.set_names(['M00000:1:000000000-AAAAA:1:1101:{}:{}'.format(1000 + i // 1000000,
                                                                         1000 + i % 1000000)
                         for i in range(args.pairs) for _ in (0, 1)])
    pipe = RemapPipeline(ctx)
    pipe.run(2.0 * args.pairs, max_iterations=1)
    remap_text = ('qname,flag,rname,pos,mapq,cigar,rnext,pnext,tlen,seq,qual\n' +
                  ctx.format_rows(1, 0, 2 * args.pairs)).encode()
    ctx.sam2aln_csv(remap_text)
    del remap_text
    aligned = ctx.sam2aln_output('aligned')
    n_rows = aligned.count('\n') - 1
    seq_bytes = sum(len(line.rsplit(',', 1)[1]) for line in aligned.splitlines()[1:])

    # aligned.csv on disk, opened the way bin/micall hands it over
    tmp = tempfile.mkdtemp(prefix='bench_a2c_')
    path = os.path.join(tmp, 'aligned.csv')
    with open(path, 'w') as f:
        f.write(aligned)

    def step():
        # a fresh process aligns every consensus: no memoised alignment
        # survives from the previous step
        a2c.aligner.forget()
        outs = [io.StringIO() for _ in range(6)]
        with open(path) as f:
            a2c.aln2counts(f, *outs[:4], failed_align_csv=outs[4], coverage_summary_csv=outs[5])
        return outs
    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    ctx.profile(True)
    ctx.a2c_timing(a2c.SLOT_REPORT)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        outs = step()
    elapsed = time.perf_counter() - t0
    host_ms = ctx.a2c_timing(a2c.SLOT_REPORT)
    kern = {k: ctx.profile_get(k) for k in ('k_a2c_count', 'k_a2c_ins')}
    n_groups = ctx.a2c_load_csv(a2c.SLOT_REPORT, aligned, a2c._CODON_CHARS)
    bins = sum(-(-max(ctx.a2c_group(a2c.SLOT_REPORT, g)['ncod']) // 21) for g in range(n_groups))
    k_ms, k_n = kern['k_a2c_count']
    avg_s = k_ms / 1e3 / max(k_n, 1)
    # algorithmic bytes per launch: every row's seq once, its 24-B record,
    # and the counters (count + first row, 4 B each) of every bin: 21 codons
    # x 3 frames x (21 amino acids + 18 bases)
    algo = seq_bytes + 24 * n_rows + 2 * 4 * bins * 63 * 39
    achieved = algo / avg_s / 1e9 if avg_s > 0 else 0.0
    sample = min(3000, n_rows)
    lines = aligned.split('\n', sample + 1)
    stext = '\n'.join(lines[:sample + 1]) + '\n'
    t2 = time.perf_counter()
    og_aln2counts.aln2counts(stext, og_aln2counts.default_projects())
    cpu_s = time.perf_counter() - t2
    out = {
        'metric': 'aln2counts aligned rows/sec (aligned.csv -> nuc/amino/coord_ins/conseq/failed)',
        'value': round(n_rows * args.steps / elapsed, 1), 'unit': 'rows/s', 'n_gpus': 1,
        'steps': args.steps, 'warmup': args.warmup,
        'ms_per_step': round(1e3 * elapsed / args.steps, 3), 'higher_is_better': True,
        'scaling': 'weak', 'vs_baseline': None, 'dtype': 'u32', 'data': 'synthetic',
        'config': {'workload': 'aln2counts over the aligned.csv sam2aln makes from one C2 remap '
                               'pass (1M pairs of synthetic 2x251 HIV-1 pol reads; coordinate '
                               'regions PR, RT, INT)',
                   'rows': n_rows, 'groups': n_groups, 'seq_bytes': seq_bytes,
                   'csv_bytes': len(aligned)},
        'host_ms_last_load': {'parse': round(host_ms[0], 1),
                             'upload_count_fetch': round(host_ms[1], 1),
                             'inserts': round(host_ms[2] / args.steps, 1)},
        'roofline': {'kernel': 'k_a2c_count', 'bound': 'hbm', 'achieved': round(achieved, 3),
                     'peak': HBM_PEAK_GBS, 'unit': 'GB/s', 'frac': round(achieved / HBM_PEAK_GBS, 6),
                     'traffic': read_pmc_traffic('k_a2c_count', args.pairs, 'aln2counts'), 'algo_bytes_per_launch': algo,
                     'avg_launch_ms': round(1e3 * avg_s, 4), 'launches': k_n},
        'kernels_ms_per_step': {k: round(v[0] / args.steps, 3) for k, v in kern.items()},
        'cpu_baseline': {'value': round(sample / cpu_s, 1), 'unit': 'rows/s', 'cores': 1,
                         'kind': 'port',
                         'sample': 'first {} rows of the same aligned.csv through the pure-Python '
                                   'restatement oracle/og_aln2counts.py, {:.1f} s'.format(sample, cpu_s)},
    }
    print(json.dumps(out))


def _free_port():
    import socket
    with socket.socket() as s:
        s.bind(('127.0.0.1', 0))
        return s.getsockname()[1]


def _self_launch(args):
    """`bench.py --gpus N` (N > 1) without a launcher: start N ranks with
    torch.distributed.run as a CHILD process (never exec: nothing here has
    touched the GPU, and nothing will), relay rank 0's one JSON line and exit
    with the child's status.  The line is refused (exit 3) unless it reports
    the N ranks asked for (n_gpus and config.dist_world).  Other output of the
    ranks goes to stderr as it comes, so a long run shows progress."""
    import subprocess
    if args.stage not in ('remap', 'chain'):
        sys.exit('bench.py: --stage {} runs on one GPU; --gpus {} needs the remap or chain '
                 'stage'.format(args.stage, args.gpus))
    backend = os.environ.get('MICALL_BENCH_BACKEND', 'nccl')
    if backend == 'nccl':
        import torch
        ndev = torch.cuda.device_count()     # counts devices without initialising HIP
        if ndev < args.gpus:
            sys.exit('bench.py: --gpus {} but this node has {} GPU(s)'.format(args.gpus, ndev))
    cmd = [sys.executable, '-m', 'torch.distributed.run', '--nnodes=1',
           '--nproc-per-node', str(args.gpus), '--master-addr', '127.0.0.1',
           '--master-port', str(_free_port()), os.path.abspath(__file__)] + sys.argv[1:]
    env = dict(os.environ, MASTER_ADDR='127.0.0.1')
    proc = subprocess.Popen(cmd, env=env, stdout=subprocess.PIPE, text=True, bufsize=1)
    lines = []
    for ln in proc.stdout:
        if ln.startswith('{"metric"'):
            lines.append(ln.strip())
        else:
            sys.stderr.write(ln)
            sys.stderr.flush()
    rc = proc.wait()
    if rc != 0:
        sys.exit(rc)
    if len(lines) != 1:
        sys.exit('bench.py: expected one JSON line from rank 0, got {}'.format(len(lines)))
    d = json.loads(lines[0])
    if d.get('n_gpus') != args.gpus or d.get('config', {}).get('dist_world') != args.gpus:
        print('bench.py: refusing a line for {} rank(s) (dist_world {}) under --gpus {}'.format(
            d.get('n_gpus'), d.get('config', {}).get('dist_world'), args.gpus), file=sys.stderr)
        sys.exit(3)
    print(lines[0], flush=True)
    return 0


def _backend_name(world, backend):
    """The process group's backend as torch.distributed reports it (None on
    one rank, which runs no group)."""
    import torch.distributed as dist
    if world == 1 or not dist.is_initialized():
        return None
    return dist.get_backend()


def _rank_devices(world, device):
    """Every rank's device index, in rank order (rank 0's view)."""
    import torch.distributed as dist
    if world == 1:
        return [device.index]
    out = [None] * world
    dist.all_gather_object(out, device.index)
    return out


def _init_job(args):
    """torch.distributed for a leg run under torchrun (WORLD_SIZE > 1): the
    device of this rank (RCCL), or device LOCAL_RANK % devices with
    MICALL_BENCH_BACKEND=gloo (several ranks on one GPU, tests only).  The
    drop-ins' session uses the same device.  Returns (world, rank, device)."""
    import torch
    import torch.distributed as dist
    world = int(os.environ.get('WORLD_SIZE', '1'))
    rank = int(os.environ.get('RANK', '0'))
    local = int(os.environ.get('LOCAL_RANK', '0'))
    if world != args.gpus:
        # a line for a world other than the one asked for would be read as
        # an N-GPU figure it is not
        sys.exit('bench.py: --gpus {} but WORLD_SIZE {}: refusing to run'.format(args.gpus, world))
    backend = os.environ.get('MICALL_BENCH_BACKEND', 'nccl')
    ndev = torch.cuda.device_count()
    device = torch.device('cuda', local if backend == 'nccl' else local % max(ndev, 1))
    torch.cuda.set_device(device)
    os.environ['MICALL_HIP_DEVICE'] = str(device.index)
    if world > 1 and not dist.is_initialized():
        if backend == 'nccl':
            dist.init_process_group('nccl', device_id=device)
        else:
            dist.init_process_group(backend)
    return world, rank, device, backend


def bench_chain(args):
    """bin/micall's per-sample chain (bin/micall:116-188) file to file with
    the drop-ins, on the C2 input as a raw MiSeq pair arrives (each FASTQ one
    gzip member): censor R1, censor R2 (2 % bad tile-cycles) -> prelim_map
    -> remap -> sam2aln -> aln2counts, every output to a file.  One line:
    reads/s through the whole chain and seconds per stage.

    Under torchrun every rank holds --pairs pairs of the files (written
    untimed, in rank order) and runs the chain on the same paths, as a
    torchrun'd bin/micall does (python -m micall_amd.run_micall); each
    stage's time is the max over ranks.  The line reports the run with the
    median total (every run listed)."""
    import shutil
    import random
    import torch.distributed as dist
    world, rank, device, backend = _init_job(args)
    devices = _rank_devices(world, device)
    from micall_amd import (aln2counts, censor_fastq, prelim_map, remap, sam2aln, session, sharded_io,
                            synth)
    job = Job()
    work = job.shared_dir('bench_chain_')
    r1, r2 = os.path.join(work, 'R1.fastq.gz'), os.path.join(work, 'R2.fastq.gz')
    pairs = synth.make_pairs(args.pairs, genomes=bench_genomes('pol'), genome_seed=SEED,
                             read_seed=SEED, block=rank)
    write_fastq_gz(pairs, r1, r2, single=True, job=job)
    del pairs
    rng = random.Random(SEED)
    bad = [{'tile': str(1101 + t), 'cycle': str(sign * c)} for t in range(8) for sign in (1, -1)
           for c in range(1, READ_LEN + 1) if rng.random() < 0.02]
    P = {k: os.path.join(work, k) for k in ('c1.fastq.gz', 'c2.fastq.gz', 'prelim.csv', 'remap.csv',
                                            'align.csv', 'nuc.csv', 'amino.csv', 'insert.csv',
                                            'conseq.csv', 'remap_counts.csv')}

    lib = {}
    gap = float(os.environ.get('MICALL_CHAIN_GAP_S', '0'))   # diagnostics: idle seconds between stages
    throttled = []
    io = []

    def run():
        # bin/micall writes each sample's outputs into a fresh directory:
        # the previous run's outputs are removed, untimed, so that opening
        # them does not truncate 2.4 GB of files (an ext4 / overlay truncate
        # also makes close() flush the file: 0.3 s + 0.3 s on the box)
        if rank == 0:
            for path in P.values():
                if os.path.exists(path):
                    os.unlink(path)
        job.barrier()
        times, stats = {}, {}
        thr = cgroup_throttle()
        sharded_io.reset_stats()
        t = time.perf_counter()
        for src, dst in ((r1, P['c1.fastq.gz']), (r2, P['c2.fastq.gz'])):
            with open(src, 'rb') as f, open(dst, 'wb') as g:
                censor_fastq.censor(f, iter(bad), g, use_gzip=True)
        times['censor'] = time.perf_counter() - t
        stats['censor'] = dict(sharded_io.IO_STATS)
        time.sleep(gap)
        sharded_io.reset_stats()
        t = time.perf_counter()
        session.context().phase_times(reset=True)
        with open(P['prelim.csv'], 'w') as f:
            prelim_map.prelim_map(P['c1.fastq.gz'], P['c2.fastq.gz'], f, gzip=True)
            lib['prelim_map_call_s'] = round(time.perf_counter() - t, 4)
        times['prelim_map'] = time.perf_counter() - t
        stats['prelim_map'] = dict(sharded_io.IO_STATS)
        time.sleep(gap)
        lib['prelim_map'] = {k: round(v / 1e3, 4) for k, v in session.context().phase_times(reset=True).items()}
        sharded_io.reset_stats()
        t = time.perf_counter()
        with open(P['prelim.csv']) as pre, open(P['remap.csv'], 'w') as out, \
                open(P['remap_counts.csv'], 'w') as counts:
            remap.remap(P['c1.fastq.gz'], P['c2.fastq.gz'], pre, out, counts, gzip=True)
            lib['remap_call_s'] = round(time.perf_counter() - t, 4)
        times['remap'] = time.perf_counter() - t
        stats['remap'] = dict(sharded_io.IO_STATS)
        time.sleep(gap)
        lib['remap'] = {k: round(v / 1e3, 4) for k, v in session.context().phase_times(reset=True).items()}
        lib['prelim_source'] = session.stats.get('prelim_source')
        t = time.perf_counter()
        with open(P['remap.csv']) as rc, open(P['align.csv'], 'w') as al:
            sam2aln.sam2aln(rc, al)
        times['sam2aln'] = time.perf_counter() - t
        time.sleep(gap)
        t = time.perf_counter()
        with open(P['align.csv']) as al, open(P['nuc.csv'], 'w') as nuc, \
                open(P['amino.csv'], 'w') as amino, open(P['insert.csv'], 'w') as ins, \
                open(P['conseq.csv'], 'w') as conseq:
            aln2counts.aln2counts(al, nuc, amino, ins, conseq)
        times['aln2counts'] = time.perf_counter() - t
        throttled.append(throttle_since(thr))
        io.append(stats)
        # the job's time per stage: the slowest rank's
        names = list(times)
        us = job.gather([int(round(times[k] * 1e6)) for k in names] +
                        [int(round(sum(times.values()) * 1e6))])
        return {'stages': {k: float(us[:, j].max()) / 1e6 for j, k in enumerate(names)},
                'total': float(us[:, -1].max()) / 1e6,
                'per_rank_total': [round(float(x) / 1e6, 3) for x in us[:, -1]]}

    for _ in range(args.warmup):
        run()
    runs = [run() for _ in range(max(args.steps, 1))]
    if os.environ.get('MICALL_CHAIN_PROFILE') and world == 1:   # diagnostics: cProfile of one more run
        import cProfile
        import pstats
        pr = cProfile.Profile()
        pr.enable()
        run()
        pr.disable()
        pstats.Stats(pr, stream=sys.stderr).sort_stats('cumulative').print_stats(60)
    order = sorted(range(len(runs)), key=lambda k: runs[k]['total'])
    med = runs[order[(len(runs) - 1) // 2]]       # the median run (the lower one of an even count)
    total = med['total']
    sizes = {k: os.path.getsize(v) for k, v in P.items()}
    sizes['R1.fastq.gz'], sizes['R2.fastq.gz'] = os.path.getsize(r1), os.path.getsize(r2)
    rank_io = {}
    last = io[-1]
    for stage in ('censor', 'prelim_map', 'remap'):
        g = job.gather([last[stage]['fastq_file_bytes'], last[stage]['fastq_text_bytes'],
                        last[stage]['written_bytes']])
        rank_io[stage] = {'fastq_file_bytes': g[:, 0].tolist(), 'fastq_text_bytes': g[:, 1].tolist(),
                          'written_bytes': g[:, 2].tolist(), 'fastq_mode': last[stage]['fastq_mode']}
    job.barrier()
    if rank == 0:
        shutil.rmtree(work, ignore_errors=True)
        out = {
            'metric': 'bin/micall per-sample chain reads/sec (raw FASTQ.gz pair -> nuc/amino/conseq)',
            'value': round(2 * args.pairs * world / total, 1), 'unit': 'reads/s', 'n_gpus': world,
            'steps': len(runs), 'warmup': args.warmup, 'ms_per_step': round(1e3 * total, 1),
            'higher_is_better': True, 'scaling': 'weak', 'vs_baseline': None, 'dtype': 'u8',
            'data': 'synthetic',
            'config': {'workload': 'C2 input ({} synthetic 2x251 HIV-1 pol pairs per GPU), each FASTQ '
                                   'one gzip member; 2 % bad tile-cycles; censor R1 + R2, prelim_map, '
                                   'remap, sam2aln, aln2counts, drop-ins file to file'.format(args.pairs),
                       'pairs': args.pairs * world, 'pairs_per_gpu': args.pairs, 'bad_cycles': len(bad),
                       'parallelism': 'dp{}{}'.format(world, '' if world == 1 else ' ({}; every rank runs '
                                                       'the chain on the shared files)'.format(
                                                           'RCCL' if backend == 'nccl' else backend)),
                       'dist_world': world, 'dist_backend': _backend_name(world, backend),
                       'rank_devices': devices},
            'reported_run': 'median of {} runs by total time (the slowest rank\'s per stage)'.format(len(runs)),
            'stages_s': {k: round(v, 3) for k, v in med['stages'].items()},
            'all_runs_s': [round(r['total'], 3) for r in runs],
            'per_rank_total_s': med['per_rank_total'] if world > 1 else None,
            'per_rank_io_last_run': rank_io if world > 1 else None,
            'library_phases_s_last_run_rank0': lib,
            'cgroup_throttled_per_run': throttled[args.warmup:args.warmup + len(runs)],
            'bytes': sizes,
        }
        print(json.dumps(out))
    session.reset()
    if world > 1:
        job.barrier()
        dist.destroy_process_group()


def run_end_to_end(args):
    """The end_to_end legs of the default line, on every rank: the C2 input
    as many gzip members per file and as one member (bcl2fastq's layout),
    each file to file through the drop-ins; at N = 1 also the CPU
    file-to-file baseline on a bounded sample.  Skipped (with the reason)
    when the scratch file system cannot hold the files."""
    import shutil
    job = Job()
    layouts = ('members', 'single') if args.e2e_gzip == 'both' else (args.e2e_gzip,)
    work = job.shared_dir('micall_e2e_')
    out = {}
    try:
        # FASTQ (~0.6 GB) + prelim.csv and remap.csv (~1.2 GB each) per 1M pairs
        need = 3.2e9 * args.pairs / 1e6 * job.world
        free = shutil.disk_usage(work).free
        if free < 1.5 * need:
            skip = {'skipped': 'scratch file system {} has {:.1f} GB free, the files need '
                               '{:.1f} GB'.format(work, free / 1e9, need / 1e9)}
            return {k: skip for k in layouts}
        for layout in layouts:
            out[layout] = end_to_end(args.pairs, work, single_member=layout == 'single', job=job)
        if job.world == 1 and not args.no_cpu_baseline and 'members' in out:
            out['members']['cpu_baseline'] = cpu_end_to_end(args.cpu_e2e_sample, work)
            for layout in out:
                out[layout]['vs_cpu'] = round(out[layout]['value'] /
                                              out['members']['cpu_baseline']['value'], 2)
    finally:
        job.barrier()
        if job.rank == 0:
            shutil.rmtree(work, ignore_errors=True)
    return out


def main():
    ap = argparse.ArgumentParser(description=__doc__.split('\n\n')[0])
    ap.add_argument('--gpus', type=int, default=1)
    ap.add_argument('--steps', type=int, default=5)
    ap.add_argument('--warmup', type=int, default=2)
    ap.add_argument('--pairs', type=int, default=1000000, help='read pairs per GPU')
    ap.add_argument('--iterations', type=int, default=1,
                    help='cap on remap iterations per step (1: C2; 3 with --pairs 10000000: C3 on '
                         'one GPU); the reference\'s stopping rules still apply')
    ap.add_argument('--unpaired', action='store_true',
                    help='unpaired reads (--pairs reads per GPU; C5-style with --read-len 300)')
    ap.add_argument('--read-len', type=int, default=READ_LEN)
    ap.add_argument('--genomes', choices=('pol', 'hiv', 'all'), default='pol',
                    help='pol: HIV-1 pol sample genome (C2/C3/C5); hiv: mixed-region reads over '
                         'the HIV-1 seeds in proportion to length (C4); all: over every seed '
                         'region (the all-seed reading of C4)')
    ap.add_argument('--force-iterations', action='store_true',
                    help='run exactly --iterations remap passes per step (C3: "3 remap '
                         'iterations"), the stopping rules applying only after them')
    ap.add_argument('--cpu-sample', type=int, default=200000)
    ap.add_argument('--cpu-e2e-sample', type=int, default=20000,
                    help='pairs for the CPU end-to-end baseline (file to file)')
    ap.add_argument('--no-cpu-baseline', action='store_true')
    ap.add_argument('--parity-full', type=int, default=0, metavar='CHUNK',
                    help='after timing, check every record of every pass of the last step over '
                         'the whole input against og_map in chunks of CHUNK units (C3: 1000000)')
    ap.add_argument('--no-parity', action='store_true',
                    help='skip the parity leg (device records of the first --cpu-sample units '
                         'against the CPU oracle, after timing)')
    ap.add_argument('--no-e2e', action='store_true',
                    help='skip the end-to-end (file to file) leg of the default C2 run')
    ap.add_argument('--e2e-gzip', choices=('members', 'single', 'both'), default='both',
                    help='gzip layout of the end-to-end FASTQ input: 64 members per file '
                         '(as a parallel gzip writes it), one member (as bcl2fastq does), or '
                         'both legs (the default line carries both)')
    ap.add_argument('--breakdown', action='store_true',
                    help='time each pipeline stage (synchronising) and print it to stderr')
    ap.add_argument('--stage', choices=('remap', 'sam2aln', 'censor', 'aln2counts', 'chain'), default='remap',
                    help='remap: the headline hot path (default); sam2aln: the next stage '
                         '(SURVEY.md 8(f)) over the remap.csv of one C2 pass; censor: the '
                         'stage before (FASTQ censor of the C2 reads) plus the FASTQ ingest')
    args = ap.parse_args()
    if args.gpus > 1 and 'WORLD_SIZE' not in os.environ:
        return _self_launch(args)
    if args.stage == 'sam2aln':
        return bench_sam2aln(args)
    if args.stage == 'aln2counts':
        return bench_aln2counts(args)
    if args.stage == 'censor':
        return bench_censor(args)
    if args.stage == 'chain':
        return bench_chain(args)

    import torch
    import torch.distributed as dist
    from micall_amd import _native
    from micall_amd.pipeline import RemapPipeline, Shard

    world, rank, device, backend = _init_job(args)
    devices = _rank_devices(world, device)

    ctx = _native.Context(device.index)
    paired = not args.unpaired
    L = args.read_len
    reads, quals = make_reads(args.pairs, block=rank, read_len=L, paired=paired, genomes=args.genomes)
    ctx.reads_load_fixed(reads, quals, paired)
    # the first units of this rank's input, kept for the CPU baseline and
    # the parity leg (rank 0; N = 1 checks 200k pairs, N > 1 a 20k sample)
    sample = None
    if rank == 0 and (not args.no_parity or (world == 1 and not args.no_cpu_baseline)):
        k = min(args.cpu_sample if world == 1 else min(args.cpu_sample, 20000), args.pairs)
        k *= 2 if paired else 1
        sample = (reads[:k].copy(), quals[:k].copy())
    full_input = (reads, quals) if args.parity_full and rank == 0 else None
    del reads, quals
    shard = Shard(rank, world, read_base=rank * (1 if args.unpaired else 2) * args.pairs, device=device) if world > 1 else None
    pipe = RemapPipeline(ctx, shard=shard)
    raw_count = 2.0 * args.pairs * world     # lines(R1) / 2, remap.py:457

    def step():
        del pipe.log[:]
        return pipe.run(raw_count, max_iterations=args.iterations,
                        min_iterations=args.iterations if args.force_iterations else None)

    stages = {}
    if args.breakdown:
        instrument(pipe, ctx, stages)
    # extensions per mapping pass (host-side counters of the last mh_map; no sync)
    dp_log = []
    real_map = ctx.map

    def counted_map(*a, **kw):
        r = real_map(*a, **kw)
        dp_log.append(ctx.map_stats())
        return r
    ctx.map = counted_map

    for _ in range(args.warmup):
        step()
    ctx.profile(True)
    del dp_log[:]
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        conseqs, new_counts, _unm = step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=device)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())

    kernels = {k: ctx.profile_get(k) for k in ('k_seed', 'k_dp', 'k_rescue', 'k_dp_rescue', 'k_pair',
                                              'k_pileup')}
    dom = max(kernels, key=lambda k: kernels[k][0])
    dom_ms, dom_n = kernels[dom]
    # every launch of a mapping / pileup kernel processes this rank's pairs once
    # per unit (pair, or read when unpaired): SURVEY.md 8(d), 756 B per 2x251
    # pair, 445 B per unpaired 300-nt read
    unit_bytes = algo_bytes_per_pair(L) if paired else -(-L // 4) + -(-L // 8) + L + 32
    bytes_per_launch = unit_bytes * args.pairs
    avg_s = dom_ms / 1e3 / max(dom_n, 1)
    achieved = bytes_per_launch / avg_s / 1e9 if avg_s > 0 else 0.0
    total_pairs = args.pairs * world * args.steps
    value = (2 if paired else 1) * total_pairs / elapsed
    # DP cell updates (GCUPS next to the roofline): every
    # extension the full DP runs is read_len rows x the 31-diagonal band
    # (seeded diagonal +- 15, bowtie2's maxhalf); the ungapped fast path
    # resolves the rest without the DP
    ext = sum(int(m[1]) for m in dp_log)
    fast = sum(int(m[3]) for m in dp_log)
    rescue = sum(int(m[4]) for m in dp_log)
    cells = (ext - fast) * L * 31
    dp_ms = kernels['k_dp'][0] + kernels['k_dp_rescue'][0]

    # the file-to-file legs (every rank: under torchrun they are the sharded
    # drop-ins over files holding every rank's block)
    e2e_legs = {}
    if (not args.no_e2e and paired and L == READ_LEN and args.genomes == 'pol'
            and args.iterations == 1 and not args.force_iterations):
        e2e_legs = run_end_to_end(args)
    parity = None
    if rank == 0:
        cpu = cpu_result = None
        if world == 1 and not args.no_cpu_baseline and sample is not None:
            cpu, cpu_result = cpu_baseline(*sample, paired=paired, iterations=args.iterations,
                                           forced=args.force_iterations,
                                           workload='{}x{} {}'.format(2 if paired else 1, L, args.genomes))
        if sample is not None and not args.no_parity:
            parity = parity_check(ctx, pipe, sample, paired, cpu_result, device.index,
                                  iterations=args.iterations, forced=args.force_iterations)
            del cpu_result
        if full_input is not None:
            parity_whole = parity_full(ctx, pipe, full_input[0], full_input[1], paired, args.parity_full)
            if parity is None:
                parity = {}
            parity['whole_input'] = parity_whole
            full_input = None
        if cpu is not None:
            cpu['device_resident_vs_cpu'] = round(value / cpu['value'], 1)
        out = {
            'metric': METRIC, 'value': round(value, 1), 'unit': 'reads/s', 'n_gpus': world,
            'steps': args.steps, 'warmup': args.warmup,
            'ms_per_step': round(1e3 * elapsed / args.steps, 3), 'higher_is_better': True,
            'scaling': 'weak', 'vs_baseline': None, 'dtype': 'int32', 'data': 'synthetic',
            'config': {'workload': ('C5-style (mapping half): synthetic unpaired 1x{} nt HIV-1 pol reads'.format(L)
                                    if not paired else
                                    'C4-style: synthetic 2x{} nt mixed-region read pairs over the HIV-1 '
                                    'seeds {}'.format(L, ','.join(bench_genomes('hiv', L)))
                                    if args.genomes == 'hiv' else
                                    'C4-style, all seed regions: synthetic 2x{} nt read pairs over the {} '
                                    'seeds of >= 260 nt'.format(L, len(bench_genomes('all', L)))
                                    if args.genomes == 'all' else
                                    ('C2' if args.iterations == 1 else 'C3-style') +
                                    ': synthetic 2x{} nt HIV-1 pol read pairs'.format(L)) +
                                   ' (10% divergent '
                                   'sample genome, 0.5% errors), prelim_map end-to-end vs 74 seeds '
                                   '+ {} remap iteration(s) (--local vs consensus) + pileups, '
                                   'default projects.json'.format(args.iterations),
                       'remap_iterations_cap': args.iterations,
                       'pairs_per_gpu' if paired else 'reads_per_gpu': args.pairs, 'read_len': L,
                       'parallelism': ('dp1 (one GPU, no collective)' if world == 1 else
                                       'dp{} (read-pair shards, {} all-reduce of pileup '
                                       'counters)'.format(world, 'RCCL' if backend == 'nccl'
                                                          else backend)),
                       'dist_world': world, 'dist_backend': _backend_name(world, backend),
                       'rank_devices': devices},
            'roofline': {'kernel': dom, 'bound': 'hbm', 'achieved': round(achieved, 3),
                         'peak': HBM_PEAK_GBS, 'unit': 'GB/s',
                         'frac': round(achieved / HBM_PEAK_GBS, 6),
                         'traffic': (read_pmc_traffic(dom, args.pairs)
                                     if paired and L == READ_LEN and args.genomes == 'pol' else None),
                         'algo_bytes_per_launch': bytes_per_launch,
                         'avg_launch_ms': round(1e3 * avg_s, 4), 'launches': dom_n},
            'valu_issue': (read_valu_issue(dom, args.pairs, 1e3 * avg_s)
                           if paired and L == READ_LEN and args.genomes == 'pol' else None),
            'kernels_ms_per_step': {k: round(v[0] / args.steps, 3) for k, v in kernels.items()},
            'dp': {'extensions_per_step': ext // max(args.steps, 1),
                   'fast_path_per_step': fast // max(args.steps, 1),
                   'rescue_per_step': rescue // max(args.steps, 1),
                   'cells_per_step': cells // max(args.steps, 1),
                   'gcups': round(cells / (dp_ms / 1e3) / 1e9, 1) if dp_ms > 0 else None},
            'cpu_baseline': cpu,
            'parity': parity,
            'end_to_end': e2e_legs.get('members'),
            'end_to_end_single_member': e2e_legs.get('single'),
            'result': {'remap_iterations_run': len(pipe.log),
                       'conseqs': {k: len(v) for k, v in conseqs.items()},
                       'mapped_lines': dict(new_counts)},
        }
        print(json.dumps(out))
        if args.breakdown:
            print(json.dumps({'stage_ms_per_step': {k: round(v[0] * 1e3 / (args.steps + args.warmup), 3)
                                                    for k, v in stages.items() if not k.startswith('_')},
                              'map_stats': stages.get('_map_stats')}), file=sys.stderr)
    del sample
    ctx.close()
    if world > 1:
        dist.barrier()     # rank 0's untimed legs (parity) end before the group does
        dist.destroy_process_group()


if __name__ == '__main__':
    main()
