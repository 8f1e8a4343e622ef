#!/usr/bin/env python3
"""
tests/golden/gen_golden.py -- regenerates the committed golden vectors.

Runs ONLY in the dev container (needs /root/reference); the vectors it writes
(tests/golden/*.json) are data: inputs and the outputs the reference code
itself produced for them.  Sections:

  gotoh    every _gotoh2.align call made by the reference's own KATs
           (micall/alignment/tests/test.py) plus seeded random pairs, all
           answered by the reference extension built from its source.
  pileup   every remap.sam_to_conseqs call made by micall/tests/remap_test.py
           (recorded around the real function, so the expected value is what
           the code returns, not the test's stale expectation -- see
           SURVEY.md 4, testSeedsConvergedWithConfusingGap) plus synthetic
           SAMs produced by the oracle mapper on synthetic reads.
  sam2aln  every apply_cigar / merge_pairs / merge_inserts call made by
           micall/tests/sam2aln_test.py.
  splitter every MixedReferenceSplitter.split() call of remap_test.py and
           seeded random SAM texts: rows kept and split FASTQ texts.

  s2a      the reference's sam2aln() (the next stage) on
           every call micall/tests/sam2aln_test.py makes, on edge-case
           remap.csv texts derived from the e2e cases below, and on every
           e2e case's remap.csv: aligned.csv / insert.csv / failed.csv under
           tests/golden/sam2aln_e2e.json and tests/golden/e2e/<case>/.

  censor   the reference's parse_interop.read_errors / write_phix_csv,
           filter_quality.report_bad_cycles and censor_fastq.censor (the
           stage before prelim_map) on a synthetic
           ErrorMetricsOut.bin and synthetic multi-tile FASTQ files, run the
           way bin/micall:90-126 chains them (R2 with the exhausted bad-cycle
           reader), plus censor_fastq_test.py's scenarios:
           tests/golden/censor/.

  a2c      aln2counts (the stage after sam2aln): every
           call micall/tests/aln2counts_test.py makes on SequenceReport,
           InsertionWriter, SeedAmino and SeedNucleotide, recorded around the
           reference code with what each call wrote or returned
           (tests/golden/aln2counts_golden.json); the reference aln2counts()
           on every e2e case's aligned.csv (tests/golden/e2e/<case>/a2c_*.csv.gz)
           and on edge-case aligned.csv texts over a small project file cut
           from HIV-1 pol (tests/golden/aln2counts_edge.json).

  chain_tail  the rest of bin/micall's run_sample (:171-188) on each chain
           case's remap.csv: the reference sam2aln(remap_csv, aligned_csv)
           and aln2counts(aligned, nuc, amino, coord_ins, conseq) called as
           bin/micall calls them; align.csv, nuc.csv, amino.csv, insert.csv
           and conseq.csv under tests/golden/chain/<case>/.

  e2e      the stock reference prelim_map() + remap() (nthreads=1, so its
           pileup runs without a process pool and is deterministic) with
           oracle/shim_bin/bowtie2 standing in for bowtie2, on small committed
           FASTQ inputs (synthetic sets and some of micall/tests/microtest/);
           outputs prelim.csv, remap.csv, remap_counts.csv, remap_conseq.csv
           and the unmapped FASTQs under tests/golden/e2e/<case>/.

usage: python tests/golden/gen_golden.py [gotoh] [pileup] [sam2aln] [e2e]
"""
import gzip
import io
import json
import os
import random
import sys
import unittest

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, HERE)
sys.path.insert(0, os.path.join(REPO, 'oracle'))
sys.path.insert(0, os.path.join(REPO, 'micall-lite_amd'))

import refharness  # noqa: E402


def _run_suite(module):
    suite = unittest.defaultTestLoader.loadTestsFromModule(module)
    unittest.TextTestRunner(stream=io.StringIO(), verbosity=0).run(suite)


def gen_gotoh():
    refmod = refharness.setup()
    records = []
    real_align = refmod.align

    class Recorder:
        @staticmethod
        def align(s1, s2, gop, gep, is_global, alphabet, matrix):
            matrix = list(matrix)
            rec = dict(seq1=s1, seq2=s2, gop=gop, gep=gep, is_global=is_global,
                       alphabet=alphabet, matrix=matrix)
            try:
                a1, a2, score = real_align(s1, s2, gop, gep, is_global, alphabet, matrix)
                rec.update(aligned1=a1, aligned2=a2, score=score, error=None)
            except RuntimeError as ex:
                rec.update(error=str(ex))
                records.append(rec)
                raise
            records.append(rec)
            return a1, a2, score

    import micall.alignment.gotoh2 as g2
    g2._gotoh2 = Recorder
    import importlib.util
    spec = importlib.util.spec_from_file_location(
        'ref_alignment_kats', os.path.join(refharness.REF, 'micall', 'alignment', 'tests', 'test.py'))
    kat = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(kat)
    _run_suite(kat)
    n_kat = len(records)

    # seeded random pairs: nucleotide (HYPHY_NUC, global gop15/gep3 as in
    # remap.py:33 and ends-free) and amino (EmpHIV25 gop40/gep10 ends-free as
    # in aln2counts), including mutated copies so alignments are non-trivial.
    rng = random.Random(20261015)
    nuc = g2.Aligner(gop=15, gep=3, is_global=True, model='HYPHY_NUC')
    amino = g2.Aligner(gop=40, gep=10, is_global=False, model='EmpHIV25')

    def mutate(s, alpha, rate):
        out = []
        for c in s:
            r = rng.random()
            if r < rate:
                out.append(rng.choice(alpha))
            elif r < rate * 1.4:
                continue
            elif r < rate * 1.8:
                out.append(c + ''.join(rng.choice(alpha) for _ in range(rng.choice([1, 3]))))
            else:
                out.append(c)
        return ''.join(out) or alpha[0]

    for k in range(160):
        n = rng.choice([1, 2, 5, 17, 40, 97, 150, 300])
        a = ''.join(rng.choice('ACGT') for _ in range(n))
        b = mutate(a, 'ACGTN', rng.choice([0.05, 0.15, 0.3]))
        if rng.random() < 0.3:
            b = b[rng.randrange(len(b)):] or b
        nuc.is_global = (k % 2 == 0)
        nuc.gap_open_penalty = rng.choice([15, 10, 5])
        nuc.gap_extend_penalty = rng.choice([3, 1])
        try:
            nuc.align(a, b)
        except RuntimeError:
            pass
    for k in range(40):
        n = rng.choice([3, 10, 33, 80])
        a = ''.join(rng.choice('ARNDCQEGHILKMFPSTWYV') for _ in range(n))
        b = mutate(a, 'ARNDCQEGHILKMFPSTWYV*', 0.2)
        amino.is_global = (k % 3 == 0)
        try:
            amino.align(a, b)
        except RuntimeError:
            pass
    out = dict(source='reference _gotoh2.c built by oracle/Makefile; KATs from '
                      'micall/alignment/tests/test.py then seeded random pairs',
               n_kat=n_kat, cases=records)
    with open(os.path.join(HERE, 'gotoh_golden.json'), 'w') as f:
        json.dump(out, f, indent=0)
    print('gotoh: {} cases ({} from KATs)'.format(len(records), n_kat))


def _synthetic_sams():
    """SAM texts made by the oracle mapper on synthetic pol reads (local and
    end-to-end), so the pileup vectors exercise soft clips, indels and
    insertions the way the product sees them."""
    import oracle
    from micall_amd import synth, projects
    seeds = projects.load_default().seed_sequences()
    pol = seeds['HIV1B-pol-seed']
    texts = []
    for mode, n_pairs, seed in ((oracle.LOCAL, 300, 1), (oracle.E2E, 300, 2), (oracle.LOCAL, 60, 3)):
        pairs = synth.make_pairs(n_pairs, genome_seed=seed, read_seed=seed + 100,
                                 genomes={'HIV1B-pol-seed': pol}, indel_rate=0.01)
        names, seqs, quals = synth.interleave(pairs)
        refnames = ['HIV1B-pol-seed']
        ix = oracle.Index([pol], oracle.seed_len(mode))
        alns = oracle.map_reads(ix, oracle.params(mode), seqs, quals, True)
        lines = ['@HD\tVN:1.0\tSO:unsorted\n', '@SQ\tSN:HIV1B-pol-seed\tLN:%d\n' % len(pol)]
        for i in range(len(seqs)):
            lines.append('\t'.join(oracle.sam_fields(alns[i], oracle.qname_of(names[i], True),
                                                     seqs[i], quals[i], refnames)) + '\n')
        texts.append((''.join(lines), {'seeds': {'HIV1B-pol-seed': pol}}))
    return texts


def gen_pileup():
    refharness.setup()
    from micall.core import remap
    records = []
    real = remap.sam_to_conseqs

    def recorder(samfile, quality_cutoff=0, debug_reports=None, seeds=None, is_filtered=False,
                 worker_pool=None, filter_coverage=1, distance_report=None):
        text = samfile.getvalue() if hasattr(samfile, 'getvalue') else samfile.read()
        result = real(io.StringIO(text), quality_cutoff, debug_reports, seeds, is_filtered,
                      None, filter_coverage, distance_report)
        if debug_reports is None:
            records.append(dict(sam=text, quality_cutoff=quality_cutoff, seeds=seeds,
                                is_filtered=is_filtered, filter_coverage=filter_coverage,
                                conseqs=result,
                                distance_report=distance_report))
        return result

    remap.sam_to_conseqs = recorder
    import micall.tests.remap_test as rt
    _run_suite(rt)
    n_tests = len(records)
    for text, extra in _synthetic_sams():
        for q in (20, 0):
            recorder(io.StringIO(text), quality_cutoff=q, seeds=extra['seeds'])
        recorder(io.StringIO(text), quality_cutoff=20)
    remap.sam_to_conseqs = real
    out = dict(source='reference remap.sam_to_conseqs; remap_test.py calls then oracle-mapped '
                      'synthetic SAMs', n_tests=n_tests, cases=records)
    with open(os.path.join(HERE, 'pileup_golden.json'), 'w') as f:
        json.dump(out, f, indent=0)
    print('pileup: {} cases ({} from remap_test)'.format(len(records), n_tests))


def gen_sam2aln():
    refharness.setup()
    from micall.core import sam2aln
    records = []
    originals = {}

    def wrap(name):
        fn = getattr(sam2aln, name)
        originals[name] = fn

        def recorder(*args, **kwargs):
            rec = dict(fn=name, args=list(args), kwargs=kwargs)
            try:
                res = fn(*args, **kwargs)
            except RuntimeError as ex:
                rec['error'] = str(ex)
                records.append(rec)
                raise
            rec['result'] = res
            records.append(rec)
            return res
        setattr(sam2aln, name, recorder)

    for name in ('apply_cigar', 'merge_pairs', 'merge_inserts'):
        wrap(name)
    import micall.tests.sam2aln_test as st
    _run_suite(st)
    for name, fn in originals.items():
        setattr(sam2aln, name, fn)

    def enc(x):
        if isinstance(x, dict):
            return {'__dict__': [[enc(k), enc(v)] for k, v in x.items()]}
        if isinstance(x, (list, tuple)):
            return [enc(v) for v in x]
        return x
    out = dict(source='reference sam2aln helpers as called by micall/tests/sam2aln_test.py',
               cases=[enc(r) for r in records])
    with open(os.path.join(HERE, 'sam2aln_golden.json'), 'w') as f:
        json.dump(out, f, indent=0)
    print('sam2aln: {} calls'.format(len(records)))


def gen_splitter():
    """Every MixedReferenceSplitter.split() call of the reference's
    MixedReferenceSplitterTest (remap_test.py:594-716), plus seeded random
    SAM texts (string-compared MAPQs such as '8' vs '44', tied MAPQ, equal
    AS, unmapped flags, lone mates): input text, the rows split() yields and
    the split FASTQ text per reference."""
    refharness.setup()
    from micall.core import remap as R
    records = []

    class Memory(R.MixedReferenceSplitter):
        def create_split_file(self, refname, direction):
            return io.StringIO()

        def close_split_file(self, split_file):
            pass

    real_split = R.MixedReferenceSplitter.split

    def record(text, source):
        sp = Memory()
        try:
            rows = list(real_split(sp, io.StringIO(text)))
            rec = dict(source=source, sam=text, rows=rows,
                       splits=[[k, f1.getvalue(), f2.getvalue()] for k, (f1, f2) in sp.splits.items()])
        except Exception as ex:      # e.g. a tied MAPQ with no AS:i tag
            rec = dict(source=source, sam=text, raises=type(ex).__name__)
        records.append(rec)

    def recorder(self, sam_lines):
        text = sam_lines.getvalue() if hasattr(sam_lines, 'getvalue') else ''.join(sam_lines)
        record(text, 'remap_test.py MixedReferenceSplitterTest')
        return real_split(self, io.StringIO(text))
    R.MixedReferenceSplitter.split = recorder
    import micall.tests.remap_test as rt
    suite = unittest.defaultTestLoader.loadTestsFromTestCase(rt.MixedReferenceSplitterTest)
    unittest.TextTestRunner(stream=io.StringIO(), verbosity=0).run(suite)
    R.MixedReferenceSplitter.split = real_split
    n_tests = len(records)
    rng = random.Random(4242)
    refs = ['HIV1B-gag-seed', 'HIV1B-pol-seed', 'HIV1B-env-seed']
    for t in range(40):
        lines = ['@HD\tVN:1.0\tSO:unsorted\n'] + ['@SQ\tSN:%s\tLN:9000\n' % r for r in refs]
        for q in range(rng.randint(1, 30)):
            qname = 'M01:%d:%d' % (t, q)
            seqs = [''.join(rng.choice('ACGTN') for _ in range(rng.randint(1, 12))) for _ in (0, 1)]
            quals = [''.join(rng.choice('#5<AFGJ') for _ in s) for s in seqs]
            r1, r2 = rng.choice(refs), rng.choice(refs)
            kind = rng.random()
            f1, f2 = 0x1 | 0x40, 0x1 | 0x80
            if kind < 0.15:
                f1 |= 0x4
                f2 |= 0x8
            elif kind < 0.25:
                f2 |= 0x4
                f1 |= 0x8
            mapqs = [rng.choice(['0', '1', '8', '11', '23', '42', '44', '255']) for _ in (0, 1)]
            if rng.random() < 0.3:
                mapqs[1] = mapqs[0]
            scores = [rng.choice([-20, 0, 15, 100, 200]) for _ in (0, 1)]
            if rng.random() < 0.3:
                scores[1] = scores[0]
            rn = [r2 if r1 != r2 else '=', r1 if r1 != r2 else '=']
            mates = []
            for k, (flag, ref, nxt) in enumerate(((f1, r1, rn[0]), (f2, r2, rn[1]))):
                tags = ['AS:i:%d' % scores[k]] if t % 4 != 3 or rng.random() > 0.05 else ['YT:Z:DP']
                mates.append('\t'.join([qname, str(flag), ref, str(rng.randint(1, 900)), mapqs[k],
                                         '%dM' % len(seqs[k]), nxt, '1', '0', seqs[k], quals[k]]
                                        + tags) + '\n')
            if rng.random() < 0.5:
                mates.reverse()
            if rng.random() < 0.05:
                mates = mates[:1]          # lone mate
            lines += mates
        record(''.join(lines), 'seeded random')
    with open(os.path.join(HERE, 'splitter_golden.json'), 'w') as f:
        json.dump(dict(source='reference remap.MixedReferenceSplitter.split', n_tests=n_tests,
                       cases=records), f, indent=0)
    print('splitter: {} cases ({} from remap_test)'.format(len(records), n_tests))


E2E_MICROTESTS = ['1234A-V3LOOP_S1', '2000A-V3LOOP_S2', '2010A-V3LOOP_S3', '2020A-GP41_S4',
                  '2030A-V3LOOP_S5', '2040A-HLA-B_S6', '2050A-V3LOOP_S7', '2060A-V3LOOP_S8',
                  '2070A-PR_S9', '2080A-V3LOOP_S10', '2090A-HCV_S11',
                  '2100A-HCV-1337B-V3LOOP_S12']
# BASELINE config C1: the reference's own example input (9,600 pairs of
# simulated HIV-1 subtype C pol reads named CONSENSUS_C-N/1, /2)
EXAMPLE = ('c1_example', 'examples/HIV1C-pol_S1_L001_R{}_001.fastq.gz')


def _gz_write(path, data):
    """gzip with a fixed header (mtime 0), so regenerating unchanged data
    leaves the committed bytes unchanged."""
    if isinstance(data, str):
        data = data.encode()
    with open(path, 'wb') as raw, gzip.GzipFile(fileobj=raw, mode='wb', mtime=0) as f:
        f.write(data)


def _garbage(pairs, n, seed):
    """Replace the first n pairs by random sequence (reads that map nowhere)."""
    import numpy as np
    rng = np.random.default_rng(seed)
    for key in ('r1', 'r2'):
        if pairs[key] is not None:
            pairs[key][:n] = np.frombuffer(b'ACGT', dtype=np.uint8)[
                rng.integers(0, 4, size=pairs[key][:n].shape)]
    return pairs


def _half_diverged(seq, keep, sub_rate, seed):
    """seq's first `keep` bases, then a sample of the rest at sub_rate."""
    import numpy as np
    from micall_amd import synth
    rng = np.random.Generator(np.random.PCG64(seed))
    return seq[:keep] + synth.sample_genome(seq[keep:], rng, sub_rate, 0.002).tobytes().decode()


def _chimeric(seeds):
    """Pairs from HIV-1 gag and env sample genomes; 60 pairs of each have
    their R2 swapped with the other's, so their mates map to two seeds and
    the final remap pass hands them to MixedReferenceSplitter (RNEXT names
    the other reference, remap.py:787-850)."""
    import numpy as np
    from micall_amd import synth
    gag = synth.make_pairs(500, genomes={'HIV1B-gag-seed': seeds['HIV1B-gag-seed']},
                           genome_seed=111, read_seed=112, sub_rate=0.06)
    env = synth.make_pairs(500, genomes={'HIV1B-env-seed': seeds['HIV1B-env-seed']},
                           genome_seed=113, read_seed=114, sub_rate=0.06)
    out = {'block': 0, 'n': 1000}
    for key in ('r1', 'q1', 'r2', 'q2'):
        out[key] = np.concatenate([gag[key], env[key]])
    for key in ('r2', 'q2'):
        a = out[key][:60].copy()
        out[key][:60] = out[key][500:560]
        out[key][500:560] = a
    return out


def _e2e_cases():
    """(name, synthetic pairs) for every synthetic end-to-end case."""
    from micall_amd import projects, synth
    seeds = projects.load_default().seed_sequences()
    pol = {'HIV1B-pol-seed': seeds['HIV1B-pol-seed']}
    cases = []

    def syn(name, n, genomes, **kw):
        cases.append((name, synth.make_pairs(n, genomes={g: seeds[g] for g in genomes}, **kw)))

    syn('syn_pol', 1500, ['HIV1B-pol-seed'], genome_seed=101, read_seed=102)
    syn('syn_pol_indel', 600, ['HIV1B-pol-seed'], genome_seed=103, read_seed=104, indel_rate=0.01)
    syn('syn_hiv3', 900, ['HIV1B-pol-seed', 'HIV1B-gag-seed', 'HIV1B-env-seed'],
        genome_seed=105, read_seed=106)
    syn('syn_unpaired300', 500, ['HIV1B-pol-seed'], genome_seed=107, read_seed=108, read_len=300,
        paired=False)
    cases.append(('syn_chimera', _chimeric(seeds)))
    # SARS-CoV-2 (29.9 kb): a sample identical to the seed over its first
    # 600 nt and 22 % divergent after that, plus 10 % random pairs.  The
    # consensus improves a stretch at a time, every pass maps more reads than
    # the one before and the mapped fraction stays below 0.95, so only
    # MAX_REMAPS (remap.py:602-603) ends the loop, after the third pass
    cases.append(('syn_maxremaps', _garbage(synth.make_pairs(
        2000, genomes={'SARS-CoV-2': _half_diverged(seeds['SARS-CoV-2'], 600, 0.22, 77)},
        genome_seed=78, read_seed=79, sub_rate=0.0, indel_rate=0.0), 200, 5)))
    # 18 % divergence: no seed reaches the count threshold, the loop never
    # runs (the reference then fails removing temp.fasta, remap.py:653-655)
    cases.append(('syn_noseed', _garbage(synth.make_pairs(1500, genomes=pol, genome_seed=201,
                                                          read_seed=202, sub_rate=0.18),
                                         150, 5)))
    return cases


def _fastq_text(pairs, mate):
    from micall_amd import synth
    r, q = pairs['r%d' % mate], pairs['q%d' % mate]
    return ''.join('{}\n{}\n+\n{}\n'.format(synth.read_name(pairs['block'], i, mate),
                                             r[i].tobytes().decode(), q[i].tobytes().decode())
                   for i in range(pairs['n']))


def _reference_e2e(r1, r2, keep):
    """Stock prelim_map() + remap() in a scratch directory; returns
    ({file name: text}, exception raised by remap or None)."""
    import shutil
    import tempfile
    from micall.core.prelim_map import prelim_map
    from micall.core.remap import remap
    shim = os.path.join(REPO, 'oracle', 'shim_bin')
    work = tempfile.mkdtemp(prefix='e2e_')
    cwd = os.getcwd()
    os.chdir(work)   # the reference writes split FASTQs into the cwd
    raised = None
    try:
        prelim = os.path.join(work, 'prelim.csv')
        with open(prelim, 'w') as handle:
            prelim_map(r1, r2, handle, bt2_path=os.path.join(shim, 'bowtie2'),
                       bt2build_path=os.path.join(shim, 'bowtie2-build-s'), nthreads=1,
                       gzip=True, work_path=work)
        names = ('remap.csv', 'remap_counts.csv', 'remap_conseq.csv', 'unmapped1.fastq',
                 'unmapped2.fastq')
        outs = {k: open(os.path.join(work, k), 'w') for k in names}
        try:
            with open(prelim) as pre:
                remap(r1, r2, pre, outs['remap.csv'], outs['remap_counts.csv'],
                      outs['remap_conseq.csv'], outs['unmapped1.fastq'], outs['unmapped2.fastq'],
                      work_path=work, bt2_path=os.path.join(shim, 'bowtie2'),
                      bt2build_path=os.path.join(shim, 'bowtie2-build-s'), nthreads=1, gzip=True,
                      keep=keep)
        except Exception as ex:    # recorded, see remap.py:653-655
            name = getattr(ex, 'filename', None)
            raised = '{} {}'.format(type(ex).__name__, os.path.basename(name) if name else ex)
        for f in outs.values():
            f.close()
        texts = {}
        for k in ('prelim.csv',) + names:
            with open(os.path.join(work, k)) as f:
                texts[k] = f.read()
        return texts, raised
    finally:
        os.chdir(cwd)
        shutil.rmtree(work, ignore_errors=True)


def gen_e2e(only=None):
    """The stock reference pipeline on every e2e input.  Outputs are taken
    from a run with keep=True (the reference completes); when the remap loop
    never ran, the same input is run again with keep=False and the exception
    the reference raises is recorded in reference_raises.txt."""
    import shutil
    refharness.setup()
    out_root = os.path.join(HERE, 'e2e')
    os.makedirs(out_root, exist_ok=True)
    inputs = []
    for name, pairs in _e2e_cases():
        d = os.path.join(out_root, name)
        os.makedirs(d, exist_ok=True)
        r1 = os.path.join(d, 'R1.fastq.gz')
        r2 = os.path.join(d, 'R2.fastq.gz') if pairs['r2'] is not None else None
        for mate, path in ((1, r1), (2, r2)):
            if path is not None:
                _gz_write(path, _fastq_text(pairs, mate))
        inputs.append((name, r1, r2))
    micro = os.path.join(refharness.REF, 'micall', 'tests', 'microtest')
    for stem in E2E_MICROTESTS:
        name = 'micro_' + stem.split('_')[0]
        d = os.path.join(out_root, name)
        os.makedirs(d, exist_ok=True)
        paths = []
        for mate in ('R1', 'R2'):
            src = os.path.join(micro, '{}_L001_{}_001.fastq'.format(stem, mate))
            dst = os.path.join(d, mate + '.fastq.gz')
            with open(src, 'rb') as fi:
                _gz_write(dst, fi.read())
            paths.append(dst)
        inputs.append((name, paths[0], paths[1]))
    name, pattern = EXAMPLE
    d = os.path.join(out_root, name)
    os.makedirs(d, exist_ok=True)
    paths = []
    for mate in (1, 2):
        dst = os.path.join(d, 'R{}.fastq.gz'.format(mate))
        shutil.copyfile(os.path.join(refharness.REF, pattern.format(mate)), dst)
        paths.append(dst)
    inputs.append((name, paths[0], paths[1]))
    for name, r1, r2 in inputs:
        if only and name not in only:
            continue
        d = os.path.join(out_root, name)
        texts, raised = _reference_e2e(r1, r2, keep=True)
        assert raised is None, (name, raised)
        for k, text in texts.items():
            _gz_write(os.path.join(d, k + '.gz'), text)
        marker = os.path.join(d, 'reference_raises.txt')
        if os.path.exists(marker):
            os.remove(marker)
        if 'remap-1 ' not in texts['remap_counts.csv']:
            _, raised = _reference_e2e(r1, r2, keep=False)
            if raised:
                with open(marker, 'w') as f:
                    f.write(raised + '\n')
        print('e2e:', name, '' if raised is None else '(reference raises without keep)')


def _s2a_edge_texts():
    """remap.csv texts that reach every branch of parse_sam / merge_pairs:
    built from the first rows of the syn_pol case's remap.csv."""
    import csv
    import gzip
    import random
    src = os.path.join(HERE, 'e2e', 'syn_pol', 'remap.csv.gz')
    with gzip.open(src, 'rt') as f:
        rows = list(csv.DictReader(f))
    fields = ['qname', 'flag', 'rname', 'pos', 'mapq', 'cigar', 'rnext', 'pnext', 'tlen', 'seq',
              'qual']
    rng = random.Random(31)

    def text(rs):
        out = io.StringIO()
        w = csv.DictWriter(out, fields, lineterminator='\n')
        w.writeheader()
        for r in rs:
            w.writerow(r)
        return out.getvalue()

    mapped = [r for r in rows if r['cigar'] != '*'][:400]
    cases = {}
    base = [dict(r) for r in mapped]
    cases['plain'] = text(base)
    # failures: unmatched mate, '*' CIGAR, different references, low quality
    t = [dict(r) for r in mapped[:120]]
    del t[5]
    t[10]['cigar'] = '*'
    t[20]['rname'] = 'OTHER-REF'
    for r in t[30:34]:
        r['qual'] = '#' * len(r['seq'])
    for r in t[40:42]:
        r['qual'] = ''.join(rng.choice('#+5') for _ in r['seq'])
    cases['failures'] = text(t)
    # indels, soft clips, far-apart and overlapping mates, unpaired flags,
    # duplicated qnames, escaped quality characters
    t = [dict(r) for r in mapped[:160]]
    for k in range(0, 40, 2):
        r = t[k]
        n = len(r['seq'])
        a = 5 + k
        if k % 4 == 0:
            r['cigar'] = '{}M3I{}M'.format(a, n - a - 3)
        else:
            r['cigar'] = '{}S{}M4D{}M'.format(3, a, n - a - 3)
    for k in range(40, 60, 2):
        t[k + 1]['pos'] = str(int(t[k]['pos']) + 700)
    for k in range(60, 70):
        t[k]['flag'] = str(int(t[k]['flag']) & ~1)
    dup = [dict(t[80]), dict(t[81]), dict(t[80])]
    t += dup
    for k in range(90, 100):
        q = list(t[k]['qual'])
        q[3] = ','
        q[7] = '"'
        t[k]['qual'] = ''.join(q)
    for k in range(100, 110):
        t[k]['seq'] = t[k]['seq'][:50] + 'N' * 10 + t[k]['seq'][60:]
    cases['shapes'] = text(t)
    # identical merged sequences (counts > 1, rank ties broken by offset/seq)
    t = []
    for k in range(0, 60, 2):
        for rep in range(1 + k % 3):
            a, b = dict(mapped[k]), dict(mapped[k + 1])
            a['qname'] = b['qname'] = '{}_{}'.format(mapped[k]['qname'], rep)
            t += [a, b]
    rng.shuffle(t)
    cases['duplicates'] = text(t)
    # two references interleaved
    t = []
    for k in range(0, 80, 2):
        a, b = dict(mapped[k]), dict(mapped[k + 1])
        if k % 3 == 0:
            a['rname'] = b['rname'] = 'HIV1B-gag-seed'
        t += [a, b]
    cases['two_refs'] = text(t)
    return cases


def gen_censor():
    import base64
    import csv
    import gzip
    import random
    import struct
    refharness.setup()
    from micall.core.censor_fastq import censor
    from micall.core.filter_quality import report_bad_cycles
    from micall.core.parse_interop import read_errors, write_phix_csv
    from micall_amd import projects, synth
    out_dir = os.path.join(HERE, 'censor')
    os.makedirs(out_dir, exist_ok=True)
    rng = random.Random(7)
    # -- synthetic ErrorMetricsOut.bin: 4 tiles, 2x251 + 2x8 cycles, ~3 % bad,
    # some cycles missing, one tile absent
    lengths = [251, 8, 8, 251]
    recs = []
    for tile in (1101, 1102, 1103, 2101):
        for cycle in range(1, sum(lengths) + 1):
            if rng.random() < 0.01:
                continue
            rate = rng.choice([0.1, 0.25, 0.5, 1.0, 2.0]) if rng.random() > 0.03 else 7.5 + rng.random() * 10
            recs.append(struct.pack('<HHHfLLLLL', 1, tile, cycle, rate, 1, 2, 3, 4, 5))
    rng.shuffle(recs)
    binary = struct.pack('!BB', 3, 30) + b''.join(recs)

    class Named(io.BytesIO):
        name = 'ErrorMetricsOut.bin'
    quality = io.StringIO()
    summary = {}
    write_phix_csv(quality, read_errors(Named(binary)), lengths, summary)
    bad = io.StringIO()
    tiles_csv = io.StringIO()
    report_bad_cycles(io.StringIO(quality.getvalue()), bad, tiles_csv)
    # -- synthetic FASTQ pair, tiles 1101-1104 (1104 has no metrics)
    pol = projects.load_default().seed_sequences()['HIV1B-pol-seed']
    pairs = synth.make_pairs(1500, genomes={'HIV1B-pol-seed': pol}, genome_seed=9, read_seed=10)
    fq = {1: [], 2: []}
    for i in range(pairs['n']):
        tile = 1101 + i % 4
        for mate, (r, q) in ((1, (pairs['r1'], pairs['q1'])), (2, (pairs['r2'], pairs['q2']))):
            name = '@M01841:45:000000000-A5FEG:1:{}:{}:{} {}:N:0:9'.format(tile, 1000 + i, 2000 + i, mate)
            fq[mate].append('{}\n{}\n+\n{}\n'.format(name, r[i].tobytes().decode(),
                                                     q[i].tobytes().decode()))
    raw = {m: ''.join(v).encode() for m, v in fq.items()}
    results = {}
    reader = csv.DictReader(io.StringIO(bad.getvalue()))

    class WriteBytes(io.BytesIO):
        mode = 'wb'        # GzipFile(fileobj=...) takes its mode from the file

    class ReadBytes(io.BytesIO):
        mode = 'rb'
    for mate in (1, 2):
        src = ReadBytes(gzip.compress(raw[mate]))
        dest = WriteBytes()
        summ = io.StringIO()
        censor(src, reader, dest, use_gzip=True, summary_file=summ)   # R2: exhausted reader
        results[mate] = (gzip.decompress(dest.getvalue()), summ.getvalue())
    for mate in (1, 2):
        with gzip.open(os.path.join(out_dir, 'R{}.fastq.gz'.format(mate)), 'wb') as f:
            f.write(raw[mate])
        with gzip.open(os.path.join(out_dir, 'R{}.censor.fastq.gz'.format(mate)), 'wb') as f:
            f.write(results[mate][0])
    # -- censor_fastq_test.py scenarios (its StringIO.StringIO set-up does
    # not run on Python 3; the same texts through BytesIO)
    one = (b'@M01841:45:000000000-A5FEG:1:1101:5296:13227 1:N:0:9\nACGT\n+\nAAAA\n')
    rev = one.replace(b' 1:N', b' 2:N')
    two = one + b'@M01841:45:000000000-A5FEG:1:1102:1234:12345 1:N:0:9\nTGCA\n+\nBBBB\n'
    scen = [(one, []), (one, [('1101', '3')]), (one, [('1101', '3'), ('1101', '4')]),
            (one, [('1102', '3')]), (rev, [('1101', '3')]), (rev, [('1101', '-3')]),
            (two, [('1101', '2'), ('1102', '3')]), (b'', []),
            (one.replace(b'AAAA', b'AACC'), [('1101', '3')]),
            (one.replace(b'ACGT\n', b'ACGT  \r\n'), [('1101', '1'), ('1101', '4')]),
            (two, [('1101', '1'), ('1101', '2'), ('1101', '3'), ('1101', '4')])]
    cases = []
    for text, bc in scen:
        dest, summ = io.BytesIO(), io.StringIO()
        censor(io.BytesIO(text), [dict(tile=t, cycle=c) for t, c in bc], dest, use_gzip=False,
               summary_file=summ)
        cases.append(dict(fastq=text.decode(), bad_cycles=bc, censored=dest.getvalue().decode(),
                          summary=summ.getvalue()))
    golden = dict(
        source='reference micall.core parse_interop / filter_quality / censor_fastq outputs',
        read_lengths=lengths, error_metrics_b64=base64.b64encode(binary).decode(),
        quality_csv=quality.getvalue(), phix_summary=summary, bad_cycles_csv=bad.getvalue(),
        bad_tiles_csv=tiles_csv.getvalue(), summary_r1=results[1][1], summary_r2=results[2][1],
        cases=cases)
    with open(os.path.join(out_dir, 'censor_golden.json'), 'w') as f:
        json.dump(golden, f, indent=0)
    print('censor: {} bad cycles, {} scenarios'.format(bad.getvalue().count('\n') - 1, len(cases)))


def gen_interop_edge():
    """Edge cases of the reference's write_phix_csv and report_bad_cycles:
    duplicate (tile, cycle) records, cycle 0, gaps at a lane's start and end,
    index cycles, lanes with only one direction, blank and bad rates inside
    a run, a tile that comes back after another, rates that are not
    numbers after the first bad cycle; plus seeded random tables.
    tests/golden/censor/interop_edge.json."""
    import random
    refharness.setup()
    from micall.core.filter_quality import report_bad_cycles
    from micall.core.parse_interop import write_phix_csv

    def rec(tile, cycle, rate):
        return dict(lane=1, tile=tile, cycle=cycle, error_rate=rate)
    phix = [
        ('dups_and_gaps', [rec(1101, 3, 0.5), rec(1101, 3, 0.25), rec(1101, 5, 1.0),
                           rec(1101, 5, 1.0), rec(1101, 6, 2.0), rec(1101, 22, 0.5),
                           rec(1101, 27, 8.0)], [6, 2, 2, 6]),
        ('cycle_zero', [rec(1102, 0, 0.5), rec(1102, 1, 0.5), rec(1102, 4, 0.75)], [4, 4]),
        ('reverse_only', [rec(1103, 9, 0.5), rec(1103, 12, 0.75), rec(1101, 11, 9.5)], [4, 4, 4]),
        ('index_only', [rec(1101, 5, 0.5), rec(1101, 6, 0.5)], [4, 4, 4]),
        ('no_index', [rec(2101, c, 0.125 * c) for c in (1, 2, 4, 5, 8)], [4, 4]),
        ('short_lengths', [rec(1101, c, 1.5) for c in range(1, 12)], [3, 2, 3]),
        ('empty', [], [5, 5]),
    ]
    rng = random.Random(11)
    for k in range(6):
        lengths = [rng.randint(3, 12), rng.randint(0, 3), rng.randint(3, 12)]
        if k % 2:
            lengths = [lengths[0], lengths[1], lengths[1], lengths[2]]
        recs = [rec(rng.choice((1101, 1102, 2101)), rng.randint(0, sum(lengths) + 2),
                    rng.choice((0.1, 0.5, 2.0, 7.5, 12.0))) for _ in range(rng.randint(5, 40))]
        phix.append(('random%d' % k, recs, lengths))
    phix_out = []
    for name, recs, lengths in phix:
        out, summary = io.StringIO(), {}
        write_phix_csv(out, iter([dict(r) for r in recs]), lengths, summary)
        phix_out.append(dict(name=name, records=recs, read_lengths=lengths, csv=out.getvalue(),
                             summary=summary))
    quality = [
        ('blank_mid_run', 'tile,cycle,errorrate\n1101,1,0.5\n1101,2,\n1101,3,0.5\n1101,-1,0.5\n'
                          '1101,-2,9.0\n1101,-3,0.1\n'),
        ('tile_returns', 'tile,cycle,errorrate\n1101,1,8.0\n1101,2,0.5\n1102,1,0.5\n1102,2,7.5\n'
                         '1101,1,0.5\n1101,2,7.49\n1101,3,7.5\n'),
        ('direction_flips', 'tile,cycle,errorrate\n1101,1,0.5\n1101,-1,8.0\n1101,2,0.5\n'
                            '1101,-2,0.5\n1101,0,9.0\n'),
        ('missing_column', 'tile,cycle,errorrate\n1101,1,0.5\n1101,2\n1101,3,0.5\n'),
        ('not_a_number_after_bad', 'tile,cycle,errorrate\n1101,1,8.0\n1101,2,oops\n1101,3,0.5\n'),
        ('all_good', 'tile,cycle,errorrate\n1101,1,0.5\n1101,-1,0.5\n'),
        ('header_only', 'tile,cycle,errorrate\n'),
    ]
    for k in range(6):
        lines = ['tile,cycle,errorrate']
        for _ in range(rng.randint(3, 30)):
            rate = rng.choice(('0.5', '1.0', '', '7.5', '7.4', '12'))
            lines.append('{},{},{}'.format(rng.choice((1101, 1102)), rng.choice((1, 2, -1, -2, 3)),
                                           rate))
        quality.append(('random%d' % k, '\n'.join(lines) + '\n'))
    quality_out = []
    for name, text in quality:
        bad, tiles = io.StringIO(), io.StringIO()
        report_bad_cycles(io.StringIO(text), bad, tiles)
        quality_out.append(dict(name=name, quality_csv=text, bad_cycles_csv=bad.getvalue(),
                                bad_tiles_csv=tiles.getvalue()))
    path = os.path.join(HERE, 'censor', 'interop_edge.json')
    with open(path, 'w') as f:
        json.dump(dict(source='reference micall.core parse_interop.write_phix_csv / '
                              'filter_quality.report_bad_cycles outputs',
                       phix=phix_out, quality=quality_out), f, indent=0)
    print('interop_edge: {} phix tables, {} quality tables'.format(len(phix_out), len(quality_out)))


def _error_metrics(lengths, tiles, bad, seed):
    """A version-3 ErrorMetricsOut.bin: every (tile, cycle) of the run, the
    (tile, run cycle) pairs in `bad` at an error rate >= 7.5.  A bad cycle
    makes every later cycle of its tile and read bad (filter_quality.py:
    report_bad_cycles), so the bad entries sit in the reads' last cycles, as
    phiX error rates climb at the end of a run."""
    import random
    import struct
    rng = random.Random(seed)
    recs = []
    for tile in tiles:
        for cycle in range(1, sum(lengths) + 1):
            rate = (7.5 + rng.random() * 10 if (tile, cycle) in bad
                    else rng.choice([0.1, 0.3, 0.6, 1.2]))
            recs.append(struct.pack('<HHHfLLLLL', 1, tile, cycle, rate, 1, 2, 3, 4, 5))
    rng.shuffle(recs)
    return struct.pack('!BB', 3, 30) + b''.join(recs)


def gen_chain():
    """BASELINE C5's chain as bin/micall:91-169 runs it, on the stock
    reference: read_errors -> write_phix_csv -> report_bad_cycles -> censor
    (R1; a paired run would censor R2 with the exhausted DictReader,
    bin/micall:116,126) -> prelim_map -U -> remap, on a synthetic
    ErrorMetricsOut.bin (~2 % bad tile-cycles) and unpaired 1x300 reads over
    4 tiles.  Every intermediate and final file is kept under
    tests/golden/chain/<case>/."""
    import csv
    import gzip
    import shutil
    import tempfile
    refharness.setup()
    from micall.core.censor_fastq import censor
    from micall.core.filter_quality import report_bad_cycles
    from micall.core.parse_interop import read_errors, write_phix_csv
    from micall.core.prelim_map import prelim_map
    from micall.core.remap import remap
    from micall_amd import projects, synth
    shim = os.path.join(REPO, 'oracle', 'shim_bin')
    seeds = projects.load_default().seed_sequences()
    for name, pairs_kw, lengths in (
            ('c5_unpaired300', dict(n=800, paired=False, read_len=300), [300, 8, 8, 300]),
            ('c5_paired251', dict(n=600, paired=True, read_len=251), [251, 8, 8, 251])):
        out = os.path.join(HERE, 'chain', name)
        os.makedirs(out, exist_ok=True)
        work = tempfile.mkdtemp(prefix='chain_')
        cwd = os.getcwd()
        os.chdir(work)
        try:
            tiles = (1101, 1102, 1103, 1104)
            interop = os.path.join(work, 'ErrorMetricsOut.bin')
            # ~2 % of the (tile, cycle) entries bad: the last 20 cycles of
            # read 1 on tile 1102 and the last 30 of read 2 on tile 1104
            r1_end, r2_end = lengths[0], sum(lengths)
            bad = ({(1102, c) for c in range(r1_end - 19, r1_end + 1)} |
                   {(1104, c) for c in range(r2_end - 29, r2_end + 1)})
            with open(interop, 'wb') as f:
                f.write(_error_metrics(lengths, tiles, bad, 11))
            pairs = synth.make_pairs(pairs_kw['n'], genomes={'HIV1B-pol-seed': seeds['HIV1B-pol-seed']},
                                     genome_seed=301, read_seed=302, read_len=pairs_kw['read_len'],
                                     paired=pairs_kw['paired'])
            fastqs = []
            for mate in ((1, 2) if pairs_kw['paired'] else (1,)):
                r, q = pairs['r%d' % mate], pairs['q%d' % mate]
                text = ''.join('@M01841:45:000000000-A5FEG:1:{}:{}:{} {}:N:0:9\n{}\n+\n{}\n'.format(
                    tiles[i % 4], 1000 + i, 2000 + i, mate, r[i].tobytes().decode(),
                    q[i].tobytes().decode()) for i in range(pairs['n']))
                path = os.path.join(work, 'S1_L001_R{}_001.fastq.gz'.format(mate))
                _gz_write(path, text)
                fastqs.append(path)
            # bin/micall censor_fastqs (:91-129)
            with open(interop, 'rb') as f:
                records = read_errors(f)
                with open('quality.csv', 'w') as q:
                    write_phix_csv(out_file=q, records=records, read_lengths=lengths)
            with open('quality.csv') as f1, open('bad_cycles.csv', 'w') as f2:
                report_bad_cycles(f1, f2)
            bad_cycles = csv.DictReader(open('bad_cycles.csv'))
            censored = []
            for k, src in enumerate(fastqs):
                dst = src.replace('.fastq', '.censor.fastq')
                with open(src, 'rb') as fi, open(dst, 'wb') as fo:
                    censor(src=fi, bad_cycles_reader=bad_cycles, dest=fo, use_gzip=True)
                censored.append(dst)
            r1, r2 = censored[0], censored[1] if len(censored) > 1 else None
            with open('prelim.csv', 'w') as handle:
                prelim_map(fastq1=r1, fastq2=r2, prelim_csv=handle, gzip=True,
                           bt2_path=os.path.join(shim, 'bowtie2'),
                           bt2build_path=os.path.join(shim, 'bowtie2-build-s'), nthreads=1,
                           work_path=work)
            names = ('remap.csv', 'remap_counts.csv', 'remap_conseq.csv', 'unmapped1.fastq',
                     'unmapped2.fastq')
            outs = {k: open(k, 'w') for k in names}
            with open('prelim.csv') as pre:
                remap(r1, r2, pre, outs['remap.csv'], outs['remap_counts.csv'],
                      outs['remap_conseq.csv'], outs['unmapped1.fastq'], outs['unmapped2.fastq'],
                      work_path=work, bt2_path=os.path.join(shim, 'bowtie2'),
                      bt2build_path=os.path.join(shim, 'bowtie2-build-s'), nthreads=1, gzip=True,
                      keep=True)
            for f in outs.values():
                f.close()
            shutil.copyfile(interop, os.path.join(out, 'ErrorMetricsOut.bin'))
            for k, src in enumerate(fastqs):
                shutil.copyfile(src, os.path.join(out, 'R{}.fastq.gz'.format(k + 1)))
                with gzip.open(censored[k], 'rb') as f:
                    _gz_write(os.path.join(out, 'R{}.censor.fastq.gz'.format(k + 1)), f.read().decode())
            for k in ('quality.csv', 'bad_cycles.csv', 'prelim.csv') + names:
                with open(k) as f:
                    _gz_write(os.path.join(out, k + '.gz'), f.read())
            with open(os.path.join(out, 'read_lengths.json'), 'w') as f:
                json.dump(lengths, f)
            print('chain:', name)
        finally:
            os.chdir(cwd)
            shutil.rmtree(work, ignore_errors=True)


def gen_chain_tail():
    """bin/micall:171-188 after remap, on the chain cases' remap.csv."""
    import gzip
    refharness.setup()
    from micall.core.aln2counts import aln2counts
    from micall.core.sam2aln import sam2aln
    for name in ('c5_unpaired300', 'c5_paired251'):
        d = os.path.join(HERE, 'chain', name)
        with gzip.open(os.path.join(d, 'remap.csv.gz'), 'rt') as f:
            text = f.read()
        align = io.StringIO()
        sam2aln(remap_csv=io.StringIO(text), aligned_csv=align)
        outs = {k: io.StringIO() for k in ('nuc', 'amino', 'insert', 'conseq')}
        aln2counts(aligned_csv=io.StringIO(align.getvalue()), nuc_csv=outs['nuc'],
                   amino_csv=outs['amino'], coord_ins_csv=outs['insert'],
                   conseq_csv=outs['conseq'])
        _gz_write(os.path.join(d, 'align.csv.gz'), align.getvalue())
        for k, v in outs.items():
            _gz_write(os.path.join(d, k + '.csv.gz'), v.getvalue())
        print('chain tail:', name, align.getvalue().count('\n') - 1, 'aligned rows')


def gen_s2a():
    import gzip
    refharness.setup()
    from micall.core import sam2aln as ref_s2a
    real = ref_s2a.sam2aln
    records = []

    def recorder(remap_csv, aligned_csv, insert_csv=None, failed_csv=None, nthreads=None):
        text = remap_csv.read()
        remap_csv.seek(0)
        real(remap_csv, aligned_csv, insert_csv, failed_csv, nthreads)
        records.append(dict(source='micall/tests/sam2aln_test.py', remap_csv=text,
                            aligned=aligned_csv.getvalue(),
                            insert=insert_csv.getvalue() if insert_csv else None,
                            failed=failed_csv.getvalue() if failed_csv else None))
    import micall.tests.sam2aln_test as st
    st.sam2aln = recorder
    _run_suite(st)
    st.sam2aln = real
    n_tests = len(records)

    def run(text):
        al, ins, fa = io.StringIO(), io.StringIO(), io.StringIO()
        real(io.StringIO(text), al, ins, fa)
        return al.getvalue(), ins.getvalue(), fa.getvalue()

    for name, text in _s2a_edge_texts().items():
        al, ins, fa = run(text)
        records.append(dict(source='edge case ' + name, remap_csv=text, aligned=al, insert=ins,
                            failed=fa))
    with open(os.path.join(HERE, 'sam2aln_e2e.json'), 'w') as f:
        json.dump(dict(source='reference micall.core.sam2aln.sam2aln outputs', cases=records), f,
                  indent=0)
    for case in sorted(os.listdir(os.path.join(HERE, 'e2e'))):
        d = os.path.join(HERE, 'e2e', case)
        with gzip.open(os.path.join(d, 'remap.csv.gz'), 'rt') as f:
            text = f.read()
        for name, body in zip(('aligned.csv', 'insert.csv', 'failed.csv'), run(text)):
            _gz_write(os.path.join(d, name + '.gz'), body)
    print('s2a: {} calls ({} from sam2aln_test)'.format(len(records), n_tests))

A2C_OUTPUTS = ('nuc', 'amino', 'coord_ins', 'conseq', 'failed', 'coverage')


def _a2c_reference(A, text, json_path=None):
    outs = {k: io.StringIO() for k in A2C_OUTPUTS}
    A.aln2counts(io.StringIO(text), outs['nuc'], outs['amino'], outs['coord_ins'],
                 outs['conseq'], failed_align_csv=outs['failed'],
                 coverage_summary_csv=outs['coverage'], json=json_path)
    return {k: v.getvalue() for k, v in outs.items()}


def _a2c_edge_config():
    """A small project file: seeds cut from HIV-1 pol, coordinate references
    translated from them (one with an inserted and a deleted amino acid), a
    seed linked to two projects, one without a coordinate region, one in no
    project."""
    from micall_amd import projects, translation
    pol = projects.load_default().seed_sequences()['HIV1B-pol-seed']
    s1, s2, s3 = pol[:420], pol[600:900], pol[1200:1350]
    aa1 = translation.translate(s1[30:390])
    c1 = aa1[:40] + 'W' + aa1[40:80] + aa1[81:]
    return {'projects': {
        'P1': {'max_variants': 0, 'regions': [
            {'coordinate_region': 'C1', 'seed_region_names': ['S1-seed']},
            {'coordinate_region': 'C1b', 'seed_region_names': ['S1-seed']}]},
        'P2': {'max_variants': 0, 'regions': [
            {'coordinate_region': 'C2', 'seed_region_names': ['S2-seed', 'S1-seed']},
            {'coordinate_region': None, 'seed_region_names': ['S3-seed']}]}},
        'regions': {
            'S1-seed': {'is_nucleotide': True, 'reference': [s1[:200], s1[200:]]},
            'S2-seed': {'is_nucleotide': True, 'reference': [s2]},
            'S3-seed': {'is_nucleotide': True, 'reference': [s3]},
            'S4-seed': {'is_nucleotide': True, 'reference': [pol[2000:2100]]},
            'C1': {'is_nucleotide': False, 'reference': [c1]},
            'C1b': {'is_nucleotide': False, 'reference': [translation.translate(s1[:150])]},
            'C2': {'is_nucleotide': False, 'reference': [translation.translate(s2, 1)[5:90]]}}}


def _a2c_edge_texts(cfg, n_texts=16, seed=77):
    """aligned.csv texts over cfg: samples with an inserted / deleted codon,
    substitutions, N, '-' (single and whole codons), 'n' gaps, junk reads
    that do not align, tied counts, several groups and a group key that
    comes back later (a new groupby group)."""
    rng = random.Random(seed)
    seqs = {k: ''.join(v['reference']) for k, v in cfg['regions'].items() if v['is_nucleotide']}
    texts = []
    for t in range(n_texts):
        keys = [(rng.choice(sorted(seqs)), rng.choice(['15', '15', '20']))
                for _ in range(rng.randint(1, 4))]
        if t % 4 == 3 and len(keys) > 1:
            keys.append(keys[0])
        rows = []
        for name, qcut in keys:
            sample = list(seqs[name])
            if rng.random() < 0.6:
                k = rng.randrange(30, len(sample) - 30) // 3 * 3
                sample[k:k] = list(rng.choice(['GGG', 'AAC', 'TTT']))
            if rng.random() < 0.4:
                k = rng.randrange(30, len(sample) - 30) // 3 * 3
                del sample[k:k + 3]
            sample = ''.join(sample)
            seen = set()
            for rank in range(rng.randint(1, 25)):
                if rng.random() < 0.08:
                    s = ''.join(rng.choice('ACGT') for _ in range(rng.randint(10, 60)))
                    off = rng.randint(0, 40)
                else:
                    off = rng.randint(0, max(0, len(sample) - 30))
                    s = list(sample[off:off + rng.randint(6, 140)])
                    for i in range(len(s)):
                        r = rng.random()
                        if r < 0.03:
                            s[i] = rng.choice('ACGT')
                        elif r < 0.05:
                            s[i] = 'N'
                    if rng.random() < 0.2 and len(s) > 12:
                        i = rng.randrange(3, len(s) - 6)
                        w = rng.randint(1, 5)
                        s[i:i + w] = ['n'] * w
                    if rng.random() < 0.15 and len(s) > 9:
                        i = rng.randrange(0, len(s) - 3)
                        w = rng.choice([1, 3])
                        s[i:i + w] = ['-'] * w
                    s = ''.join(s).strip('-')
                if not s or (off, s) in seen:
                    continue
                seen.add((off, s))
                rows.append('{},{},{},{},{},{}\n'.format(name, qcut, rank,
                                                         rng.choice([1, 1, 2, 3, 5, 8, 13, 40]),
                                                         off, s))
        texts.append('refname,qcut,rank,count,offset,seq\n' + ''.join(rows))
    texts.append('refname,qcut,rank,count,offset,seq\n')
    texts.append('')
    return texts


def gen_a2c():
    import copy
    import gzip
    import tempfile
    refharness.setup()
    from micall.core import aln2counts as A
    from micall.core import project_config as PC

    # Python-3 harness fixes, no algorithm touched: ProjectConfig.load keeps
    # json_file.name, which io.StringIO lacks, and the tests call both
    # StringIO() and StringIO.StringIO().
    def load(self, json_file):
        self.json_file = getattr(json_file, 'name', None)
        self.config = json.load(json_file)
    PC.ProjectConfig.load = load
    import micall.tests.aln2counts_test as T

    class _SIO(io.StringIO):
        StringIO = io.StringIO
    T.StringIO = _SIO
    st = {'depth': 0, 'calls': None, 'tags': {}}

    def tag(obj):
        t = st['tags'].get(id(obj))
        if t is None:
            t = st['tags'][id(obj)] = 'o{}'.format(len(st['tags']))
        return t

    def plain(v):
        return sorted(v) if isinstance(v, (set, frozenset)) else list(v) if isinstance(v, tuple) else v

    def wrap(cls, name, kind):
        fn = getattr(cls, name)

        def wrapper(self, *args, **kwargs):
            top = st['depth'] == 0 and st['calls'] is not None
            st['depth'] += 1
            try:
                entry = {'op': name, 'obj': tag(self)} if top else None
                f = n0 = summary = None
                if kind == 'read':
                    rows = [dict(r) for r in args[0]]
                    args = (rows,) + args[1:]
                    if top:
                        entry.update(rows=rows, config=copy.deepcopy(self.projects.config),
                                     overrides=[[k[0], k[1], list(v)] for k, v in
                                                getattr(self, 'overrides', {}).items()])
                elif kind == 'file':
                    f = args[0]
                    summary = kwargs.get('coverage_summary')
                    if top:
                        entry['file'] = tag(f)
                        if summary is not None:
                            entry['summary_in'] = dict(summary)
                elif kind == 'ins':
                    f = (self.insert_writer if isinstance(self, A.SequenceReport) else self)._rec_file
                    if top:
                        entry['args'] = [plain(a) for a in args]
                        entry['kwargs'] = {k: plain(v) for k, v in kwargs.items()}
                elif kind == 'args' and top:
                    entry['args'] = [plain(a) for a in args]
                    entry['kwargs'] = {k: plain(v) for k, v in kwargs.items()}
                if f is not None:
                    n0 = len(f.getvalue())
                try:
                    res = fn(self, *args, **kwargs)
                except Exception as ex:
                    if top:
                        entry['raises'] = type(ex).__name__
                        st['calls'].append(entry)
                    raise
                if top:
                    if f is not None:
                        entry['out'] = f.getvalue()[n0:]
                    if summary is not None:
                        entry['summary_out'] = dict(summary)
                    if kind == 'args':
                        entry['result'] = res
                    st['calls'].append(entry)
                return res
            finally:
                st['depth'] -= 1
        setattr(cls, name, wrapper)

    def wrap_init(cls, describe):
        fn = cls.__init__

        def init(self, *args, **kwargs):
            top = st['depth'] == 0 and st['calls'] is not None
            st['depth'] += 1
            try:
                f = (args[0] if args else kwargs['insert_file']) if cls is A.InsertionWriter else None
                n0 = len(f.getvalue()) if f is not None else 0
                fn(self, *args, **kwargs)
                if f is not None:
                    self._rec_file = f
                if top:
                    entry = {'op': cls.__name__, 'obj': tag(self)}
                    entry.update(describe(self, args, kwargs))
                    if f is not None:
                        entry['out'] = f.getvalue()[n0:]
                    st['calls'].append(entry)
            finally:
                st['depth'] -= 1
        cls.__init__ = init

    wrap_init(A.InsertionWriter, lambda s, a, k: {'file': tag(a[0] if a else k['insert_file'])})
    wrap_init(A.SequenceReport, lambda s, a, k: {'writer': tag(a[0]), 'cutoffs': list(a[2])})
    wrap_init(A.SeedAmino, lambda s, a, k: {'index': a[0], 'nucs': [tag(n) for n in s.nucleotides]})
    wrap_init(A.SeedNucleotide, lambda s, a, k: {})
    wrap(A.SequenceReport, 'read', 'read')
    for name in ('write_amino_header', 'write_nuc_header', 'write_consensus_header',
                 'write_nuc_variants_header', 'write_failure_header', 'write_amino_counts',
                 'write_nuc_counts', 'write_consensus', 'write_failure', 'write_nuc_variants'):
        wrap(A.SequenceReport, name, 'file')
    wrap(A.SequenceReport, 'write_insertions', 'ins')
    wrap(A.InsertionWriter, 'write', 'ins')
    for name in ('start_group', 'add_nuc_read'):
        wrap(A.InsertionWriter, name, 'args')
    for name in ('count_aminos', 'get_report', 'get_consensus'):
        wrap(A.SeedAmino, name, 'args')
    for name in ('count_nucleotides', 'get_report', 'get_consensus'):
        wrap(A.SeedNucleotide, name, 'args')

    def each(suite):
        for t in suite:
            if isinstance(t, unittest.TestSuite):
                yield from each(t)
            else:
                yield t
    scripts = []
    for test in each(unittest.defaultTestLoader.loadTestsFromModule(T)):
        st['calls'], st['tags'] = [], {}
        test.run(unittest.TestResult())
        scripts.append({'test': '.'.join(test.id().split('.')[-2:]), 'calls': st['calls']})
    st['calls'] = None
    with open(os.path.join(HERE, 'aln2counts_golden.json'), 'w') as f:
        json.dump({'source': 'reference micall.core.aln2counts classes as called by '
                             'micall/tests/aln2counts_test.py', 'scripts': scripts}, f, indent=0)
    n_calls = sum(len(s['calls']) for s in scripts)
    print('a2c: {} scripts, {} calls'.format(len(scripts), n_calls))

    # the reference aln2counts() on every e2e case
    for case in sorted(os.listdir(os.path.join(HERE, 'e2e'))):
        d = os.path.join(HERE, 'e2e', case)
        with gzip.open(os.path.join(d, 'aligned.csv.gz'), 'rt') as f:
            text = f.read()
        for k, body in _a2c_reference(A, text).items():
            _gz_write(os.path.join(d, 'a2c_{}.csv.gz'.format(k)), body)
        print('a2c e2e:', case)

    # edge cases over a small project file
    cfg = _a2c_edge_config()
    tmp = tempfile.mkdtemp(prefix='a2c_')
    path = os.path.join(tmp, 'projects.json')
    with open(path, 'w') as f:
        json.dump(cfg, f)
    cases = []
    for text in _a2c_edge_texts(cfg):
        try:
            cases.append({'text': text, 'outputs': _a2c_reference(A, text, path)})
        except Exception as ex:
            print('a2c edge: reference raised {!r}; case dropped'.format(ex))
    with open(os.path.join(HERE, 'aln2counts_edge.json'), 'w') as f:
        json.dump({'source': 'reference micall.core.aln2counts.aln2counts on edge-case texts',
                   'config': cfg, 'cases': cases}, f, indent=0)
    print('a2c edge: {} cases'.format(len(cases)))


if __name__ == '__main__':
    which = sys.argv[1:] or ['gotoh', 'pileup', 'sam2aln', 'splitter', 'e2e', 's2a', 'censor',
                             'a2c']
    for w in which:
        globals()['gen_' + w]()
