"""GPU parity: the HIP path through the C-ABI against the CPU oracle on the
same seeded inputs (bit-exact: every SAM field and CIGAR op, every pileup
counter), and against the reference-generated golden vectors."""
import json
import os
import re
from collections import Counter

import numpy as np
import pytest

import oracle
from micall_amd import _native, projects, synth

pytestmark = pytest.mark.gpu

SEEDS = projects.load_default().seed_sequences()
POL = SEEDS['HIV1B-pol-seed']


@pytest.fixture(scope='module')
def ctx():
    c = _native.Context(0)
    yield c
    c.close()


def _oracle_alns(refseqs, mode, seqs, quals, paired):
    ix = oracle.Index(refseqs, oracle.seed_len(mode))
    out = oracle.map_reads(ix, oracle.params(mode), seqs, quals, paired)
    return np.frombuffer(bytes(out), dtype=_native.ALN_DTYPE)[:len(seqs)]


def _gpu_alns(ctx, names, refseqs, mode, seqs, quals, paired):
    ctx.index_build(names, refseqs, oracle.seed_len(mode))
    ctx.reads_load(seqs, quals, paired)
    ctx.map(_native.params(mode))
    return ctx.fetch()


def _assert_same(gpu, ref, seqs):
    assert gpu.shape == ref.shape
    for i in range(len(ref)):
        g, r = gpu[i], ref[i]
        for f in _native.ALN_FIELDS:
            assert g[f] == r[f], (i, f, g[f], r[f], seqs[i][:60])
        n = r['n_cigar']
        assert np.array_equal(g['cigar'][:n], r['cigar'][:n]), (i, _native.cigar_text(g),
                                                                 _native.cigar_text(r))


def _reads(n_pairs, seed, genomes=None, **kw):
    pairs = synth.make_pairs(n_pairs, genomes=genomes or {'HIV1B-pol-seed': POL},
                             genome_seed=seed, read_seed=seed + 1000, **kw)
    return synth.interleave(pairs)


@pytest.mark.parametrize('mode', [oracle.E2E, oracle.LOCAL])
def test_map_pol_vs_oracle(ctx, mode):
    names, seqs, quals = _reads(1500, 7, indel_rate=0.01)
    ref = _oracle_alns([POL], mode, seqs, quals, True)
    gpu = _gpu_alns(ctx, ['HIV1B-pol-seed'], [POL], mode, seqs, quals, True)
    _assert_same(gpu, ref, seqs)
    assert (ref["flag"] & 4 == 0).mean() > 0.25  # the test exercises real alignments


def _unseedable(seq, rng, every=12):
    """A copy with a substitution every `every` bases (phase random): no
    exact 20- or 22-mer survives, the read still aligns in the band."""
    out = list(seq)
    for i in range(int(rng.integers(0, every)), len(out), every):
        out[i] = 'ACGT'[('ACGT'.index(out[i]) + 1) % 4] if out[i] in 'ACGT' else out[i]
    return ''.join(out)


@pytest.mark.parametrize('mode', [oracle.E2E, oracle.LOCAL])
def test_mate_rescue_vs_oracle(ctx, mode):
    """Pairs whose second (or first) mate has no exact seed left: only mate
    rescue (og_mapper.c rescue_pair, k_rescue) can align it, in the -X window
    next to its aligned mate.  Includes mates near the reference ends (window
    clipped), a mate that is random sequence (scan runs, DP fails) and pairs
    whose anchor is reverse."""
    rng = np.random.default_rng(21)
    names, seqs, quals = _reads(600, 17, sub_rate=0.02)
    seqs = list(seqs)
    for p in range(len(seqs) // 2):
        k = 2 * p + (p % 2)              # mate 1 of odd pairs, mate 2 of even ones
        if p % 7 == 3:
            seqs[k] = ''.join(rng.choice(list('ACGT'), size=len(seqs[k])))
        elif p % 5 != 4:
            seqs[k] = _unseedable(seqs[k], rng)
    # anchors at both reference ends
    for st in (0, len(POL) - 251):
        a = POL[st:st + 251]
        b = _unseedable(POL[max(0, st - 200):max(0, st - 200) + 251] if st else POL[300:551], rng)
        comp = str.maketrans('ACGT', 'TGCA')
        seqs += [a, b.translate(comp)[::-1]]
        quals += ['G' * 251, 'F' * 251]
        names += ['@end%d 1:N:0:1' % st, '@end%d 2:N:0:1' % st]
    diag = []
    ix = oracle.Index([POL], oracle.seed_len(mode))
    out = oracle.map_reads(ix, oracle.params(mode), seqs, quals, True, diag=diag)
    ref = np.frombuffer(bytes(out), dtype=_native.ALN_DTYPE)[:len(seqs)]
    gpu = _gpu_alns(ctx, ['HIV1B-pol-seed'], [POL], mode, seqs, quals, True)
    _assert_same(gpu, ref, seqs)
    rescued = sum(1 for c, _ in diag if oracle.CAUSES[c] == 'rescued')
    assert rescued > 150, rescued
    stats = ctx.map_stats()
    assert stats[4] >= rescued, stats       # rescue extensions (some fail the DP)


@pytest.mark.parametrize('mode', [oracle.E2E, oracle.LOCAL])
def test_mate_rescue_ties_and_ambiguous_bases(ctx, mode):
    """The rescue window search picks the diagonal with the most matches,
    the leftmost on ties (k_rescue): a reference of tandem repeats (many
    diagonals tie or come within a few matches of the maximum), mates with N
    bases and N bases in the window (the 2-bit path with N masks), mates
    shorter than 64 bases (windows of more than one 1024-diagonal chunk) and
    random mates."""
    rng = np.random.default_rng(44)
    unit = ''.join(rng.choice(list('ACGT'), size=37))
    rep = ''.join(unit if i % 3 else unit[:-1] + 'A' for i in range(60))   # ~2.2 kb of near-repeats
    ref = POL[:1500] + rep + POL[1500:2600].replace('G', 'N', 3)
    comp = str.maketrans('ACGTN', 'TGCAN')
    seqs, quals, names = [], [], []

    def pair(a_st, b_st, lb, tweak):
        a = ref[a_st:a_st + 251]
        b = tweak(_unseedable(ref[b_st:b_st + lb], rng))
        seqs.extend([a, b.translate(comp)[::-1]])
        quals.extend(['I' * 251, ''.join(chr(33 + int(q)) for q in rng.integers(2, 41, size=lb))])
        names.extend(['@p%d 1:N:0:1' % len(names), '@p%d 2:N:0:1' % len(names)])

    for k in range(60):
        st = 1500 + int(rng.integers(0, 1500))
        pair(st, st + int(rng.integers(100, 700)), 251, lambda s: s)               # repeats: near ties
        pair(st, st + int(rng.integers(100, 700)), 251,
             lambda s: s[:40] + 'N' + s[41:120] + 'NN' + s[122:])                 # N in the mate
        pair(st, st + 300, int(rng.integers(20, 64)), lambda s: s)                 # < 64 bases
    for k in range(20):
        st = 2800 + int(rng.integers(0, 700))                                      # N in the window
        pair(st, st + int(rng.integers(100, 500)), 251, lambda s: s)
        pair(st, st + 200, 251, lambda s: ''.join(rng.choice(list('ACGT'), size=len(s))))
    want = _oracle_alns([ref], mode, seqs, quals, True)
    gpu = _gpu_alns(ctx, ['rep'], [ref], mode, seqs, quals, True)
    _assert_same(gpu, want, seqs)
    assert ctx.map_stats()[4] > 100


@pytest.mark.parametrize('mode', [oracle.E2E, oracle.LOCAL])
def test_mate_rescue_long_mates(ctx, mode):
    """Mates of 255-1024 bases rescued next to a 251-base anchor (the -X 1200
    window still holds them): the bit-plane count's read words run to 32 per
    diagonal with every tail length around the 32-base word edges, the
    window's staged words to 65; either mate order, N bases in some mates."""
    rng = np.random.default_rng(77)
    ref = POL + SEEDS['HIV1B-env-seed'][:1500]
    comp = str.maketrans('ACGTN', 'TGCAN')
    seqs, quals = [], []
    lens = [255, 256, 257, 288, 300, 383, 480, 511, 512, 513, 600, 700, 767, 800, 900, 1000, 1023, 1024]
    for k in range(90):
        lb = lens[k % len(lens)]
        st = int(rng.integers(0, len(ref) - 1200))
        off = int(rng.integers(0, 1200 - lb + 1))
        a = ref[st:st + 251]
        b = _unseedable(ref[st + off:st + off + lb], rng, every=int(rng.integers(9, 14)))
        if k % 4 == 1:
            b = b[:100] + 'N' + b[101:]
        b = b.translate(comp)[::-1]
        qa = 'I' * 251
        qb = ''.join(chr(33 + int(q)) for q in rng.integers(2, 41, size=lb))
        if k % 2:
            seqs += [b, a]
            quals += [qb, qa]
        else:
            seqs += [a, b]
            quals += [qa, qb]
    want = _oracle_alns([ref], mode, seqs, quals, True)
    gpu = _gpu_alns(ctx, ['polenv'], [ref], mode, seqs, quals, True)
    _assert_same(gpu, want, seqs)
    assert ctx.map_stats()[4] >= 60


def test_map_all_seeds_e2e_vs_oracle(ctx):
    """prelim_map's pass: every seed of projects.json, reads from 3 HIV genes."""
    genomes = {k: SEEDS[k] for k in ('HIV1B-pol-seed', 'HIV1B-env-seed', 'HIV1B-gag-seed')}
    names, seqs, quals = _reads(1500, 11, genomes=genomes)
    refnames = list(SEEDS)
    refseqs = [SEEDS[k] for k in refnames]
    ref = _oracle_alns(refseqs, oracle.E2E, seqs, quals, True)
    gpu = _gpu_alns(ctx, refnames, refseqs, oracle.E2E, seqs, quals, True)
    _assert_same(gpu, ref, seqs)


def test_map_unpaired_long_and_edge_reads(ctx):
    """Unpaired 1x300, reads with Ns, short, empty and overhanging reads."""
    rng = np.random.default_rng(5)
    names, seqs, quals = _reads(400, 13, read_len=300, paired=False)
    seqs = list(seqs)
    quals = list(quals)
    extra = ['', 'ACGT', POL[:30], POL[-120:] + 'ACGTACGTAC' * 10, 'N' * 60 + POL[500:700],
             POL[1000:1250].replace('A', 'N', 30), POL[2000:2251].lower(), 'ACGTRYKM' + POL[10:200]]
    for s in extra:
        seqs.append(s)
        quals.append(''.join(chr(33 + int(q)) for q in rng.integers(2, 41, size=len(s))))
    for mode in (oracle.E2E, oracle.LOCAL):
        ref = _oracle_alns([POL, SEEDS['HIV1B-gag-seed']], mode, seqs, quals, False)
        gpu = _gpu_alns(ctx, ['pol', 'gag'], [POL, SEEDS['HIV1B-gag-seed']], mode, seqs, quals,
                        False)
        _assert_same(gpu, ref, seqs)


def _sam_lines(alns, names, seqs, quals, refnames, paired):
    lines = ['@HD\tVN:1.0\tSO:unsorted\n'] + ['@SQ\tSN:{}\tLN:0\n'.format(r) for r in refnames]
    for i in range(len(seqs)):
        a = oracle.OgAln.from_buffer_copy(alns[i].tobytes())
        lines.append('\t'.join(oracle.sam_fields(a, oracle.qname_of(names[i], paired), seqs[i],
                                                 quals[i], refnames)) + '\n')
    return lines


def test_format_rows_matches_oracle_text(ctx):
    names, seqs, quals = _reads(300, 17, indel_rate=0.01)
    ctx.index_build(['HIV1B-pol-seed'], [POL], 20)
    ctx.reads_load(seqs, quals, True, names=[oracle.qname_of(n, True) for n in names])
    ctx.map(_native.params(oracle.LOCAL))
    gpu_text = ctx.format_rows(0)
    ref = _oracle_alns([POL], oracle.LOCAL, seqs, quals, True)
    want = ''.join(_sam_lines(ref, names, seqs, quals, ['HIV1B-pol-seed'], True)[2:])
    assert gpu_text == want


def _gpu_pileup_as_refmap(ctx, refnames, reflens, q_cutoff, source=0):
    ctx.pileup(source, q_cutoff, reflens)
    p = ctx.pileup_fetch()
    events = {}
    for r, pos, tok, count in p['events']:
        events.setdefault((r, pos), Counter())[tok] += count
    refmap, counts = {}, Counter()
    order = sorted((p['first_unit'][r], r) for r in range(len(refnames)) if p['first_unit'][r] >= 0)
    for _, r in order:
        counts[refnames[r]] = int(p['read_counts'][r])
        pos_nucs = {}
        for pos in range(1, int(p['max_pos'][r]) + 1):
            c = Counter()
            for k, tok in enumerate('ACGT'):
                if p['dense'][r, pos - 1, k]:
                    c[tok] = int(p['dense'][r, pos - 1, k])
            if p['nflag'][r, pos - 1]:
                c['N'] = -1
            if p['dflag'][r, pos - 1]:
                c['-'] = -2
            c.update(events.get((r, pos), {}))
            if c:
                pos_nucs[pos] = c
        refmap[refnames[r]] = (pos_nucs, int(p['max_pos'][r]))
    return refmap, counts


def test_pileup_only_selected_references(ctx):
    """mh_pileup_only: pairs over three references (pol, env, gag, with
    insertions), piled up in full and with only pol and gag counted: the
    counted references' counters, flags, scalars and insertion tokens are
    the full pileup's, env's stay empty."""
    env, gag = SEEDS['HIV1B-env-seed'], SEEDS['HIV1B-gag-seed']
    names, seqs, quals = _reads(1500, 29, genomes={'HIV1B-pol-seed': POL, 'HIV1B-env-seed': env,
                                                   'HIV1B-gag-seed': gag}, indel_rate=0.01)
    refs = ['HIV1B-pol-seed', 'HIV1B-env-seed', 'HIV1B-gag-seed']
    ctx.index_build(refs, [POL, env, gag], 20)
    ctx.reads_load(seqs, quals, True)
    ctx.map(_native.params(oracle.LOCAL))
    lens = [len(POL), len(env), len(gag)]
    ctx.pileup(0, 20, lens)
    full = ctx.pileup_fetch()
    ctx.pileup(0, 20, lens, only=[0, 2])
    part = ctx.pileup_fetch()
    assert full['read_counts'][1] > 0
    for r in (0, 2):
        for k in ('dense', 'nflag', 'dflag'):
            assert np.array_equal(part[k][r], full[k][r]), (r, k)
        for k in ('read_counts', 'first_unit', 'max_pos'):
            assert part[k][r] == full[k][r], (r, k)
    assert part['read_counts'][1] == 0 and part['first_unit'][1] < 0 and part['max_pos'][1] == 0
    assert not part['dense'][1].any() and not part['nflag'][1].any() and not part['dflag'][1].any()
    assert sorted(e for e in part['events'] if e[0] != 1) == sorted(e for e in full['events'] if e[0] != 1)
    assert not [e for e in part['events'] if e[0] == 1]


@pytest.mark.parametrize('mode,q', [(oracle.LOCAL, 20), (oracle.E2E, 20), (oracle.LOCAL, 0)])
def test_pileup_vs_oracle(ctx, mode, q):
    names, seqs, quals = _reads(2000, 23, indel_rate=0.01)
    refnames = ['HIV1B-pol-seed', 'HIV1B-gag-seed']
    refseqs = [POL, SEEDS['HIV1B-gag-seed']]
    gpu = _gpu_alns(ctx, refnames, refseqs, mode, seqs, quals, True)
    lines = _sam_lines(gpu, names, seqs, quals, refnames, True)
    want_refmap, want_counts = oracle.pileup(*oracle.matchmaker(lines), q)
    got_refmap, got_counts = _gpu_pileup_as_refmap(ctx, refnames, [len(s) for s in refseqs], q)
    assert list(got_refmap) == list(want_refmap)
    assert got_counts == want_counts
    for name in want_refmap:
        assert got_refmap[name] == want_refmap[name], name


def test_pileup_rows_vs_golden_sams(ctx, golden_dir):
    """Source 1 (rows read back from text) on every golden SAM case."""
    with open(os.path.join(golden_dir, 'pileup_golden.json')) as f:
        cases = json.load(f)['cases']
    for c in cases:
        _rows_case_vs_oracle(ctx, c['sam'], c['quality_cutoff'])


def _random_cigar_sam(rng, n_pairs, ref_len=240):
    """SAM text whose CIGARs start with deletions, insertions or soft clips
    (k_pileup's merge-start shortcut does not apply to a padded read that
    starts with '-'), with inner indels; bases and qualities random."""
    lines = ['@HD\tVN:1.0\tSO:unsorted\n', '@SQ\tSN:r1\tLN:{}\n'.format(ref_len)]
    quals = 'FFFFF5#(:?'

    def cigar(m):
        ops, left = [], m
        lead = rng.integers(0, 4)
        if lead == 1:
            ops.append('{}D'.format(int(rng.integers(1, 4))))
        elif lead == 2:
            k = int(rng.integers(1, 4)); ops.append('{}I'.format(k)); left -= k
        elif lead == 3:
            k = int(rng.integers(1, 6)); ops.append('{}S'.format(k)); left -= k
        while left > 0:
            k = int(min(left, rng.integers(4, 20)))
            ops.append('{}M'.format(k)); left -= k
            if left > 6 and rng.random() < 0.3:
                if rng.random() < 0.5:
                    ops.append('{}D'.format(int(rng.integers(1, 4))))
                else:
                    k = int(rng.integers(1, 4)); ops.append('{}I'.format(k)); left -= k
        return ''.join(ops)

    for p in range(n_pairs):
        for mate, flag in ((1, 99), (2, 147)):
            m = int(rng.integers(20, 60))
            seq = ''.join(rng.choice(list('ACGTN'), p=[0.24, 0.24, 0.24, 0.24, 0.04], size=m))
            qual = ''.join(rng.choice(list(quals), size=m))
            pos = int(rng.integers(1, ref_len - 80))
            lines.append('\t'.join(['q{}'.format(p), str(flag), 'r1', str(pos), '44', cigar(m), '=',
                                    '1', '0', seq, qual]) + '\n')
    return ''.join(lines)


@pytest.mark.parametrize('q', [0, 20])
def test_pileup_rows_leading_gaps_vs_oracle(ctx, q):
    """Rows whose CIGARs start with D / I / S (the merge start found by the
    scan, not from the pads) against the oracle pileup."""
    rng = np.random.default_rng(41 + q)
    _rows_case_vs_oracle(ctx, _random_cigar_sam(rng, 300), q)


def _rows_case_vs_oracle(ctx, sam, quality_cutoff):
    """One SAM text through source 1 (rows) against the oracle pileup."""
    ref_names, pairs = oracle.matchmaker(sam.splitlines(True))
    want_refmap, want_counts = oracle.pileup(ref_names, pairs, quality_cutoff)
    rows, units = [], []
    for r1, r2 in pairs:
        ids = []
        for r in (r1, r2):
            if r is None:
                ids.append(-1)
            else:
                ids.append(len(rows))
                rows.append(r)
        units += ids
    flag = [int(r[1]) for r in rows]
    ref = [ref_names.index(r[2]) for r in rows]
    pos = [int(r[3]) for r in rows]
    cig, cig_off, n_cig = [], [], []
    for r, f in zip(rows, flag):
        ops = oracle.parse_cigar(r[5]) if not (f & 4) else []
        cig_off.append(len(cig))
        n_cig.append(len(ops))
        cig += ops
    seq = ''.join(r[9] for r in rows).encode()
    qual = ''.join(r[10][:len(r[9])].ljust(len(r[9]), 'J') for r in rows).encode()
    lens = [len(r[9]) for r in rows]
    offs = np.concatenate([[0], np.cumsum(lens)[:-1]]) if rows else []
    ctx.rows_load(flag, ref, pos, cig_off, n_cig, cig or [0], np.frombuffer(seq, np.uint8),
                  np.frombuffer(qual, np.uint8), offs, lens, units)
    # reference span of a row <= read length + its deletions
    dels = [sum(int(n) for n, op in re.findall(r'(\d+)([MIDNS])', r[5]) if op == 'D') for r in rows]
    span = {id(r): len(r[9]) + d for r, d in zip(rows, dels)}
    cap_lens = [max([int(r[3]) + span[id(r)] for p in pairs for r in p if r] + [8])
                for _ in ref_names]
    got_refmap, got_counts = _gpu_pileup_as_refmap(ctx, ref_names, cap_lens, quality_cutoff,
                                                   source=1)
    assert list(got_refmap) == list(want_refmap)
    assert got_counts == want_counts
    for name in want_refmap:
        assert got_refmap[name][0] == want_refmap[name][0], (name, sam[:200])


def test_gotoh_vs_golden(ctx, golden_dir):
    with open(os.path.join(golden_dir, 'gotoh_golden.json')) as f:
        cases = json.load(f)['cases']
    for c in cases:
        args = (c['seq1'], c['seq2'], c['gop'], c['gep'], c['is_global'], c['alphabet'], c['matrix'])
        want = oracle.gotoh_align(*args) if not c['error'] else None
        if c['error']:
            with pytest.raises(RuntimeError):
                ctx.gotoh_align(*args)
            continue
        assert ctx.gotoh_align(*args) == want, c


def test_gotoh_batch_vs_golden(ctx, golden_dir):
    """Every golden case with the same scoring in one mh_gotoh_align_batch
    launch (one workgroup each): the same strings, scores and traceback
    failures as the oracle (pinned on these cases, test_oracle_gotoh.py)."""
    with open(os.path.join(golden_dir, 'gotoh_golden.json')) as f:
        cases = json.load(f)['cases']
    groups = {}
    for c in cases:
        key = (c['gop'], c['gep'], c['is_global'], c['alphabet'], tuple(c['matrix']))
        groups.setdefault(key, []).append(c)
    assert max(len(g) for g in groups.values()) > 20
    for (gop, gep, is_global, alphabet, matrix), group in groups.items():
        got = ctx.gotoh_align_many([(c['seq1'], c['seq2']) for c in group], gop, gep, is_global,
                                   alphabet, list(matrix))
        for c, g in zip(group, got):
            if c['error']:
                assert isinstance(g, RuntimeError), c
            else:
                assert g == oracle.gotoh_align(c['seq1'], c['seq2'], gop, gep, is_global, alphabet,
                                               list(matrix)), c


def test_gotoh_pol_sized(ctx):
    """A 3,039 x ~2,900 global alignment (the remap filter's size) vs oracle."""
    rng = np.random.default_rng(3)
    conseq = synth.sample_genome(POL, rng, 0.1, 0.004).tobytes().decode()[100:3000]
    mat, alpha = [5, -4, -4, -4, 0, -4, 5, -4, -4, 0, -4, -4, 5, -4, 0, -4, -4, -4, 5, 0,
                  0, 0, 0, 0, 0], 'ACGT?'
    want = oracle.gotoh_align(POL, conseq, 15, 3, True, alpha, mat)
    assert ctx.gotoh_align(POL, conseq, 15, 3, True, alpha, mat) == want


@pytest.mark.parametrize('is_global', [True, False])
def test_gotoh_profile_in_global_memory(ctx, is_global):
    """A batch whose longest seq2 makes the score profile too large for LDS
    (5 x 14k bytes > 64 KiB: k_gotoh_fwd<false> streams each lane's profile
    bytes from global memory, realigned per block of 32 columns) holding
    pairs of every block kind -- long rows, rows shorter than one block,
    seq1 shorter than a strip -- all equal to the oracle."""
    rng = np.random.default_rng(23)
    mat, alpha = [5, -4, -4, -4, 0, -4, 5, -4, -4, 0, -4, -4, 5, -4, 0, -4, -4, -4, 5, 0,
                  0, 0, 0, 0, 0], 'ACGT?'
    rand = lambda k: ''.join(rng.choice(list('ACGT'), size=k))
    long2 = ''.join(synth.sample_genome(POL, rng, 0.05, 0.01).tobytes().decode() for _ in range(5))[:14000]
    pairs = [(long2[2000:2700], long2),                          # 700 x 14,000
             (POL[:130], long2[:90]),                            # n < one block past the skew
             (rand(40), long2[5000:5450]),                       # m < one strip
             (long2[9000:9300] + rand(20), long2[8900:13950])]
    got = ctx.gotoh_align_many(pairs, 15, 3, is_global, alpha, mat)
    for (a, b), g in zip(pairs, got):
        assert g == oracle.gotoh_align(a, b, 15, 3, is_global, alpha, mat)


@pytest.mark.parametrize('is_global', [True, False])
def test_gotoh_traceback_runs(ctx, is_global):
    """k_gotoh_tb walks by runs of one move (a ballot over the next 64
    cells of each move): paths with long diagonal runs, insertions and
    deletions of 1-300 bases (runs longer than the wave and than the
    128 x 128 window), gaps right at the ends, alternating short gaps, and
    ties (repeats) -- every aligned pair equal to the oracle's, global and
    local."""
    rng = np.random.default_rng(41)
    mat, alpha = [5, -4, -4, -4, 0, -4, 5, -4, -4, 0, -4, -4, 5, -4, 0, -4, -4, -4, 5, 0,
                  0, 0, 0, 0, 0], 'ACGT?'
    rand = lambda k: ''.join(rng.choice(list('ACGT'), size=k))
    base = POL[:2400]
    pairs = [
        (base, base[:700] + base[770:]),                     # a 70-base deletion
        (base, base[:500] + rand(130) + base[500:]),         # a 130-base insertion
        (base, base[:900] + base[1200:]),                    # 300 bases: past the window
        (base, rand(200) + base + rand(150)),                # end gaps, both sides
        (base[300:] , base),                                 # seq1 starts inside seq2
        (base, ''.join(base[i:i + 40] + ('' if i % 80 else rand(2)) for i in range(0, 2400, 40))),
        (('ACGTTGCA' * 150)[:1100], ('ACGTTGCA' * 160)[3:1203]),   # repeats: ties
        (base[:64], base[:64]), (base[:65], base[1:64]),     # one run of exactly the wave
    ]
    got = ctx.gotoh_align_many(pairs, 15, 3, is_global, alpha, mat)
    for (a, b), g in zip(pairs, got):
        assert g == oracle.gotoh_align(a, b, 15, 3, is_global, alpha, mat), (len(a), len(b))


def _filter_distance_oracle(seq1, seq2, text, alpha, mat):
    from micall_amd.consensus import extract_relevant_seed
    a_seed, a_conseq, _ = oracle.gotoh_align(seq1, seq2, 15, 3, True, alpha, mat)
    return oracle.levenshtein(extract_relevant_seed(a_conseq, a_seed), text)


def test_gotoh_distance_batch(ctx):
    """mh_gotoh_distance_batch (the filter's alignment, relevant seed and
    edit distance on the device, remap.py:249-251) against the oracle's
    Gotoh + extract_relevant_seed + Levenshtein: patterns of one block, of
    exactly 64 blocks (one strip), one row into a second strip and three
    strips (the strips hand their bottom deltas on through global memory),
    texts shorter than a block of columns, with characters outside the
    alphabet, empty, and the filter's own shape (a seed against a mutated
    part of itself and against an unrelated seed)."""
    rng = np.random.default_rng(31)
    mat, alpha = [5, -4, -4, -4, 0, -4, 5, -4, -4, 0, -4, -4, 5, -4, 0, -4, -4, -4, 5, 0,
                  0, 0, 0, 0, 0], 'ACGT?'
    rand = lambda k: ''.join(rng.choice(list('ACGT'), size=k))
    mut = lambda x, r: synth.sample_genome(x, rng, r, r / 10).tobytes().decode()
    long1 = ''.join(mut(POL, 0.05) for _ in range(4))[:9000]
    triples = [
        (POL, mut(POL, 0.1)[200:2900], None),              # the filter's shape
        (POL, mut(SEEDS['HIV1B-env-seed'], 0.05)[:1500], None),
        (rand(30), rand(25), None),                         # one block
        (long1[:4096], mut(long1[:4096], 0.05), None),      # exactly one strip
        (long1[:4097], mut(long1[:4097], 0.05), None),      # one row into strip 2
        (long1, mut(long1, 0.08)[100:8700], None),          # three strips
        (long1[3000:3900], mut(long1[3000:3900], 0.1)[:20], None),   # text < 32 columns
        (POL[:700].replace('A', '?', 9), POL[100:600], 'xx' + POL[100:600].lower()[:50] + '-N?'),
        (POL[:500], POL[50:400], ''),                        # empty text
    ]
    jobs = [(a, b, b if t is None else t) for a, b, t in triples]
    got = ctx.gotoh_distance_many(jobs, 15, 3, True, alpha, mat)
    for (a, b, t), g in zip(jobs, got):
        assert g == _filter_distance_oracle(a, b, t, alpha, mat), (len(a), len(b), len(t))


def test_gotoh_distance_batch_no_nongap_column(ctx):
    """An aligned seq2 that is all gap characters ('-' in the alphabet) has
    no relevant span: AttributeError, as the reference's re.match gives
    None; the other pairs of the batch are unaffected."""
    mat = [5, -4, -4, -4, 0, -4, 5, -4, -4, 0, -4, -4, 5, -4, 0, -4, -4, -4, 5, 0,
           0, 0, 0, 0, 0]
    got = ctx.gotoh_distance_many([(POL[:80], '---', 'ACG'), (POL[:80], POL[10:60], POL[10:60])],
                                  15, 3, True, 'ACGT-', mat)
    assert isinstance(got[0], AttributeError)
    assert got[1] == _filter_distance_oracle(POL[:80], POL[10:60], POL[10:60], 'ACGT-', mat)


def test_gotoh_planes_need_no_zeroing(ctx, golden_dir, monkeypatch):
    """The tie planes are not zeroed between batches (k_gotoh_fwd writes
    every cell of the grid before anything reads it): with them poisoned
    first (MH_GOTOH_POISON_PLANES=1) the golden batch, the long-profile
    batches and the distance batch still equal the oracle."""
    monkeypatch.setenv('MH_GOTOH_POISON_PLANES', '1')
    test_gotoh_batch_vs_golden(ctx, golden_dir)
    test_gotoh_profile_in_global_memory(ctx, True)
    test_gotoh_profile_in_global_memory(ctx, False)
    test_gotoh_distance_batch(ctx)


@pytest.mark.parametrize('is_global', [True, False])
def test_gotoh_long_seq1_global_memory_variant(ctx, is_global):
    """seq1 too long for the rolling diagonals in LDS (k_gotoh<false>: they
    stay in global memory), in a batch with a short pair, and a batch of
    LDS-sized pairs of ragged shapes: both variants equal the oracle."""
    rng = np.random.default_rng(17)
    mat, alpha = [5, -4, -4, -4, 0, -4, 5, -4, -4, 0, -4, -4, 5, -4, 0, -4, -4, -4, 5, 0,
                  0, 0, 0, 0, 0], 'ACGT?'
    rand = lambda k: ''.join(rng.choice(list('ACGT'), size=k))
    long1 = POL + rand(2500)                                   # 5,539 nt
    part = synth.sample_genome(POL, rng, 0.08, 0.01).tobytes().decode()[400:900]
    pairs = [(long1, part), (part[:37], long1[1000:1011])]
    got = ctx.gotoh_align_many(pairs, 15, 3, is_global, alpha, mat)
    for (a, b), g in zip(pairs, got):
        assert g == oracle.gotoh_align(a, b, 15, 3, is_global, alpha, mat)
    ragged = [(rand(int(rng.integers(1, 900))), rand(int(rng.integers(1, 900)))) for _ in range(12)]
    ragged.append((POL[:50], POL[:50]))
    got = ctx.gotoh_align_many(ragged, 10, 2, is_global, alpha, mat)
    for (a, b), g in zip(ragged, got):
        want = None
        try:
            want = oracle.gotoh_align(a, b, 10, 2, is_global, alpha, mat)
        except RuntimeError:
            assert isinstance(g, RuntimeError)
            continue
        assert g == want


@pytest.mark.parametrize('mode', [oracle.E2E, oracle.LOCAL])
def test_map_overhang_trimming(ctx, mode):
    """Reads from a genome that extends past both ends of the reference:
    overhanging columns become soft clips (trimming on the CIGAR runs)."""
    rng = np.random.default_rng(29)
    flank = lambda n: ''.join(rng.choice(list('ACGT'), size=n))
    genome = flank(200) + POL[:600] + flank(150)
    names, seqs, quals = _reads(600, 31, genomes={'g': genome}, indel_rate=0.02, sub_rate=0.03)
    ref = _oracle_alns([POL[:600]], mode, seqs, quals, True)
    gpu = _gpu_alns(ctx, ['p'], [POL[:600]], mode, seqs, quals, True)
    _assert_same(gpu, ref, seqs)
    clipped = sum(1 for a in ref if a['n_cigar'] and (a['cigar'][0] & 15) == 4)
    assert clipped > 20


@pytest.mark.parametrize('mode,rdg,rfg', [(oracle.E2E, (10, 3), (10, 3)), (oracle.LOCAL, (10, 3), (10, 3)),
                                          (oracle.E2E, (4, 3), (14, 2)), (oracle.LOCAL, (20, 5), (6, 1))])
def test_map_ragged_pairs_band_widths(ctx, mode, rdg, rfg):
    """Pairs whose mates have different lengths (30-300 nt, so the two
    extensions sharing a k_dp wave end on different rows and short reads get
    a band narrower than bowtie2's maxhalf of 15), 2 % indels, and gap
    penalties other than MiCall's (the band half-width follows them)."""
    rng = np.random.default_rng(31)
    names, seqs, quals = _reads(700, 23, read_len=300, sub_rate=0.03, indel_rate=0.02)
    seqs, quals = list(seqs), list(quals)
    for i in range(len(seqs)):
        L = int(rng.integers(30, 301))
        if rng.random() < 0.5:
            seqs[i], quals[i] = seqs[i][:L], quals[i][:L]
        else:
            seqs[i], quals[i] = seqs[i][-L:], quals[i][-L:]
    ix = oracle.Index([POL], oracle.seed_len(mode))
    out = oracle.map_reads(ix, oracle.params(mode, rdg=rdg, rfg=rfg), seqs, quals, True)
    ref = np.frombuffer(bytes(out), dtype=_native.ALN_DTYPE)[:len(seqs)]
    ctx.index_build(['HIV1B-pol-seed'], [POL], oracle.seed_len(mode))
    ctx.reads_load(seqs, quals, True)
    ctx.map(_native.params(mode, rdg=rdg, rfg=rfg))
    gpu = ctx.fetch()
    _assert_same(gpu, ref, seqs)
    assert (ref['flag'] & 4 == 0).mean() > 0.2
    assert (ref['xo'] > 0).sum() > 20      # gapped alignments among them
