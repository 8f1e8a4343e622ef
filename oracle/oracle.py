"""
oracle/oracle.py -- TEST INFRASTRUCTURE ONLY.

ctypes front end of the CPU restatement in oracle/*.c plus the small pure
Python parts of the reference algorithm (matchmaker, counts_to_conseqs,
find_top_token, the consensus-distance filter).  Only tests/,
__graft_entry__.smoke() and bench.py's cpu_baseline leg import this module,
and only as the checker: the product (micall-lite_amd/) never does.

Reference provenance of each function is in its docstring.
"""
import ctypes
import os
import re
import subprocess
from collections import Counter, defaultdict

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, '_build', 'liboracle.so')

E2E, LOCAL = 0, 1
OP_M, OP_I, OP_D, OP_S = 0, 1, 2, 4
OP_CHARS = {OP_M: 'M', OP_I: 'I', OP_D: 'D', OP_S: 'S'}
CHAR_OPS = {'M': OP_M, 'I': OP_I, 'D': OP_D, 'S': OP_S}
YT_NAMES = ['CP', 'DP', 'UP', 'UU']
YF_NAMES = [None, 'NS', 'LN']
MAXOPS = 128
INT32_MIN = -2 ** 31

_lib = None


def build():
    """Compile oracle/_build/liboracle.so with the committed Makefile."""
    subprocess.run(['make', '-s', '-C', HERE], check=True)


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        _lib = ctypes.CDLL(LIB_PATH)
        _declare(_lib)
    return _lib


class OgParams(ctypes.Structure):
    _fields_ = [('mode', ctypes.c_int), ('rdg_open', ctypes.c_int),
                ('rdg_ext', ctypes.c_int), ('rfg_open', ctypes.c_int),
                ('rfg_ext', ctypes.c_int), ('maxins', ctypes.c_int)]


class OgAln(ctypes.Structure):
    _fields_ = [(name, ctypes.c_int32) for name in (
        'ref', 'pos', 'rev', 'score', 'secbest', 'flag', 'mapq', 'rnext', 'pnext',
        'tlen', 'sam_ref', 'sam_pos', 'xm', 'xo', 'xg', 'nm', 'ys', 'yt', 'yf',
        'n_cigar')] + [('cigar', ctypes.c_uint32 * MAXOPS)]


class OgRow(ctypes.Structure):
    _fields_ = [('flag', ctypes.c_int32), ('ref', ctypes.c_int32), ('pos', ctypes.c_int32),
                ('n_cigar', ctypes.c_int32), ('cigar', ctypes.POINTER(ctypes.c_uint32)),
                ('len', ctypes.c_int32), ('seq', ctypes.c_char_p), ('qual', ctypes.c_char_p)]


class OgEvent(ctypes.Structure):
    _fields_ = [('ref', ctypes.c_int32), ('pos', ctypes.c_int32),
                ('tok_off', ctypes.c_int32), ('tok_len', ctypes.c_int32)]


def _declare(L):
    L.og_gotoh_align.argtypes = [ctypes.c_char_p, ctypes.c_char_p, ctypes.c_int, ctypes.c_int,
                                 ctypes.c_int, ctypes.c_char_p, ctypes.POINTER(ctypes.c_int),
                                 ctypes.c_char_p, ctypes.c_char_p, ctypes.c_int,
                                 ctypes.POINTER(ctypes.c_int)]
    L.og_levenshtein.argtypes = [ctypes.c_char_p, ctypes.c_char_p]
    L.og_index_build.restype = ctypes.c_void_p
    L.og_index_build.argtypes = [ctypes.c_int, ctypes.POINTER(ctypes.c_char_p), ctypes.c_int]
    L.og_index_free.argtypes = [ctypes.c_void_p]
    L.og_map.argtypes = [ctypes.c_void_p, ctypes.POINTER(OgParams), ctypes.c_int64, ctypes.c_int,
                         ctypes.c_char_p, ctypes.c_char_p, ctypes.POINTER(ctypes.c_int64),
                         ctypes.POINTER(ctypes.c_int32), ctypes.POINTER(OgAln), ctypes.c_int]
    L.og_map_diag.argtypes = L.og_map.argtypes + [ctypes.POINTER(ctypes.c_int32)]
    L.og_seed_interval.argtypes = [ctypes.c_int, ctypes.c_int]
    L.og_min_score.argtypes = [ctypes.c_int, ctypes.c_int]
    L.og_n_ceil.argtypes = [ctypes.c_int]
    L.og_band_half.argtypes = [ctypes.POINTER(OgParams), ctypes.c_int]
    L.og_mapq.argtypes = [ctypes.c_int] * 5
    L.og_pileup.argtypes = [ctypes.c_int, ctypes.c_int32, ctypes.POINTER(OgRow), ctypes.c_int64,
                            ctypes.POINTER(ctypes.c_int64), ctypes.c_int,
                            ctypes.POINTER(ctypes.c_int32), ctypes.POINTER(ctypes.c_int64),
                            ctypes.POINTER(ctypes.c_int64), ctypes.POINTER(ctypes.c_int32),
                            ctypes.POINTER(OgEvent), ctypes.c_int64,
                            ctypes.POINTER(ctypes.c_int64), ctypes.c_char_p, ctypes.c_int64,
                            ctypes.POINTER(ctypes.c_int64)]


# ---------------------------------------------------------------------------
# Gotoh (micall/alignment/src/_gotoh2.c, micall/alignment/gotoh2.py)
# ---------------------------------------------------------------------------
def gotoh_align(seq1, seq2, gop, gep, is_global, alphabet, matrix):
    """Restatement of _gotoh2.align (_gotoh2.c:544-607): returns
    (aligned1, aligned2, score); raises RuntimeError on traceback failure."""
    cap = len(seq1) + len(seq2) + 1
    o1 = ctypes.create_string_buffer(cap)
    o2 = ctypes.create_string_buffer(cap)
    score = ctypes.c_int()
    mat = (ctypes.c_int * len(matrix))(*matrix)
    st = lib().og_gotoh_align(seq1.encode(), seq2.encode(), gop, gep, int(is_global),
                              alphabet.encode(), mat, o1, o2, cap, ctypes.byref(score))
    if st == -1:
        raise RuntimeError('Traceback failed, try local alignment')
    if st != 0:
        raise ValueError('og_gotoh_align status {}'.format(st))
    return o1.value.decode(), o2.value.decode(), score.value


def levenshtein(a, b):
    """Unit-cost edit distance (Levenshtein.distance at remap.py:251)."""
    return lib().og_levenshtein(a.encode(), b.encode())


def read_matrix_csv(path):
    """gotoh2.Aligner.read_matrix_from_csv (gotoh2.py:45-62)."""
    with open(path) as handle:
        alphabet = ''.join(next(handle).strip('\n').split(','))
        rows = []
        for line in handle:
            rows.extend(int(x) for x in line.strip('\n').split(','))
    return rows, alphabet


def clean_sequence(seq, alphabet):
    """gotoh2.Aligner.clean_sequence (gotoh2.py:70-72)."""
    return re.sub('[^%s]' % (alphabet,), '?', seq.upper())


# ---------------------------------------------------------------------------
# mapper (bowtie2 stand-in; parity with bowtie2 itself is unpinned)
# ---------------------------------------------------------------------------
class Index:
    def __init__(self, seqs, seedlen):
        arr = (ctypes.c_char_p * len(seqs))(*[s.encode() for s in seqs])
        self.handle = lib().og_index_build(len(seqs), arr, seedlen)
        self.n_refs = len(seqs)

    def __del__(self):
        if getattr(self, 'handle', None):
            lib().og_index_free(self.handle)
            self.handle = None


def seed_len(mode):
    return 20 if mode == LOCAL else 22


def params(mode, rdg=(10, 3), rfg=(10, 3), maxins=1200):
    return OgParams(mode, rdg[0], rdg[1], rfg[0], rfg[1], maxins)


def band_half(par, length):
    """Half-width of the DP band around the seeded diagonal (og_band_half)."""
    return lib().og_band_half(ctypes.byref(par), length)


CAUSES = ['aligned', 'rescued', 'filtered (N / empty)', 'no candidate', 'below --score-min',
          'over --n-ceil', 'other']


def map_reads(index, par, seqs, quals, paired, nthreads=0, diag=None):
    """Map reads (paired: mates interleaved).  Returns a ctypes OgAln array.
    diag: optional list that receives (cause index into CAUSES, seed-hit
    clusters) per read."""
    n = len(seqs)
    offs = (ctypes.c_int64 * max(n, 1))()
    lens = (ctypes.c_int32 * max(n, 1))()
    pos = 0
    for i, s in enumerate(seqs):
        offs[i] = pos
        lens[i] = len(s)
        pos += len(s)
    sbuf = ''.join(seqs).encode()
    qbuf = ''.join(quals).encode()
    out = (OgAln * max(n, 1))()
    if diag is None:
        st = lib().og_map(index.handle, ctypes.byref(par), n, int(paired), sbuf, qbuf, offs, lens,
                          out, nthreads)
    else:
        d = (ctypes.c_int32 * max(2 * n, 1))()
        st = lib().og_map_diag(index.handle, ctypes.byref(par), n, int(paired), sbuf, qbuf, offs,
                               lens, out, nthreads, d)
        diag[:] = [(d[2 * i], d[2 * i + 1]) for i in range(n)]
    if st != 0:
        raise ValueError('og_map status {}'.format(st))
    return out


def cigar_string(aln):
    if aln.ref < 0:
        return '*'
    return ''.join('{}{}'.format(c >> 4, OP_CHARS[c & 15]) for c in aln.cigar[:aln.n_cigar])


_COMP = str.maketrans('ACGTN', 'TGCAN')


_DECODE = {i: 'N' for i in range(256)}
_DECODE.update({ord(c): c.upper() for c in 'ACGTacgt'})


def decode_seq(seq):
    """bowtie2 prints reads as upper-case ACGT with every other letter N."""
    return seq.translate(_DECODE)


def sam_fields(aln, qname, seq, qual, refnames):
    """SAM record text for one mate, in the bowtie2 layout the reference
    consumes (remap.py:740-755, prelim_map.py:137-140)."""
    s = decode_seq(seq)
    q = qual
    if aln.ref >= 0 and aln.rev:
        s = s.translate(_COMP)[::-1]
        q = q[::-1]
    rname = refnames[aln.sam_ref] if aln.sam_ref >= 0 else '*'
    if aln.rnext == -2:
        rnext = '*'
    elif aln.rnext == -1:
        rnext = '='
    else:
        rnext = refnames[aln.rnext]
    fields = [qname, str(aln.flag), rname, str(aln.sam_pos), str(aln.mapq), cigar_string(aln),
              rnext, str(aln.pnext), str(aln.tlen), s or '*', q or '*']
    tags = []
    if aln.ref >= 0:
        tags.append('AS:i:{}'.format(aln.score))
        if aln.secbest != INT32_MIN:
            tags.append('XS:i:{}'.format(aln.secbest))
        tags += ['XN:i:0', 'XM:i:{}'.format(aln.xm), 'XO:i:{}'.format(aln.xo),
                 'XG:i:{}'.format(aln.xg), 'NM:i:{}'.format(aln.nm)]
        if aln.ys != INT32_MIN:
            tags.append('YS:i:{}'.format(aln.ys))
    else:
        if aln.ys != INT32_MIN:
            tags.append('YS:i:{}'.format(aln.ys))
        if aln.yf:
            tags.append('YF:Z:{}'.format(YF_NAMES[aln.yf]))
    tags.append('YT:Z:{}'.format(YT_NAMES[aln.yt]))
    return fields + tags


def qname_of(header, paired):
    """bowtie2's read name: header up to the first whitespace, with a /1 or
    /2 suffix removed for paired reads."""
    name = header[1:] if header.startswith('@') else header
    name = name.split()[0] if name.split() else ''
    if paired and len(name) > 2 and name[-2] == '/' and name[-1] in '12':
        name = name[:-2]
    return name


def read_fastq(path):
    import gzip
    opener = gzip.open if path.endswith('.gz') else open
    names, seqs, quals = [], [], []
    with opener(path, 'rt') as f:
        while True:
            h = f.readline()
            if not h:
                break
            s = f.readline().rstrip('\n')
            f.readline()
            q = f.readline().rstrip('\n')
            names.append(h.rstrip('\n'))
            seqs.append(s)
            quals.append(q)
    return names, seqs, quals


def map_fastq_to_sam(refnames, refseqs, mode, fastq1, fastq2=None, rdg=(10, 3), rfg=(10, 3),
                     maxins=1200, nthreads=0):
    """bowtie2 stand-in: SAM lines (no header) for the reads, in input order."""
    n1, s1, q1 = read_fastq(fastq1)
    paired = fastq2 is not None
    if paired:
        n2, s2, q2 = read_fastq(fastq2)
        names, seqs, quals = [], [], []
        for a in range(len(n1)):
            names += [n1[a], n2[a]]
            seqs += [s1[a], s2[a]]
            quals += [q1[a], q2[a]]
    else:
        names, seqs, quals = n1, s1, q1
    ix = Index(refseqs, seed_len(mode))
    alns = map_reads(ix, params(mode, rdg, rfg, maxins), seqs, quals, paired, nthreads)
    lines = []
    for i in range(len(seqs)):
        lines.append('\t'.join(sam_fields(alns[i], qname_of(names[i], paired), seqs[i], quals[i],
                                          refnames)) + '\n')
    return lines


# ---------------------------------------------------------------------------
# pileup + consensus (remap.py:141-333, sam2aln.py:84-273)
# ---------------------------------------------------------------------------
def parse_cigar(cigar):
    if not re.match(r'^((\d+)([MIDNSHPX=]))*$', cigar):
        raise RuntimeError('Invalid CIGAR string: {!r}.'.format(cigar))
    ops = []
    for n, op in re.findall(r'(\d+)([MIDNSHPX=])', cigar):
        if op not in CHAR_OPS:
            raise RuntimeError('Unsupported CIGAR token: {!r}.'.format(n + op))
        ops.append((int(n) << 4) | CHAR_OPS[op])
    return ops


def matchmaker(sam_lines, include_singles=True):
    """remap.matchmaker (remap.py:853-889) over SAM text lines; yields
    (row, row_or_None) with rows split on tabs, and returns ref names
    in @SQ order via the first yielded item."""
    ref_names = []
    ref_set = set()
    cached = {}
    pairs = []
    for line in sam_lines:
        row = line.strip('\n').split('\t')
        if line.startswith('@'):
            if row[0] == '@SQ':
                for field in row[1:]:
                    k, v = field.split(':', 1)
                    if k == 'SN' and v not in ref_set:
                        ref_set.add(v)
                        ref_names.append(v)
            continue
        if row[2] in ref_set:
            old = cached.pop(row[0], None)
            if old is None:
                cached[row[0]] = row
            else:
                pairs.append((old, row))
    if include_singles:
        for row in cached.values():
            pairs.append((row, None))
    return ref_names, pairs


def pileup(ref_names, pairs, q_cutoff, cap=None):
    """Dense refmap of the merged pairs (og_pileup).  Returns
    (refmap, read_counts) with refmap = {rname: {pos: Counter}} in the
    reference's insertion order (remap.py:186-204)."""
    index = {n: i for i, n in enumerate(ref_names)}
    rows, unit_rows, keep = [], [], []
    for r1, r2 in pairs:
        for r in (r1, r2):
            if r is None:
                unit_rows.append(-1)
                continue
            # merge_reads parses the CIGAR of mapped mates only (remap.py:105-115)
            ops = parse_cigar(r[5]) if not (int(r[1]) & 4) else []
            s, q = r[9].encode(), r[10].encode()
            arr = (ctypes.c_uint32 * max(len(ops), 1))(*ops)
            keep.append((s, q, arr))
            rows.append(OgRow(int(r[1]), index[r[2]], int(r[3]), len(ops), arr, len(s), s, q))
            unit_rows.append(len(rows) - 1)
    n_refs = len(ref_names)
    if cap is None:
        cap = max([int(r[3]) + len(r[9]) * 2 + 8 for p in pairs for r in p if r] + [8])
    row_arr = (OgRow * max(len(rows), 1))(*rows)
    units = (ctypes.c_int64 * max(len(unit_rows), 1))(*unit_rows)
    dense = (ctypes.c_int32 * (n_refs * cap * 6))()
    read_counts = (ctypes.c_int64 * max(n_refs, 1))()
    first_unit = (ctypes.c_int64 * max(n_refs, 1))(*([-1] * max(n_refs, 1)))
    max_pos = (ctypes.c_int32 * max(n_refs, 1))()
    ev_cap = sum(len(k[1]) for k in keep) + 16
    ev = (OgEvent * ev_cap)()
    pool_cap = sum(2 * len(k[1]) for k in keep) + 16
    pool = ctypes.create_string_buffer(pool_cap)
    n_ev = ctypes.c_int64()
    used = ctypes.c_int64()
    st = lib().og_pileup(n_refs, cap, row_arr, len(pairs), units, q_cutoff, dense, read_counts,
                         first_unit, max_pos, ev, ev_cap, ctypes.byref(n_ev), pool, pool_cap,
                         ctypes.byref(used))
    if st != 0:
        raise RuntimeError('og_pileup status {}'.format(st))
    raw = pool.raw
    events = defaultdict(Counter)
    for e in ev[:n_ev.value]:
        events[(e.ref, e.pos)][raw[e.tok_off:e.tok_off + e.tok_len].decode()] += 1
    order = sorted((first_unit[r], r) for r in range(n_refs) if first_unit[r] >= 0)
    refmap, counts = {}, Counter()
    for _, r in order:
        name = ref_names[r]
        counts[name] = read_counts[r]
        pos_nucs = {}
        for pos in range(1, max_pos[r] + 1):
            base = (r * cap + pos - 1) * 6
            c = Counter()
            for k, tok in enumerate('ACGT'):
                if dense[base + k]:
                    c[tok] = dense[base + k]
            if dense[base + 4]:
                c['N'] = -1
            if dense[base + 5]:
                c['-'] = -2
            c.update(events.get((r, pos), {}))
            if c:
                pos_nucs[pos] = c
        refmap[name] = (pos_nucs, max_pos[r])
    return refmap, counts


def find_top_token(base_counts):
    """remap.find_top_token (remap.py:892-902): highest count, ties to the
    lexicographically smallest token; None for an empty counter."""
    top_count = top_token = None
    for token, count in base_counts.items():
        if top_count is None or count > top_count or (count == top_count and token < top_token):
            top_token, top_count = token, count
    return top_token


def counts_to_conseqs(refmap, seeds=None):
    """remap.counts_to_conseqs (remap.py:309-333) over the dense refmap,
    with the seed prefill of remap.py:195-197 applied (count 0)."""
    conseqs = {}
    full = {}
    for name, (pos_nucs, max_pos) in refmap.items():
        seed = seeds.get(name, '') if seeds else ''
        if not any(n > 0 for c in pos_nucs.values() for n in c.values()):
            full[name] = (pos_nucs, seed)
            continue
        end = max(max_pos, len(seed)) + 1
        conseq, deletion = '', ''
        for pos in range(1, end):
            counts = Counter(pos_nucs.get(pos, {}))
            if pos <= len(seed) and seed[pos - 1] not in counts:
                counts[seed[pos - 1]] = 0
            top = find_top_token(counts)
            if top is None:
                conseq += 'N'
            elif top == '-':
                deletion += '-'
            else:
                if deletion:
                    if len(deletion) % 3 != 0:
                        conseq += deletion
                    deletion = ''
                conseq += top
        conseqs[name] = conseq
        full[name] = (pos_nucs, seed)
    return conseqs, full


def extract_relevant_seed(aligned_conseq, aligned_seed):
    """remap.extract_relevant_seed (remap.py:129-138)."""
    match = re.match('-*([^-](.*[^-])?)', aligned_conseq)
    return aligned_seed[match.start(1):match.end(1)].replace('-', '')


def sam_to_conseqs(sam_lines, quality_cutoff=0, seeds=None, is_filtered=False,
                   filter_coverage=1, distance_report=None, nuc_model=None):
    """Restatement of remap.sam_to_conseqs (remap.py:141-268) on the oracle
    pileup.  nuc_model = (matrix, alphabet) of HYPHY_NUC for the filter."""
    ref_names, pairs = matchmaker(sam_lines)
    refmap, read_counts = pileup(ref_names, pairs, quality_cutoff)
    new_conseqs, full = counts_to_conseqs(refmap, seeds)
    if not (seeds and is_filtered) or len(new_conseqs) < 2:
        return new_conseqs
    matrix, alphabet = nuc_model
    filtered = {}
    for name in sorted(new_conseqs):
        conseq = new_conseqs[name]
        pos_nucs, seed = full[name]
        relevant = ''
        for pos, c in enumerate(conseq, 1):
            counts = Counter(pos_nucs.get(pos, {}))
            if pos <= len(seed) and seed[pos - 1] not in counts:
                counts[seed[pos - 1]] = 0
            if sum(counts.values()) >= filter_coverage:
                relevant += c
        if not relevant:
            continue
        other_seed = other_dist = seed_dist = None
        for seed_name in sorted(new_conseqs):
            a_seed, a_conseq, _ = gotoh_align(clean_sequence(seeds[seed_name], alphabet),
                                              clean_sequence(relevant, alphabet), 15, 3, True,
                                              alphabet, matrix)
            d = levenshtein(extract_relevant_seed(a_conseq, a_seed), relevant)
            if seed_name == name:
                seed_dist = d
            elif other_dist is None or d < other_dist:
                other_seed, other_dist = seed_name, d
        if seed_dist <= other_dist:
            filtered[name] = conseq
        if distance_report is not None:
            distance_report[name] = dict(seed_dist=seed_dist, other_dist=other_dist,
                                         other_seed=other_seed)
    if not filtered:
        best_ref = read_counts.most_common(1)[0][0]
        filtered[best_ref] = new_conseqs[best_ref]
    return filtered
