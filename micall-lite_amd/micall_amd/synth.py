"""
Synthetic paired FASTQ generator for the BASELINE.json configs (SURVEY.md
8(d)): a sample genome drawn from a seed reference (10% substitutions,
0.2% indels, 70% of them 3 nt), fragments N(450, 100) clipped to
[260, 1200], R1 = the fragment's 5' read_len nt, R2 = reverse complement of
its 3' read_len nt, 0.5% sequencing errors, qualities drawn from the
per-character histogram of the reference's examples/*.fastq.gz, Illumina
style headers.  Deterministic: numpy PCG64 seeded per (seed, block), so a
rank can generate its shard without the others.
"""
import gzip

import numpy as np

DEFAULT_SEED = 20261015

# Per-character quality counts over examples/HIV1C-pol_S1_L001_R{1,2}_001.fastq.gz
QUAL_COUNTS = {
    '#': 105226, '(': 7548, ')': 26646, '*': 64283, '+': 52869, ',': 97903, '-': 4979,
    '.': 4775, '/': 9900, '0': 11277, '1': 11051, '2': 12883, '3': 14495, '4': 13842,
    '5': 21466, '6': 24712, '7': 41528, '8': 40628, '9': 40778, ':': 45702, ';': 18114,
    '<': 52739, '=': 23561, '>': 26934, '?': 23437, '@': 71678, 'A': 34089, 'B': 28524,
    'C': 378055, 'D': 94530, 'E': 182553, 'F': 457518, 'G': 2755777}

_BASES = np.frombuffer(b'ACGT', dtype=np.uint8)
_COMP = np.zeros(256, dtype=np.uint8)
for _a, _b in zip(b'ACGTN', b'TGCAN'):
    _COMP[_a] = _b
_CODE = np.full(256, 4, dtype=np.uint8)
for _i, _c in enumerate(b'ACGT'):
    _CODE[_c] = _i


def _qual_table(size=1 << 16):
    chars = np.frombuffer(''.join(QUAL_COUNTS).encode(), dtype=np.uint8)
    counts = np.array(list(QUAL_COUNTS.values()), dtype=np.float64)
    edges = np.cumsum(counts) / counts.sum()
    u = (np.arange(size) + 0.5) / size
    return chars[np.searchsorted(edges, u)]


_QTABLE = _qual_table()


def sample_genome(seq, rng, sub_rate=0.10, indel_rate=0.002):
    """A sample genome: the seed with substitutions and short indels."""
    src = np.frombuffer(seq.upper().encode(), dtype=np.uint8).copy()
    codes = _CODE[src]
    sub = (rng.random(len(src)) < sub_rate) & (codes < 4)
    shift = rng.integers(1, 4, size=len(src))
    src[sub] = _BASES[(codes[sub] + shift[sub]) % 4]
    out = []
    i = 0
    ev = rng.random(len(src)) < indel_rate
    lens = np.where(rng.random(len(src)) < 0.7, 3, rng.integers(1, 3, size=len(src)))
    is_ins = rng.random(len(src)) < 0.5
    while i < len(src):
        if ev[i]:
            k = int(lens[i])
            if is_ins[i]:
                out.append(src[i:i + 1])
                out.append(_BASES[rng.integers(0, 4, size=k)])
                i += 1
            else:
                i += k
            continue
        j = i + 1
        while j < len(src) and not ev[j]:
            j += 1
        out.append(src[i:j])
        i = j
    return np.concatenate(out) if out else src


def make_pairs(n_pairs, genomes, genome_seed=DEFAULT_SEED, read_seed=None, read_len=251,
               sub_rate=0.10, indel_rate=0.002, err_rate=0.005, block=0, paired=True,
               frag_mean=450, frag_sd=100):
    """n_pairs read pairs from sample genomes derived from `genomes`
    ({name: seed sequence}); reads are drawn from each genome in proportion to
    its length.  Returns dict(r1, q1, r2, q2) of (n, read_len) uint8 arrays
    (r2/q2 None when paired is False) and 'block' for naming."""
    grng = np.random.Generator(np.random.PCG64(genome_seed))
    samples = [sample_genome(s, grng, sub_rate, indel_rate) for s in genomes.values()]
    rrng = np.random.Generator(np.random.PCG64(
        [genome_seed if read_seed is None else read_seed, block]))
    lens = np.array([len(g) for g in samples], dtype=np.float64)
    which = rrng.choice(len(samples), size=n_pairs, p=lens / lens.sum())
    flat = np.concatenate(samples)
    starts = np.concatenate([[0], np.cumsum([len(g) for g in samples])[:-1]])
    frag = np.clip(rrng.normal(frag_mean, frag_sd, size=n_pairs), max(260, read_len + 9), 1200)
    frag = np.minimum(frag.astype(np.int64), lens[which].astype(np.int64))
    frag = np.maximum(frag, read_len)
    off = (rrng.random(n_pairs) * (lens[which] - frag + 1)).astype(np.int64)
    base = starts[which] + off
    cols = np.arange(read_len, dtype=np.int64)
    out = {'block': block, 'n': n_pairs}
    r1 = flat[base[:, None] + cols[None, :]]
    out['r1'] = _add_errors(r1, rrng, err_rate)
    out['q1'] = _QTABLE[rrng.integers(0, len(_QTABLE), size=(n_pairs, read_len))]
    if paired:
        tail = base + frag - read_len
        r2 = _COMP[flat[tail[:, None] + cols[None, ::-1]]]
        out['r2'] = _add_errors(r2, rrng, err_rate)
        out['q2'] = _QTABLE[rrng.integers(0, len(_QTABLE), size=(n_pairs, read_len))]
    else:
        out['r2'] = out['q2'] = None
    return out


def _add_errors(reads, rng, rate):
    mask = rng.random(reads.shape) < rate
    codes = _CODE[reads[mask]]
    shift = rng.integers(1, 4, size=codes.shape)
    reads = reads.copy()
    reads[mask] = np.where(codes < 4, _BASES[(codes + shift) % 4], reads[mask])
    return reads


def read_name(block, i, mate):
    """Illumina-style header (censor_fastq.py needs tile and cycle fields)."""
    tile = 1101 + (i // 1000000) % 20
    return '@M00000:1:000000000-AAAAA:1:{}:{}:{} {}:N:0:1'.format(
        tile, 1000 + block * 37 % 9000, 1000 + i % 1000000, mate)


def interleave(pairs):
    """(names, seqs, quals) lists with mates interleaved, for small cases."""
    names, seqs, quals = [], [], []
    for i in range(pairs['n']):
        for mate, (r, q) in enumerate(((pairs['r1'], pairs['q1']), (pairs['r2'], pairs['q2'])), 1):
            if r is None:
                continue
            names.append(read_name(pairs['block'], i, mate))
            seqs.append(r[i].tobytes().decode())
            quals.append(q[i].tobytes().decode())
    return names, seqs, quals


def write_fastq(pairs, path1, path2=None, gz=None):
    """Write R1 (and R2) FASTQ files; gzip when the name ends in .gz."""
    for mate, path, (r, q) in ((1, path1, (pairs['r1'], pairs['q1'])),
                               (2, path2, (pairs['r2'], pairs['q2']))):
        if path is None or r is None:
            continue
        use_gz = path.endswith('.gz') if gz is None else gz
        opener = gzip.open if use_gz else open
        with opener(path, 'wt') as f:
            for i in range(pairs['n']):
                f.write('{}\n{}\n+\n{}\n'.format(read_name(pairs['block'], i, mate),
                                                 r[i].tobytes().decode(), q[i].tobytes().decode()))
