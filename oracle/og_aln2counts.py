"""
oracle/og_aln2counts.py -- TEST INFRASTRUCTURE ONLY.

Pure-Python restatement of micall/core/aln2counts.py (the stage after
sam2aln), written from the reference's documented
behaviour to check the device path (micall-lite_amd/csrc/mh_a2c.hip and
micall_amd/aln2counts.py) on small inputs.  Pinned against outputs the
reference itself produced (tests/golden/aln2counts_golden.json: every call
micall/tests/aln2counts_test.py makes on SequenceReport / InsertionWriter /
SeedAmino / SeedNucleotide; tests/golden/e2e/*/a2c_*.csv.gz: aln2counts() on
every e2e case's aligned.csv; tests/golden/aln2counts_edge.json), generated
by tests/golden/gen_golden.py a2c.  Only tests/ and bench.py's cpu_baseline
import it.  Gotoh alignments go through oracle.gotoh_align (og_gotoh.c).

    translation          micall/utils/translation.py:40-142
    codon counting       aln2counts.py:115-172, 582-653
    consensus letters    aln2counts.py:618-626, 655-695
    coordinate mapping   aln2counts.py:174-304
    reports              aln2counts.py:377-579
    insertions           aln2counts.py:711-811
    aln2counts()         aln2counts.py:822-898
"""
import csv
import io
import itertools
import json
import os
import re
from collections import Counter

import oracle

AMINOS = 'ACDEFGHIKLMNPQRSTVWY*'
CUTOFFS = [0.01, 0.02, 0.05, 0.1, 0.2, 0.25]
MAX = 'MAX'
GOP, GEP = 40, 10
_REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
_DATA = os.path.join(_REPO, 'micall-lite_amd', 'micall_amd', 'data')

_ORDER = 'TCAG'
_TABLE = 'FFLLSSSSYY**CC*WLLLLPPPPHHQQRRRRIIIMTTTTNNKKSSRRVVVVAAAADDEEGGGG'
_IUPAC = {'W': 'AT', 'R': 'AG', 'K': 'GT', 'Y': 'CT', 'S': 'CG', 'M': 'AC', 'V': 'AGC',
          'H': 'ATC', 'D': 'ATG', 'B': 'TGC', 'N': 'ATGC', '-': 'ATGC'}
_LETTER = {''.join(sorted(v)): k for k, v in _IUPAC.items() if k != '-'}
_EOL = os.linesep


def _plain(codon):
    i, j, k = (_ORDER.index(c) for c in codon)
    return _TABLE[16 * i + 4 * j + k]


def codon_to_amino(codon, ambig='?'):
    """One upper-case codon: '---' -> '-', two or more gaps or '?' ->
    ambig, mixtures resolved when every expansion agrees."""
    if codon.count('-') > 1 or '?' in codon:
        return '-' if codon == '---' else ambig
    options = ['']
    for c in codon:
        options = [o + b for o in options for b in _IUPAC.get(c, c)]
    aminos = {_plain(o) for o in options}
    return aminos.pop() if len(aminos) == 1 else ambig


def translate(seq, offset=0, ambig='?'):
    if isinstance(seq, bytes):
        seq = seq.decode()
    seq = '-' * offset + seq.upper()
    return ''.join(codon_to_amino(seq[i:i + 3], ambig) for i in range(0, len(seq) - 2, 3))


# ---------------------------------------------------------------------------
# counters
# ---------------------------------------------------------------------------
class NucTally(object):
    """SeedNucleotide."""

    def __init__(self):
        self.counts = Counter()

    def count_nucleotides(self, nuc_seq, count):
        if nuc_seq != 'n':
            self.counts[nuc_seq] += count

    def get_report(self):
        return ','.join(str(self.counts[b]) for b in 'ACGT')

    def get_consensus(self, mixture_cutoff):
        cutoff = mixture_cutoff
        if not self.counts:
            return ''
        ranked = self.counts.most_common()
        # from the end, drop '-' and 'N' while more than one entry is left
        i = len(ranked) - 1
        while i >= 0:
            if ranked[i][0] in ('N', '-') and len(ranked) > 1:
                del ranked[i]
            i -= 1
        total = sum(self.counts.values())
        floor = ranked[0][1] if cutoff == MAX else total * cutoff
        chosen = sorted(b for b, c in ranked if c >= floor)
        if not chosen:
            return 'N'
        return chosen[0] if len(chosen) == 1 else _LETTER[''.join(chosen)]


class AminoTally(object):
    """SeedAmino."""

    def __init__(self, consensus_index):
        self.consensus_index = consensus_index
        self.counts = Counter()
        self.nucleotides = [NucTally(), NucTally(), NucTally()]

    def count_aminos(self, codon_seq, count):
        aa = translate(codon_seq.upper())
        if aa in AMINOS:
            self.counts[aa] += count
        for k in range(3):
            self.nucleotides[k].count_nucleotides(codon_seq[k], count)

    def get_report(self):
        return ','.join(str(self.counts[a]) for a in AMINOS)

    def get_consensus(self):
        best = None
        for aa, c in self.counts.items():     # first maximum in insertion order
            if best is None or c > best[1]:
                best = (aa, c)
        return '-' if best is None else best[0]


# ---------------------------------------------------------------------------
# projects and alignment
# ---------------------------------------------------------------------------
class Projects(object):
    """The two lookups aln2counts makes, over either projects-file format."""

    def __init__(self, cfg):
        if 'project_seed_regions' in cfg:
            self.seqs = {k: v['seq'] for k, v in cfg['regions'].items()}
            self.links = [link for links in cfg['project_regions'].values() for link in links]
        else:
            self.seqs = {k: ''.join(v['reference']) for k, v in cfg['regions'].items()}
            self.links = [[r['coordinate_region'], r['seed_region_names']]
                          for p in cfg['projects'].values() for r in p['regions']]

    def getReference(self, name):
        return self.seqs[name].encode()

    def getCoordinateReferences(self, seed):
        out = {}
        for coord, seeds in self.links:
            if coord and seed in seeds:
                out[coord] = self.getReference(coord)
        return out


def default_projects():
    with open(os.path.join(_DATA, 'micall_regions.json')) as f:
        return Projects(json.load(f))


_MODEL = None


def align_coord(seq1, seq2):
    """gotoh2.Aligner(gop=40, gep=10, is_global=False, model='EmpHIV25').align."""
    global _MODEL
    if _MODEL is None:
        with open(os.path.join(_DATA, 'gotoh_models.json')) as f:
            m = json.load(f)['EmpHIV25']
        _MODEL = (m['alphabet'], m['matrix'])
    alpha, matrix = _MODEL
    assert isinstance(seq1, str) and isinstance(seq2, str)
    assert len(seq1) > 0 and len(seq2) > 0
    clean = lambda s: re.sub('[^%s]' % (alpha,), '?', s.upper())  # noqa: E731
    return oracle.gotoh_align(clean(seq1), clean(seq2), GOP, GEP, False, alpha, matrix)


def _walk(a_x, x, a_y, y):
    """{y index: x index} for every alignment column where x advances."""
    out, xi, yi = {}, 0, 0
    for cx, cy in zip(a_x, a_y):
        if xi < len(x) and cx == x[xi]:
            out[yi] = xi
            xi += 1
        if yi < len(y) and cy == y[yi]:
            yi += 1
    return out


# ---------------------------------------------------------------------------
# SequenceReport
# ---------------------------------------------------------------------------
def fmt_cutoff(cut):
    return cut if cut == MAX else '{:0.3f}'.format(cut)


def _writer(f):
    return csv.writer(f, lineterminator=_EOL)


class Report(object):
    """SequenceReport."""

    def __init__(self, insert_writer, projects, cutoffs):
        self.insert_writer = insert_writer
        self.projects = projects
        self.conseq_mixture_cutoffs = [MAX] + list(cutoffs)

    def _pair_align(self, reference, query):
        if isinstance(reference, bytes):
            reference = reference.decode()
        if isinstance(query, bytes):
            query = query.decode()
        return align_coord(reference, query)

    def read(self, rows):
        rows = list(rows)
        self.seed_aminos, self.reports, self.reading_frames = {}, {}, {}
        self.inserts, self.consensus, self.variants = {}, {}, {}
        if rows:
            self.seed, self.qcut = rows[0]['refname'], rows[0]['qcut']
            self.insert_writer.start_group(self.seed, self.qcut)
            frames = {0: [], 1: [], 2: []}
            for row in rows:
                seq, off, n = row['seq'], int(row['offset']), int(row['count'])
                self.insert_writer.add_nuc_read('-' * off + seq, n)
                for f in range(3):
                    padded = '-' * (f + off) + seq
                    padded += '-' * (-len(padded) % 3)
                    for k in range(off // 3, len(padded) // 3):
                        while len(frames[f]) <= k:
                            frames[f].append(AminoTally(len(frames[f])))
                        frames[f][k].count_aminos(padded[3 * k:3 * k + 3], n)
            self.seed_aminos = frames
            self.coordinate_refs = self.projects.getCoordinateReferences(self.seed)
            if not self.coordinate_refs:
                length = len(self.projects.getReference(self.seed))
                while len(frames[0]) * 3 < length:
                    frames[0].append(AminoTally(len(frames[0])))
        else:
            self.coordinate_refs = {}
        for name, ref in self.coordinate_refs.items():
            self._map(name, ref)

    def _map(self, name, ref):
        if isinstance(ref, bytes):
            ref = ref.decode()
        covered = sum(1 for a in self.seed_aminos[0] if a.counts)
        best_score, best = min(covered, len(ref)), None
        for f, tallies in self.seed_aminos.items():
            cons = ''.join(a.get_consensus() for a in tallies)
            if f == 0:
                self.consensus[name] = cons
            score = self._pair_align(ref, cons)[2]
            if score > best_score:
                best_score, best = score, (f, cons)
        mapped = []
        if best is not None:
            f, cons = best
            self.reading_frames[name] = f
            self.consensus[name] = cons
            seed_nucs = self.projects.getReference(self.seed)
            seed_best, seed_score = None, 0
            for sf in range(3):
                seed_aa = translate(seed_nucs, sf, '-')
                a_seed, a_ref, score = self._pair_align(seed_aa, ref)
                if score > seed_score:
                    seed_score, seed_best = score, (seed_aa, a_seed, a_ref)
            seed_aa, a_seed, a_ref = seed_best
            ref_to_seed = _walk(a_seed, seed_aa, a_ref, ref)
            a_seed2, a_cons, _ = self._pair_align(seed_aa, cons)
            seed_to_cons = _walk(a_cons.replace('?', '-'), cons, a_seed2, seed_aa)
            inserts = self.inserts[name] = set(range(len(cons)))
            blank = AminoTally(None)
            tallies = self.seed_aminos[f]
            for ri in sorted(ref_to_seed):
                ci = seed_to_cons.get(ref_to_seed[ri])
                t = blank if ci is None else tallies[ci]
                mapped.append((t, ri + 1))
                if t.consensus_index is not None:
                    inserts.remove(t.consensus_index)
        self.reports[name] = mapped

    # headers
    def write_amino_header(self, f):
        _writer(f).writerow(['seed', 'region', 'q-cutoff', 'query.aa.pos', 'refseq.aa.pos'] +
                            list(AMINOS))

    def write_nuc_header(self, f):
        _writer(f).writerow(['seed', 'region', 'q-cutoff', 'query.nuc.pos', 'refseq.nuc.pos',
                             'A', 'C', 'G', 'T'])

    def write_consensus_header(self, f):
        _writer(f).writerow(['region', 'q-cutoff', 'consensus-percent-cutoff', 'offset',
                             'sequence'])

    def write_failure_header(self, f):
        _writer(f).writerow(['seed', 'region', 'qcut', 'queryseq', 'refseq'])

    def write_nuc_variants_header(self, f):
        _writer(f).writerow(['seed', 'qcut', 'region', 'index', 'count', 'seq'])

    # reports
    def write_amino_counts(self, f, coverage_summary=None):
        w = _writer(f)
        for region in sorted(self.reports):
            total, n = 0.0, 0
            for t, pos in self.reports[region]:
                counts = [t.counts[a] for a in AMINOS]
                qpos = '' if t.consensus_index is None else t.consensus_index + 1
                w.writerow([self.seed, region, self.qcut, qpos, pos] + counts)
                total += sum(counts)
                n += 1
            if coverage_summary is not None and n:
                cov = total / n
                if cov > coverage_summary.get('avg_coverage', -1):
                    coverage_summary['avg_coverage'] = cov
                    coverage_summary['coverage_region'] = region
                    coverage_summary['region_width'] = n

    def write_nuc_counts(self, f):
        w = _writer(f)

        def emit(region, t, pos):
            for i, nt in enumerate(t.nucleotides):
                qpos = '' if t.consensus_index is None else i + 3 * t.consensus_index + 1
                rpos = '' if pos is None else i + 3 * pos - 2
                w.writerow([self.seed, region, self.qcut, qpos, rpos] +
                           [nt.counts[b] for b in 'ACGT'])
        if not self.coordinate_refs:
            for t in self.seed_aminos[0]:
                emit(self.seed, t, None)
        else:
            for region, mapped in self.reports.items():
                for t, pos in mapped:
                    emit(region, t, pos)

    def write_consensus(self, f, min_coverage=100):
        w = _writer(f)
        tallies = self.seed_aminos[0]
        for cut in self.conseq_mixture_cutoffs:
            seq, offset = [], None
            for t in tallies:
                if offset is None:
                    if not t.counts:
                        continue
                    offset = t.consensus_index * 3
                for nt in t.nucleotides:
                    letter = nt.get_consensus(cut)
                    depth = sum(nt.counts.values())
                    seq.append(letter.upper() if depth >= min_coverage else letter.lower())
            if offset is not None:
                w.writerow([self.seed, self.qcut, fmt_cutoff(cut), offset, ''.join(seq)])

    def write_failure(self, f):
        w = _writer(f)
        for region, mapped in self.reports.items():
            if not mapped:
                w.writerow([self.seed, region, self.qcut, self.consensus[region],
                            self.projects.getReference(region)])

    def write_insertions(self):
        for name, ins in self.inserts.items():
            self.insert_writer.write(ins, name, self.reading_frames[name], self.reports[name])

    def write_nuc_variants(self, f):
        keys = self.variants.keys()
        keys.sort()      # AttributeError under Python 3, as in the reference


class Inserts(object):
    """InsertionWriter."""

    def __init__(self, f):
        self.w = _writer(f)
        self.w.writerow(['seed', 'region', 'qcut', 'left', 'insert', 'count', 'before'])

    def start_group(self, seed, qcut):
        self.seed, self.qcut, self.nuc_seqs = seed, qcut, Counter()

    def add_nuc_read(self, offset_sequence, count):
        self.nuc_seqs[offset_sequence] += count

    def write(self, inserts, region, reading_frame=0, report_aminos=()):
        if len(inserts) == 0:
            return
        runs = []
        for i in sorted(inserts):
            if runs and runs[-1][1] == i:
                runs[-1][1] += 1
            else:
                runs.append([i, i + 1])
        for left, right in runs:
            before = None
            for item in report_aminos:
                t, pos = item if isinstance(item, tuple) else (item.seed_amino, item.position)
                if t.consensus_index == right:
                    before = pos
                    break
            tally = Counter()
            for s, n in self.nuc_seqs.items():
                piece = ('-' * reading_frame + s)[3 * left:3 * right]
                if piece and 'n' not in piece and '-' not in piece:
                    aa = translate(piece)
                    if aa:
                        tally[aa] += n
            if report_aminos and before in (1, None):
                continue
            for aa, n in tally.items():
                self.w.writerow([self.seed, region, self.qcut, left + 1, aa, n,
                                 '' if before is None else before])


def aln2counts(aligned_text, projects):
    """aln2counts() on aligned.csv text: {'nuc', 'amino', 'coord_ins',
    'conseq', 'failed', 'coverage': CSV text}."""
    outs = {k: io.StringIO() for k in ('nuc', 'amino', 'coord_ins', 'conseq', 'failed',
                                       'coverage')}
    rep = Report(Inserts(outs['coord_ins']), projects, CUTOFFS)
    rep.write_nuc_header(outs['nuc'])
    rep.write_amino_header(outs['amino'])
    rep.write_consensus_header(outs['conseq'])
    rep.write_failure_header(outs['failed'])
    cw = _writer(outs['coverage'])
    cw.writerow(['avg_coverage', 'coverage_region', 'region_width'])
    summary = {}
    rows = csv.DictReader(io.StringIO(aligned_text))
    for _key, group in itertools.groupby(rows, lambda r: (r['refname'], r['qcut'])):
        rep.read(group)
        rep.write_amino_counts(outs['amino'], coverage_summary=summary)
        rep.write_consensus(outs['conseq'])
        rep.write_failure(outs['failed'])
        rep.write_insertions()
        rep.write_nuc_counts(outs['nuc'])
    if summary:
        cw.writerow([summary['avg_coverage'], summary['coverage_region'], summary['region_width']])
    return {k: v.getvalue() for k, v in outs.items()}
