"""
aln2counts stage on the MI355X: the drop-in for micall/core/aln2counts.py.

Input is aligned.csv (sam2aln's distinct merged reads with their counts).
Rows are taken in runs of equal (refname, qcut) -- the reference groups them
with itertools.groupby (aln2counts.py:884-887) -- and every run produces
amino-acid and nucleotide counts in coordinate-reference positions, the
mixture consensus at each cutoff, the insertions relative to the coordinate
reference and the consensus sequences that did not align.  Output files are
byte-identical to the reference's (tests/test_gpu_aln2counts.py).

Split of the work:
  device -- everything per read: 3-frame codon / base counting of a run,
            with the first row that touched each counter (k_a2c_count), and
            the grouping of inserted amino-acid strings (k_a2c_ins_*),
            csrc/mh_a2c.hip.  The first row replaces the reference's Counter
            insertion order, which decides most_common() ties.
  host   -- everything per run and O(reference length): consensus letters
            from the counters (numpy), the coordinate mapping with its local
            EmpHIV25 Gotoh alignments (run on the device by mh_gotoh_align)
            and the CSV text.

Public names (SequenceReport, InsertionWriter, SeedAmino, SeedNucleotide,
ReportAmino, format_cutoff, aln2counts) and their signatures are the
reference's, so callers and the reference's tests drive this module
unchanged.  Differences that never reach an output file:
  * the progress callback hears the start and the end of each run, not every
    1 % of the file (aln2counts.py:136-141);
  * the nucleotide variant counts that the reference computes and drops
    (aln2counts.py:346-375) are not computed;
  * an InsertionWriter fed by a SequenceReport reads the run's rows from the
    device, so its nuc_seqs stays empty;
  * characters other than A C G T N - n, negative offsets and counts of 2**32
    or more raise NativeError.
There is no CPU path: without libmicall_hip.so or a device the first call
raises NativeUnavailable.
"""
import argparse
import csv
import io
import json as jsonlib
import os
import re
from collections import Counter, namedtuple

import numpy as np

from . import _native
from . import projects as project_config
from . import session
from .translation import AMBIG, codon_chars, translate

AMINO_ALPHABET = 'ACDEFGHIKLMNPQRSTVWY*'
CONSEQ_MIXTURE_CUTOFFS = [0.01, 0.02, 0.05, 0.1, 0.2, 0.25]
GAP_OPEN_COORD, GAP_EXTEND_COORD = 40, 10
MAX_CUTOFF = 'MAX'

# Column order of every file the stage writes (the reference's output schema).
_SCHEMA = {
    'amino': ['seed', 'region', 'q-cutoff', 'query.aa.pos', 'refseq.aa.pos'] + list(AMINO_ALPHABET),
    'nuc': ['seed', 'region', 'q-cutoff', 'query.nuc.pos', 'refseq.nuc.pos'] + list('ACGT'),
    'conseq': ['region', 'q-cutoff', 'consensus-percent-cutoff', 'offset', 'sequence'],
    'nuc_variants': ['seed', 'qcut', 'region', 'index', 'count', 'seq'],
    'failed': ['seed', 'region', 'qcut', 'queryseq', 'refseq'],
    'insert': ['seed', 'region', 'qcut', 'left', 'insert', 'count', 'before'],
    'coverage': ['avg_coverage', 'coverage_region', 'region_width'],
}

SLOT_REPORT, SLOT_INSERTS = 0, 1      # device row tables (mh_a2c slots) used here
_CODON_CHARS = codon_chars()
_NONE = np.uint32(0xffffffff)         # "no row touched this counter"
_AA = np.array(list(AMINO_ALPHABET))
# IUPAC letter of a set of bases, indexed by the mask A=1 C=2 G=4 T=8
_MIX = np.array(['', 'A', 'C', 'M', 'G', 'R', 'S', 'V', 'T', 'W', 'Y', 'H', 'K', 'D', 'B', 'N'])
_MODELS = os.path.join(os.path.dirname(os.path.abspath(__file__)), 'data', 'gotoh_models.json')


def _csv_writer(handle, kind):
    return csv.DictWriter(handle, _SCHEMA[kind], lineterminator=os.linesep)


def _text(value):
    return value.decode('utf-8') if isinstance(value, bytes) else value


class _CoordinateAligner(object):
    """The module-level coordinate aligner of aln2counts.py:34-37 (local
    Gotoh, gap open 40 / extend 10, EmpHIV25 scores), evaluated on the device
    by mh_gotoh_align.  A seed's three translations meet the same coordinate
    references in every run, so results are kept (bounded) by input pair."""

    MEMO_LIMIT = 4096

    def __init__(self, gop, gep, is_global, model):
        with open(_MODELS) as f:
            spec = jsonlib.load(f)[model]
        self.gap_open_penalty, self.gap_extend_penalty = gop, gep
        self.is_global = is_global
        self.matrix, self.alphabet = spec['matrix'], spec['alphabet']
        self._outside = re.compile('[^%s]' % (self.alphabet,))
        self._memo = {}

    def forget(self):
        self._memo.clear()

    @staticmethod
    def _check(seq1, seq2):
        # gotoh2.py:74-96 asserts these (AssertionError as there)
        for name, seq in (('seq1', seq1), ('seq2', seq2)):
            if type(seq) is not str:
                raise AssertionError('%s must be a string' % name)
            if not seq:
                raise AssertionError('%s cannot be an empty string' % name)

    def align(self, seq1, seq2):
        """(aligned seq1, aligned seq2, score)."""
        return self.align_many([(seq1, seq2)])[0]

    def align_many(self, pairs):
        """align() of every pair; the pairs not seen before go to the device
        in one launch (mh_gotoh_align_batch).  A pair that fails raises, in
        pair order."""
        for seq1, seq2 in pairs:
            self._check(seq1, seq2)
        todo = list(dict.fromkeys(p for p in pairs if p not in self._memo))
        if todo:
            found = session.context().gotoh_align_many(
                [(self._outside.sub('?', a.upper()), self._outside.sub('?', b.upper()))
                 for a, b in todo],
                self.gap_open_penalty, self.gap_extend_penalty, self.is_global, self.alphabet,
                self.matrix)
            if len(self._memo) + len(todo) > self.MEMO_LIMIT:
                self._memo.clear()
            self._memo.update(zip(todo, found))
        out = [self._memo[p] for p in pairs]
        for result in out:
            if isinstance(result, Exception):
                raise result
        return out


aligner = _CoordinateAligner(GAP_OPEN_COORD, GAP_EXTEND_COORD, False, 'EmpHIV25')


# ---------------------------------------------------------------------------
# consensus letters and alignment walks
# ---------------------------------------------------------------------------
def _nuc_letters(cnt, first, cutoff):
    """The nucleotide consensus letter of every position at once
    (SeedNucleotide.get_consensus semantics, aln2counts.py:655-695).
    cnt / first: (positions, 6) over A C G T N -, `first` = first row that
    read the base (_NONE: never).  Returns (letters, coverage)."""
    present = first != _NONE
    total = cnt.sum(axis=1)
    acgt = present[:, :4]
    if cutoff == MAX_CUTOFF:
        score = np.where(acgt, cnt[:, :4], -1)
        mix = acgt & (score == score.max(axis=1, initial=-1)[:, None])
    else:
        mix = acgt & (cnt[:, :4] >= (total * cutoff)[:, None])
    letters = _MIX[mix.astype(np.int64) @ np.array([1, 2, 4, 8])]
    letters[letters == ''] = 'N'                  # every base below the cutoff
    # Only 'N' and / or '-' read: the first of them in most_common() order
    # is the one the removal of gaps and poor quality keeps.
    solo = present.any(axis=1) & ~acgt.any(axis=1)
    if solo.any():
        nc, dc = cnt[solo, 4], cnt[solo, 5]
        dash = present[solo, 5] & (~present[solo, 4] | (dc > nc) |
                                   ((dc == nc) & (first[solo, 5] < first[solo, 4])))
        kept = np.where(dash, dc, nc)
        ok = True if cutoff == MAX_CUTOFF else kept >= total[solo] * cutoff
        letters[solo] = np.where(ok, np.where(dash, '-', 'N'), 'N')
    letters[~present.any(axis=1)] = ''
    return letters, total


def _index_map(aligned_from, seq_from, aligned_to, seq_to):
    """{index in seq_to: index in seq_from} along an alignment: at every
    column where seq_from advances, the current seq_to index maps to it
    (the two walks of aln2counts.py:255-264 and :272-281)."""
    out = {}
    i = j = 0
    n_from, n_to = len(seq_from), len(seq_to)
    for a, b in zip(aligned_from, aligned_to):
        if i < n_from and a == seq_from[i]:
            out[j] = i
            i += 1
        if j < n_to and b == seq_to[j]:
            j += 1
    return out


def _fill(counter, letters, cnt, first):
    """Counter entries in first-row (insertion) order."""
    for k in np.argsort(first, kind='stable'):
        if first[k] == _NONE:
            break
        counter[letters[k]] = int(cnt[k])


# ---------------------------------------------------------------------------
# device counters of one run
# ---------------------------------------------------------------------------
_Run = namedtuple('_Run', 'ctx slot group ncod seed qcut')


class _Frame(object):
    """Device counters of one reading frame of one run."""

    def __init__(self, ctx, slot, g, frame, ncod):
        self.ncod = ncod
        if ncod:
            aa_cnt, aa_first, nt_cnt, nt_first = ctx.a2c_counts(slot, g, frame, ncod)
        else:
            aa_cnt = aa_first = np.zeros((0, 21), np.uint32)
            nt_cnt = nt_first = np.zeros((0, 18), np.uint32)
        self.aa_cnt = aa_cnt.astype(np.int64)
        self.aa_first = aa_first
        self.nt_cnt = nt_cnt.astype(np.int64).reshape(-1, 3, 6)
        self.nt_first = nt_first.reshape(-1, 3, 6)
        self.has = (aa_first != _NONE).any(axis=1)      # the codon's Counter is not empty
        self._consensus = None

    def consensus(self):
        """Amino-acid consensus of the frame: the most counted amino acid of
        each codon, ties to the first one counted; '-' where none was."""
        if self._consensus is None:
            present = self.aa_first != _NONE
            score = np.where(present, self.aa_cnt, -1)
            tied = present & (score == score.max(axis=1, initial=-1)[:, None])
            pick = np.where(tied, self.aa_first, _NONE).argmin(axis=1)
            self._consensus = ''.join(np.where(self.has, _AA[pick], '-').tolist())
        return self._consensus

    def seed_amino(self, i):
        """A SeedAmino holding the device counts of codon i."""
        amino = SeedAmino(i)
        if i < self.ncod:
            _fill(amino.counts, AMINO_ALPHABET, self.aa_cnt[i], self.aa_first[i])
            for t, nuc in enumerate(amino.nucleotides):
                _fill(nuc.counts, 'ACGTN-', self.nt_cnt[i, t], self.nt_first[i, t])
        return amino


class _FrameAminos(object):
    """seed_aminos[frame] as a sequence of SeedAmino, materialised on access."""

    def __init__(self, frame, length):
        self._frame = frame
        self._len = length

    def __len__(self):
        return self._len

    def __getitem__(self, i):
        if isinstance(i, slice):
            return [self[k] for k in range(*i.indices(self._len))]
        if i < 0:
            i += self._len
        if not 0 <= i < self._len:
            raise IndexError('list index out of range')
        return self._frame.seed_amino(i)

    def __iter__(self):
        return (self[i] for i in range(self._len))


class _LazySeedAmino(object):
    """A report position's SeedAmino: its index now, its counts on access."""

    def __init__(self, frame, index):
        self.consensus_index = index
        self._frame = frame
        self._amino = None

    def __getattr__(self, name):
        if name.startswith('_'):
            raise AttributeError(name)
        if self._amino is None:
            self._amino = self._frame.seed_amino(self.consensus_index)
        return getattr(self._amino, name)

    def __repr__(self):
        return repr(self._frame.seed_amino(self.consensus_index))


class _CoordinateMap(object):
    """Where one coordinate region sits in a run: the chosen reading frame,
    and per coordinate position the consensus codon index (-1: none)."""

    def __init__(self, frame=0, conseq_index=(), positions=()):
        self.frame = frame
        self.conseq_index = np.asarray(conseq_index, dtype=np.int64)
        self.positions = np.asarray(positions, dtype=np.int64)

    def __len__(self):
        return len(self.conseq_index)


# ---------------------------------------------------------------------------
# SequenceReport
# ---------------------------------------------------------------------------
class SequenceReport(object):
    """Counts and reports of one (refname, qcut) run of aligned reads
    (aln2counts.py:73-579).  read() a run, then call the write_* methods."""

    def __init__(self, insert_writer, projects, conseq_mixture_cutoffs):
        self.insert_writer = insert_writer
        self.projects = projects
        self.conseq_mixture_cutoffs = [MAX_CUTOFF] + list(conseq_mixture_cutoffs)
        self.callback = None

    def enable_callback(self, callback, file_size):
        """Report reading progress to callback(message, progress, max_progress)."""
        self.callback = callback
        self.callback_max = file_size
        callback(message='... extracting statistics from alignments', progress=0,
                 max_progress=file_size)

    def _pair_align(self, reference, query):
        """(aligned reference, aligned query, score) of the coordinate aligner;
        test doubles override this one method."""
        return aligner.align(_text(reference), _text(query))

    def _pair_align_many(self, pairs):
        """_pair_align of every (reference, query) pair: one device launch,
        unless a subclass (a test double) replaces _pair_align, which then
        answers each pair in turn."""
        if type(self)._pair_align is not SequenceReport._pair_align:
            return [self._pair_align(r, q) for r, q in pairs]
        return aligner.align_many([(_text(r), _text(q)) for r, q in pairs])

    # ---- reading a run ----
    def read(self, aligned_reads):
        """Start over with the rows given (dicts with refname, qcut, count,
        offset, seq); they go to the device as one run."""
        rows = list(aligned_reads)
        run = None
        if rows:
            ctx = session.context()
            ctx.a2c_load_rows(SLOT_REPORT, [r['seq'] for r in rows],
                              [int(r['offset']) for r in rows], [int(r['count']) for r in rows],
                              [0, len(rows)], _CODON_CHARS)
            run = _Run(ctx, SLOT_REPORT, 0, ctx.a2c_group(SLOT_REPORT, 0)['ncod'],
                       rows[0]['refname'], rows[0]['qcut'])
        self._start(run)

    def _read_group(self, ctx, slot, g):
        """read() of run g of a row table that is already on the device."""
        info = ctx.a2c_group(slot, g)
        self._start(_Run(ctx, slot, g, info['ncod'], info['refname'], info['qcut']))

    def _start(self, run):
        # state the write_* methods use; attribute names are the reference's
        for name in ('seed_aminos', 'reports', 'reading_frames', 'inserts', 'consensus',
                     'variants'):
            setattr(self, name, {})
        self._frames = None
        self._coord_maps = {}
        if run is not None:
            self.seed, self.qcut = run.seed, run.qcut
            self.insert_writer.start_group(run.seed, run.qcut)
            self.insert_writer._attach(run.ctx, run.slot, run.group)
            self._frames = [_Frame(run.ctx, run.slot, run.group, f, run.ncod[f])
                            for f in range(3)]
            self.seed_aminos = {f: _FrameAminos(fr, fr.ncod) for f, fr in enumerate(self._frames)}
        if self.callback:
            self.callback(progress=self.callback_max)
        self.coordinate_refs = {}
        if self.seed_aminos:
            self.coordinate_refs = self.projects.getCoordinateReferences(self.seed)
            if not self.coordinate_refs:
                # no coordinate region: frame 0 covers the whole seed
                codons = -(-len(self.projects.getReference(self.seed)) // 3)
                frame0 = self._frames[0]
                self.seed_aminos[0] = _FrameAminos(frame0, max(frame0.ncod, codons))
        if self.coordinate_refs:
            self._locate_all({name: _text(ref) for name, ref in self.coordinate_refs.items()})

    def _locate_all(self, refs):
        """Coordinate position -> seed position -> consensus codon for every
        coordinate region of the seed (aln2counts.py:191-304), the regions'
        alignments batched in three launches:
          1. every frame's amino-acid consensus against every coordinate
             reference: a region's frame is the one scoring above
             min(covered codons, reference length), best first;
          2. the seed's three translations against each located region's
             reference: the best one maps coordinate -> seed positions;
          3. that translation against the chosen consensus: seed ->
             consensus positions."""
        frames = list(self.seed_aminos)
        conseqs = [self._frames[f].consensus() for f in frames]
        covered = int(self._frames[0].has.sum())
        for name in refs:
            self.consensus[name] = conseqs[0]           # kept if no frame aligns
        scores = iter(r[2] for r in self._pair_align_many(
            [(refs[name], c) for name in refs for c in conseqs]))
        chosen = {}
        for name, ref in refs.items():
            bar = min(covered, len(ref))
            for f, c in zip(frames, conseqs):
                score = next(scores)
                if score > bar:
                    bar, chosen[name] = score, (f, c)
        placed = {}
        if chosen:
            seed_nucs = self.projects.getReference(self.seed)
            translations = [translate(seed_nucs, offset=o, ambig_char='-') for o in range(3)]
            found = iter(self._pair_align_many(
                [(t, refs[name]) for name in chosen for t in translations]))
            for name in chosen:
                best_score, best = 0, None
                for t in translations:
                    aligned_seed, aligned_ref, score = next(found)
                    if score > best_score:
                        best_score, best = score, (t, aligned_seed, aligned_ref)
                t, aligned_seed, aligned_ref = best   # TypeError if none scored, as the reference
                placed[name] = (t, _index_map(aligned_seed, t, aligned_ref, refs[name]))
            final = self._pair_align_many([(placed[name][0], chosen[name][1]) for name in chosen])
        else:
            final = []
        blank = SeedAmino(None)
        finals = dict(zip(chosen, final))
        for name in refs:
            report, cmap = [], _CoordinateMap()
            if name in chosen:
                frame, consensus = chosen[name]
                self.reading_frames[name] = frame
                self.consensus[name] = consensus
                seed_aminos, ref_to_seed = placed[name]
                aligned_seed, aligned_conseq, _ = finals[name]
                # the aligner pads the left of a local alignment with '?'
                seed_to_conseq = _index_map(aligned_conseq.replace('?', '-'), consensus,
                                            aligned_seed, seed_aminos)
                unplaced = set(range(len(consensus)))
                self.inserts[name] = unplaced
                index, positions = [], []
                for ref_index in sorted(ref_to_seed):
                    k = seed_to_conseq.get(ref_to_seed[ref_index])
                    if k is None:
                        index.append(-1)
                        amino = blank
                    else:
                        index.append(k)
                        amino = _LazySeedAmino(self._frames[frame], k)
                        unplaced.remove(k)
                    positions.append(ref_index + 1)
                    report.append(ReportAmino(amino, ref_index + 1))
                cmap = _CoordinateMap(frame, index, positions)
            self.reports[name] = report
            self._coord_maps[name] = cmap

    def _gather(self, cmap, table, shape):
        """Rows of a per-codon counter table at the map's consensus codons
        (zeros where the coordinate position has none)."""
        out = np.zeros((len(cmap),) + shape, dtype=np.int64)
        hit = cmap.conseq_index >= 0
        if hit.any():
            out[hit] = table(self._frames[cmap.frame])[cmap.conseq_index[hit]]
        return out

    # ---- headers ----
    def write_amino_header(self, amino_file):
        _csv_writer(amino_file, 'amino').writeheader()

    def write_nuc_header(self, nuc_file):
        _csv_writer(nuc_file, 'nuc').writeheader()

    def write_consensus_header(self, conseq_file):
        _csv_writer(conseq_file, 'conseq').writeheader()

    def write_nuc_variants_header(self, nuc_variants_file):
        _csv_writer(nuc_variants_file, 'nuc_variants').writeheader()

    def write_failure_header(self, fail_file):
        _csv_writer(fail_file, 'failed').writeheader()

    # ---- bodies ----
    def write_amino_counts(self, amino_file, coverage_summary=None):
        """Amino-acid counts per coordinate position, regions in name order;
        the region with the highest mean count goes to coverage_summary."""
        out = csv.writer(amino_file, lineterminator=os.linesep)
        for name in sorted(self.reports):
            cmap = self._coord_maps[name]
            if not len(cmap):
                continue
            counts = self._gather(cmap, lambda fr: fr.aa_cnt, (len(AMINO_ALPHABET),))
            query = ['' if k < 0 else str(k + 1) for k in cmap.conseq_index.tolist()]
            out.writerows([self.seed, name, self.qcut, q, p] + c for q, p, c in
                          zip(query, cmap.positions.tolist(), counts.tolist()))
            if coverage_summary is not None:
                mean = float(counts.sum()) / len(cmap)
                if mean > coverage_summary.get('avg_coverage', -1):
                    coverage_summary.update(avg_coverage=mean, coverage_region=name,
                                            region_width=len(cmap))

    def write_nuc_counts(self, nuc_file):
        """A/C/G/T counts per nucleotide: in coordinate positions, or in seed
        positions when the seed has no coordinate region."""
        out = csv.writer(nuc_file, lineterminator=os.linesep)
        lines = []
        if not self.coordinate_refs:
            n = len(self.seed_aminos[0])      # KeyError without reads, as the reference
            frame = self._frames[0]
            counts = np.zeros((n, 3, 4), dtype=np.int64)
            counts[:frame.ncod] = frame.nt_cnt[:, :, :4]
            for codon, per_base in enumerate(counts.tolist()):
                lines.extend([self.seed, self.seed, self.qcut, 3 * codon + t + 1, ''] + acgt
                             for t, acgt in enumerate(per_base))
        else:
            for name, cmap in ((n, self._coord_maps[n]) for n in self.reports):
                counts = self._gather(cmap, lambda fr: fr.nt_cnt[:, :, :4], (3, 4))
                for k, pos, per_base in zip(cmap.conseq_index.tolist(), cmap.positions.tolist(),
                                            counts.tolist()):
                    lines.extend([self.seed, name, self.qcut, '' if k < 0 else 3 * k + t + 1,
                                  3 * pos - 2 + t] + acgt for t, acgt in enumerate(per_base))
        out.writerows(lines)

    def write_consensus(self, conseq_file, min_coverage=100):
        """The nucleotide consensus of frame 0 from its first counted codon
        on, one row per mixture cutoff; bases read fewer than min_coverage
        times in lower case."""
        seed_aminos = self.seed_aminos[0]     # KeyError without reads, as the reference
        frame = self._frames[0]
        counted = np.flatnonzero(frame.has[:len(seed_aminos)])
        if not len(counted):
            return
        start = int(counted[0])
        cnt = frame.nt_cnt[start:].reshape(-1, 6)
        first = frame.nt_first[start:].reshape(-1, 6)
        out = _csv_writer(conseq_file, 'conseq')
        for cutoff in self.conseq_mixture_cutoffs:
            letters, depth = _nuc_letters(cnt, first, cutoff)
            letters = np.where(depth >= min_coverage, letters, np.char.lower(letters))
            out.writerow({'region': self.seed, 'q-cutoff': self.qcut,
                          'consensus-percent-cutoff': format_cutoff(cutoff),
                          'offset': start * 3, 'sequence': ''.join(letters.tolist())})

    def write_nuc_variants(self, nuc_variants_file):
        """The reference sorts dict.keys() in place here, which fails under
        Python 3 with AttributeError; so does this (no output either way)."""
        getattr(self.variants.keys(), 'sort')()

    def write_failure(self, fail_file):
        """One row per coordinate region that no reading frame aligned to."""
        out = _csv_writer(fail_file, 'failed')
        out.writerows(dict(seed=self.seed, region=name, qcut=self.qcut,
                           queryseq=self.consensus[name],
                           refseq=self.projects.getReference(name))
                      for name, report in self.reports.items() if not report)

    def write_insertions(self):
        for name in self.inserts:
            self.insert_writer.write(self.inserts[name], name, self.reading_frames[name],
                                     self.reports[name])


# ---------------------------------------------------------------------------
# per-codon / per-base counters (the reference's object API)
# ---------------------------------------------------------------------------
class SeedNucleotide(object):
    """Counts of the letters read at one nucleotide position."""

    def __init__(self):
        self.counts = Counter()

    def count_nucleotides(self, nuc_seq, count):
        # 'n' marks the unread gap between the forward and the reverse read
        if nuc_seq == 'n':
            return
        self.counts[nuc_seq] += count

    def get_report(self):
        return ','.join(str(self.counts[base]) for base in 'ACGT')

    def get_consensus(self, mixture_cutoff):
        """Consensus letter at a mixture cutoff (a fraction, or MAX_CUTOFF for
        the most counted bases only); a tie or a mixture is an IUPAC code.
        'N' and '-' count only when nothing else was read."""
        if not self.counts:
            return ''
        ranked = self.counts.most_common()
        informative = [pair for pair in ranked if pair[0] not in 'N-']
        candidates = informative or ranked[:1]
        if mixture_cutoff == MAX_CUTOFF:
            floor = candidates[0][1]
        else:
            floor = sum(self.counts.values()) * mixture_cutoff
        chosen = sorted(base for base, n in candidates if n >= floor)
        if not chosen:
            return 'N'
        return chosen[0] if len(chosen) == 1 else AMBIG[''.join(chosen)]


class SeedAmino(object):
    """Counts of the amino acids read at one codon, plus its three bases."""

    def __init__(self, consensus_index):
        self.consensus_index = consensus_index
        self.counts = Counter()
        self.nucleotides = [SeedNucleotide(), SeedNucleotide(), SeedNucleotide()]

    def __repr__(self):
        return '%s(%s): %s' % (type(self).__name__, self.consensus_index, self.counts)

    def count_aminos(self, codon_seq, count):
        amino = translate(codon_seq.upper())
        if amino in AMINO_ALPHABET:
            self.counts[amino] += count
        for k, nuc in enumerate(self.nucleotides):
            nuc.count_nucleotides(codon_seq[k], count)

    def get_report(self):
        return ','.join(str(self.counts[a]) for a in AMINO_ALPHABET)

    def get_consensus(self):
        top = self.counts.most_common(1)
        return top[0][0] if top else '-'


class ReportAmino(object):
    """A coordinate position (1-based) and the SeedAmino reported there."""

    __slots__ = ('seed_amino', 'position')

    def __init__(self, seed_amino, position):
        self.seed_amino, self.position = seed_amino, position

    def __repr__(self):
        return '%s(%r, %s)' % (type(self).__name__, self.seed_amino, self.position)


# ---------------------------------------------------------------------------
# insertions
# ---------------------------------------------------------------------------
def _ranges(indices):
    """Sorted indices -> [left, right) runs of consecutive values."""
    runs = []
    for k in sorted(indices):
        if runs and runs[-1][1] == k:
            runs[-1][1] = k + 1
        else:
            runs.append([k, k + 1])
    return runs


class InsertionWriter(object):
    """Writes the amino-acid strings read at consensus codons that have no
    coordinate position (insert.csv).  The counting over the reads runs on
    the device: over the run a SequenceReport attached, or over the reads
    given to add_nuc_read."""

    def __init__(self, insert_file):
        self._file = insert_file
        self.insert_writer = _csv_writer(insert_file, 'insert')
        self.insert_writer.writeheader()
        self.nuc_seqs = Counter()
        self._source = None

    def start_group(self, seed, qcut):
        self.seed, self.qcut = seed, qcut
        self.nuc_seqs = Counter()
        self._source = None

    def add_nuc_read(self, offset_sequence, count):
        """A read already padded with '-' to its consensus offset."""
        self.nuc_seqs[offset_sequence] += count

    def _attach(self, ctx, slot, g):
        """The reads of this run are run g of the device table `slot`."""
        self._source = (ctx, slot, g)

    def _source_of(self):
        """(ctx, slot, group) of the reads to count insertions over."""
        if self._source is not None:
            return self._source
        if not self.nuc_seqs:
            return None
        reads = list(self.nuc_seqs)
        ctx = session.context()
        ctx.a2c_load_rows(SLOT_INSERTS, reads, [0] * len(reads),
                          [self.nuc_seqs[r] for r in reads], [0, len(reads)], _CODON_CHARS)
        return ctx, SLOT_INSERTS, 0

    def write(self, inserts, region, reading_frame=0, report_aminos=()):
        """Rows for each run of inserted consensus codons: the 1-based left
        codon, each amino-acid string with its count, and the coordinate
        position the run precedes.  Runs placed before coordinate position 1
        or past the end are skipped when report_aminos is given.  The strings
        are counted and the rows formatted by the library (mh_a2c_inserts,
        mh_a2c_insert_rows)."""
        if len(inserts) == 0:
            return
        before = {}
        for ra in report_aminos:
            before.setdefault(ra.seed_amino.consensus_index, ra.position)
        target = {}
        for left, right in _ranges(inserts):
            if right in before:
                target[left] = before[right]
        kept = [r for r in _ranges(inserts)
                if not report_aminos or target.get(r[0]) not in (1, None)]
        if not kept:
            return
        source = self._source_of()
        if source is None:
            return
        # the leading text columns go through the csv module (quoting); the
        # rest are numbers and amino-acid letters, which never need quotes
        lead = io.StringIO()
        csv.writer(lead, lineterminator='').writerow([self.seed, region, self.qcut, ''])
        ctx, slot, g = source
        lefts, rights = [r[0] for r in kept], [r[1] for r in kept]
        targets = [target.get(r[0]) for r in kept]
        if _SHARD is not None and slot == SLOT_REPORT:
            # every rank's strings over its own rows, added up (the first
            # rows are the job's row numbers within the group)
            from .sharded_io import _checked
            mine = _checked(_SHARD, lambda: ctx.a2c_inserts_local(slot, g, reading_frame, lefts, rights))
            text = ctx.a2c_inserts_merged_text(slot, b''.join(_SHARD.all_gather_bytes(mine)), lefts,
                                               lead.getvalue(), targets, os.linesep)
        else:
            text = ctx.a2c_inserts_text(slot, g, reading_frame, lefts, rights, lead.getvalue(), targets,
                                        os.linesep)
        if text:
            self._file.write(text)


def format_cutoff(cutoff):
    """Name of a mixture cutoff in conseq.csv: 'MAX' or three decimals."""
    return cutoff if cutoff == MAX_CUTOFF else '%.3f' % cutoff


SHARD_STATS = {}   # how the last sharded call ran (tests): rows and bytes this rank parsed
_SHARD = None      # the job's Shard while a sharded aln2counts runs (InsertionWriter.write)


def aln2counts(aligned_csv, nuc_csv, amino_csv, coord_ins_csv, conseq_csv,
               failed_align_csv=None, nuc_variants_csv=None, callback=None,
               coverage_summary_csv=None, json=None):
    """aligned.csv -> nucleotide, amino-acid, insertion, consensus (and the
    optional failure, variant and coverage) reports; every argument is an
    open file except json, a project-file path (None: the default).

    In a sharded job the counting is split: every rank counts the rows in
    its share of aligned.csv and the ranks add their counters up
    (_load_sharded); every rank then builds the same reports from the
    job's counters, and rank 0 writes them (session.writer_stage).  The
    insertion strings are counted the same way (InsertionWriter.write).
    When aligned.csv cannot be split (not a plain file on every rank, '\r'
    or quoted fields), rank 0 computes alone while the others wait."""
    global _SHARD
    sh = session.shard()
    SHARD_STATS.clear()
    handles = (nuc_csv, amino_csv, coord_ins_csv, conseq_csv, failed_align_csv, nuc_variants_csv,
               coverage_summary_csv)
    with session.writer_stage(*handles) as stage:
        groups = _load_sharded(sh, aligned_csv) if sh is not None else None
        if groups is None:
            if stage.active:
                _aln2counts(aligned_csv, nuc_csv, amino_csv, coord_ins_csv, conseq_csv,
                            failed_align_csv, nuc_variants_csv, callback, coverage_summary_csv, json)
            return
        # every rank builds the reports; the others' go nowhere
        outs = handles if stage.active else tuple(None if h is None else io.StringIO() for h in handles)
        _SHARD = sh
        try:
            _aln2counts(aligned_csv, outs[0], outs[1], outs[2], outs[3], outs[4], outs[5],
                        callback if stage.active else None, outs[6], json, groups=groups)
        finally:
            _SHARD = None


def _load_sharded(sh, aligned_csv):
    """This rank's share of aligned.csv counted into the job's groups, the
    counters added up over the ranks: the number of (refname, qcut) groups,
    or None (on every rank) when the file is not split."""
    from .sharded_io import _agree_ok, _checked
    ctx = session.context()
    fd = session.readable_fd(aligned_csv)
    if not _agree_ok(sh, fd is not None):
        return None
    part = _checked(sh, lambda: ctx.a2c_part_open(SLOT_REPORT, fd, sh.rank, sh.world, _CODON_CHARS))
    if not _agree_ok(sh, part is not None):
        return None
    aligned_csv.seek(0, 2)    # consumed, as the reference's DictReader leaves it
    keys, rows, ncod, total = ctx.a2c_part_groups(SLOT_REPORT, part['groups'])
    all_keys = sh.all_gather_bytes(keys)
    all_meta = sh.all_gather_bytes(np.concatenate([rows, ncod.reshape(-1), total]).astype(np.int64).tobytes())
    # the job's groups: runs of equal keys in rank order (a run can go on
    # across the ranks' cuts)
    g_keys, g_ncod, g_total, g_rows = [], [], [], []
    mine_gid, mine_base = [], []
    for r in range(sh.world):
        ks = all_keys[r].split(b'\n')[:-1] if all_keys[r] else []
        meta = np.frombuffer(all_meta[r], dtype=np.int64)
        n = len(ks)
        rr, nc, tt = meta[:n], meta[n:4 * n].reshape(n, 3), meta[4 * n:5 * n]
        for k in range(n):
            if k == 0 and g_keys and g_keys[-1] == ks[k]:
                g = len(g_keys) - 1
                g_ncod[g] = np.maximum(g_ncod[g], nc[k])
            else:
                g = len(g_keys)
                g_keys.append(ks[k])
                g_ncod.append(nc[k].copy())
                g_total.append(0)
                g_rows.append(0)
            if r == sh.rank:
                mine_gid.append(g)
                mine_base.append(g_rows[g])
            g_total[g] += int(tt[k])
            g_rows[g] += int(rr[k])
    for g, t in enumerate(g_total):
        if t > 0xffffffff:
            raise _native.NativeError('aln2counts: the counts of group %d add up to more than 2**32-1' % g)
    cells = ctx.a2c_part_count(SLOT_REPORT, b''.join(k + b'\n' for k in g_keys), mine_gid,
                               np.array(g_ncod, dtype=np.int32).reshape(-1, 3), mine_base)
    cnt, first = ctx.a2c_part_counters(SLOT_REPORT, cells)
    total_cnt = sh.sum_i64(cnt.astype(np.int64))
    first64 = np.where(first == np.uint32(0xffffffff), -1, first.astype(np.int64))
    least = sh.min_i64(first64)
    ctx.a2c_part_counters(SLOT_REPORT, cells, (total_cnt.astype(np.uint32),
                                               np.where(least < 0, 0xffffffff, least).astype(np.uint32)))
    SHARD_STATS.update(mode='sharded', rows=part['rows'], bytes=part['bytes'])
    return len(g_keys)


def _aln2counts(aligned_csv, nuc_csv, amino_csv, coord_ins_csv, conseq_csv, failed_align_csv,
                nuc_variants_csv, callback, coverage_summary_csv, json, groups=None):
    projects = (project_config.ProjectConfig.loadDefault() if json is None
                else project_config.ProjectConfig.loadCustom(json))
    report = SequenceReport(InsertionWriter(coord_ins_csv), projects, CONSEQ_MIXTURE_CUTOFFS)
    report.write_nuc_header(nuc_csv)
    report.write_amino_header(amino_csv)
    report.write_consensus_header(conseq_csv)
    # what is written for each run, in the reference's file order
    per_run = [lambda: report.write_amino_counts(amino_csv, coverage_summary=summary),
               lambda: report.write_consensus(conseq_csv)]
    if failed_align_csv:
        report.write_failure_header(failed_align_csv)
        per_run.append(lambda: report.write_failure(failed_align_csv))
    per_run += [report.write_insertions, lambda: report.write_nuc_counts(nuc_csv)]
    if nuc_variants_csv:
        report.write_nuc_variants_header(nuc_variants_csv)
        per_run.append(lambda: report.write_nuc_variants(nuc_variants_csv))
    summary = None
    if coverage_summary_csv is not None:
        summary_writer = _csv_writer(coverage_summary_csv, 'coverage')
        summary_writer.writeheader()
        summary = {}
    source = getattr(aligned_csv, 'name', None) if callback else None
    if source:
        report.enable_callback(callback, os.stat(source).st_size)
    ctx = session.context()
    if groups is None:           # not loaded by the ranks of a sharded job
        fd = session.readable_fd(aligned_csv)
        if fd is not None:   # the file mmap'd by the library (no '\r' in it)
            groups = ctx.a2c_load_file(SLOT_REPORT, fd, _CODON_CHARS)
            if groups is not None:
                aligned_csv.seek(0, 2)
        if groups is None:
            groups = ctx.a2c_load_csv(SLOT_REPORT, session.read_text(aligned_csv), _CODON_CHARS)
    for g in range(groups):
        report._read_group(ctx, SLOT_REPORT, g)
        for step in per_run:
            step()
    if summary:
        summary_writer.writerow(summary)


def _arguments():
    cli = argparse.ArgumentParser(description='aln2counts on the MI355X: counts, consensus and '
                                              'insertions from aligned.csv.')
    cli.add_argument('aligned_csv', type=argparse.FileType('r'), help='aligned.csv from sam2aln')
    for name, what in (('nuc_csv', 'nucleotide counts'), ('amino_csv', 'amino-acid counts'),
                       ('coord_ins_csv', 'insertions in coordinate positions'),
                       ('conseq_csv', 'consensus sequences')):
        cli.add_argument(name, type=argparse.FileType('w'), help='output: ' + what)
    cli.add_argument('--failed_align_csv', type=argparse.FileType('w'),
                     help='output: consensus sequences that did not align')
    cli.add_argument('--nuc_variants_csv', type=argparse.FileType('w'),
                     help='output: nucleotide variants')
    return cli.parse_args()


parseArgs = _arguments


def main():
    a = _arguments()
    aln2counts(a.aligned_csv, a.nuc_csv, a.amino_csv, a.coord_ins_csv, a.conseq_csv,
               a.failed_align_csv, a.nuc_variants_csv)


if __name__ == '__main__':
    main()
