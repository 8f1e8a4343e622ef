"""
Drop-in for micall/core/aln2counts.py: the same function, classes, arguments
and output files.

aln2counts() reads aligned.csv (sam2aln's distinct merged reads and their
counts), takes consecutive rows with the same (refname, qcut) as one group
(itertools.groupby, aln2counts.py:884-887) and writes, per group, amino-acid
and nucleotide counts in coordinate-reference positions, the mixture
consensus, insertions relative to the coordinate reference and the
consensus sequences that failed to align (aln2counts.py:822-898).

Where the work runs:
  * per read -- SequenceReport._count_reads (:115-172) and the read loop of
    InsertionWriter.write (:786-795) -- on the device: mh_a2c_load_csv /
    mh_a2c_load_rows count codons and bases in all three reading frames
    (k_a2c_count) and mh_a2c_inserts groups the insertion strings
    (k_a2c_ins_*), csrc/mh_a2c.hip.  Every counter comes with the first row
    that touched it: the Counter insertion order most_common() breaks ties by.
  * per group, O(reference length) -- here: the consensus letters (numpy),
    the coordinate mapping of _map_to_coordinate_ref (:191-304) with its
    local EmpHIV25 Gotoh alignments on the device (mh_gotoh_align, k_gotoh),
    and the CSV text.
There is no CPU fallback: without libmicall_hip.so or a device the first
call raises NativeUnavailable.  SeedAmino and SeedNucleotide keep the
reference's per-object API for code that uses them directly; the report does
not count through them (seed_aminos / reports hand them out, built from the
device counters on access).

Deviations, none of which changes an output file: the progress callback
hears the start and the end of each group, not every 1 % of :136-141; the
variant counts of :346-375, which the reference computes and discards, are
not computed; an InsertionWriter fed by a SequenceReport reads the group's
rows on the device, so its nuc_seqs stays empty; aligned.csv characters
outside A C G T N - n, negative offsets and counts >= 2**32 are rejected.
"""
import argparse
import csv
import io
import json as jsonlib
import os
import re
from collections import Counter

import numpy as np

from . import projects as project_config
from . import session
from .translation import AMBIG as ambig_dict, codon_chars, translate

AMINO_ALPHABET = 'ACDEFGHIKLMNPQRSTVWY*'
CONSEQ_MIXTURE_CUTOFFS = [0.01, 0.02, 0.05, 0.1, 0.2, 0.25]
GAP_OPEN_COORD = 40
GAP_EXTEND_COORD = 10
MAX_CUTOFF = 'MAX'

SLOT_REPORT, SLOT_INSERTS = 0, 1      # mh_a2c row tables used here
_CODON_CHARS = codon_chars()
_NONE = np.uint32(0xffffffff)
_AA = np.array(list(AMINO_ALPHABET))
# IUPAC letter of a set of bases, indexed by the bit mask A=1 C=2 G=4 T=8
_MIX = np.array(['', 'A', 'C', 'M', 'G', 'R', 'S', 'V', 'T', 'W', 'Y', 'H', 'K', 'D', 'B', 'N'])
_MODELS = os.path.join(os.path.dirname(os.path.abspath(__file__)), 'data', 'gotoh_models.json')


class Aligner(object):
    """gotoh2.Aligner (gotoh2.py:7-96) with the alignment on the device
    (mh_gotoh_align).  Alignments are memoised per (seq1, seq2): the seed's
    translations meet the same coordinate references in every group."""

    def __init__(self, gop=10, gep=1, is_global=False, model='HYPHY_NUC'):
        self.gap_open_penalty = gop
        self.gap_extend_penalty = gep
        self.is_global = is_global
        with open(_MODELS) as f:
            self.models = {name: (m['matrix'], m['alphabet']) for name, m in jsonlib.load(f).items()}
        self.set_model(model)
        self._memo = {}

    def set_model(self, model):
        if model in self.models:
            self.matrix, self.alphabet = self.models[model]
        else:
            print('ERROR: Unrecognized model name {}'.format(model))

    def clean_sequence(self, seq):
        return re.sub(pattern='[^%s]' % (self.alphabet,), repl='?', string=seq.upper())

    def align(self, seq1, seq2):
        assert type(seq1) is str, 'seq1 must be a string'
        assert type(seq2) is str, 'seq2 must be a string'
        assert len(seq1) > 0, 'seq1 cannot be an empty string'
        assert len(seq2) > 0, 'seq2 cannot be an empty string'
        key = (seq1, seq2)
        hit = self._memo.get(key)
        if hit is None:
            hit = session.context().gotoh_align(
                self.clean_sequence(seq1), self.clean_sequence(seq2), self.gap_open_penalty,
                self.gap_extend_penalty, self.is_global, self.alphabet, self.matrix)
            if len(self._memo) >= 4096:
                self._memo.clear()
            self._memo[key] = hit
        return hit


aligner = Aligner(gop=GAP_OPEN_COORD, gep=GAP_EXTEND_COORD, is_global=False, model='EmpHIV25')


def _nuc_letters(cnt, first, cutoff):
    """SeedNucleotide.get_consensus (:655-695) at every position at once.
    cnt / first: (positions, 6) over A C G T N -, first = the first row that
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
    # Only 'N' and / or '-' read here: the first of them in most_common()
    # order survives the removal of gaps and poor quality (:671-674).
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
    (the walks of :255-264 and :272-281)."""
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


class _Frame(object):
    """Device counters of one reading frame of one group."""

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
        self.has = (aa_first != _NONE).any(axis=1)      # SeedAmino.counts is not empty
        self._consensus = None

    def consensus(self):
        """''.join(SeedAmino.get_consensus()) over the frame (:214-215): the
        most counted amino acid, ties to the first one seen; '-' if none."""
        if self._consensus is None:
            present = self.aa_first != _NONE
            score = np.where(present, self.aa_cnt, -1)
            tied = present & (score == score.max(axis=1, initial=-1)[:, None])
            pick = np.where(tied, self.aa_first, _NONE).argmin(axis=1)
            self._consensus = ''.join(np.where(self.has, _AA[pick], '-').tolist())
        return self._consensus

    def seed_amino(self, i):
        """SeedAmino(i) holding the device counts of codon i."""
        amino = SeedAmino(i)
        if i < self.ncod:
            _fill(amino.counts, AMINO_ALPHABET, self.aa_cnt[i], self.aa_first[i])
            for t, nuc in enumerate(amino.nucleotides):
                _fill(nuc.counts, 'ACGTN-', self.nt_cnt[i, t], self.nt_first[i, t])
        return amino


class _FrameAminos(object):
    """seed_aminos[frame]: the reference's list of SeedAmino, built on access."""

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
    """A report's SeedAmino: consensus_index at once, the counts on access."""

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


class SequenceReport(object):
    """SequenceReport (:73-579): read the aligned reads of one (refname,
    qcut) group, then write its reports."""

    def __init__(self, insert_writer, projects, conseq_mixture_cutoffs):
        self.insert_writer = insert_writer
        self.projects = projects
        self.conseq_mixture_cutoffs = list(conseq_mixture_cutoffs)
        self.conseq_mixture_cutoffs.insert(0, MAX_CUTOFF)
        self.callback = None

    def enable_callback(self, callback, file_size):
        """:98-113."""
        self.callback = callback
        self.callback_max = file_size
        self.callback_chunk_size = file_size / 100
        self.callback_next = self.callback_chunk_size
        self.callback_progress = 0
        self.callback(message='... extracting statistics from alignments',
                      progress=0,
                      max_progress=self.callback_max)

    def _pair_align(self, reference, query):
        """:174-189."""
        if type(reference) == bytes:
            reference = reference.decode('utf-8')
        if type(query) == bytes:
            query = query.decode('utf-8')
        return aligner.align(reference, query)

    def read(self, aligned_reads):
        """SequenceReport.read (:306-375) on rows given here (dicts with
        refname, qcut, count, offset and seq): they go to the device as one
        group."""
        rows = list(aligned_reads)
        group = None
        if rows:
            seqs = [row['seq'] for row in rows]
            offsets = [int(row['offset']) for row in rows]
            counts = [int(row['count']) for row in rows]
            ctx = session.context()
            ctx.a2c_load_rows(SLOT_REPORT, seqs, offsets, counts, [0, len(rows)], _CODON_CHARS)
            ncod = ctx.a2c_group(SLOT_REPORT, 0)['ncod']
            group = (ctx, SLOT_REPORT, 0, ncod, rows[0]['refname'], rows[0]['qcut'])
        self._read(group)

    def _read_group(self, ctx, slot, g):
        """read() of group g of a table already on the device."""
        info = ctx.a2c_group(slot, g)
        self._read((ctx, slot, g, info['ncod'], info['refname'], info['qcut']))

    def _read(self, group):
        self.seed_aminos = {}  # {reading_frame: [SeedAmino(consensus_index)]}
        self.reports = {}  # {coord_name: [ReportAmino()]}
        self.reading_frames = {}  # {coord_name: reading_frame}
        self.inserts = {}  # {coord_name: set([consensus_index])}
        self.consensus = {}  # {coord_name: consensus_amino_seq}
        self.variants = {}  # {coord_name: [(count, nuc_seq)]}
        self._frames = None
        self._report_index = {}  # {coord_name: (frame, conseq indices, positions)}
        if group is not None:
            ctx, slot, g, ncod, self.seed, self.qcut = group
            self.insert_writer.start_group(self.seed, self.qcut)
            self.insert_writer._attach(ctx, slot, g)
            self._frames = [_Frame(ctx, slot, g, f, ncod[f]) for f in range(3)]
            for f in range(3):
                self.seed_aminos[f] = _FrameAminos(self._frames[f], ncod[f])
        if self.callback:
            self.callback(progress=self.callback_max)
        if not self.seed_aminos:
            self.coordinate_refs = {}
        else:
            self.coordinate_refs = self.projects.getCoordinateReferences(self.seed)
            if not self.coordinate_refs:
                # pad frame 0 to the seed reference's length (:336-338)
                seed_len = len(self.projects.getReference(self.seed))
                n0 = max(len(self.seed_aminos[0]), -(-seed_len // 3))
                self.seed_aminos[0] = _FrameAminos(self._frames[0], n0)
        for coordinate_name, coordinate_ref in self.coordinate_refs.items():
            self._map_to_coordinate_ref(coordinate_name, coordinate_ref)

    def _map_to_coordinate_ref(self, coordinate_name, coordinate_ref):
        """_map_to_coordinate_ref (:191-304): the best reading frame by local
        alignment with the coordinate reference, then coordinate position ->
        seed position -> consensus position."""
        if type(coordinate_ref) == bytes:
            coordinate_ref = coordinate_ref.decode('utf-8')
        consensus_length = int(self._frames[0].has.sum())
        max_score = min(consensus_length, len(coordinate_ref))
        best_alignment = None
        for reading_frame in self.seed_aminos:
            consensus = self._frames[reading_frame].consensus()
            if reading_frame == 0:
                # best guess before aligning
                self.consensus[coordinate_name] = consensus
            _aref, _aquery, score = self._pair_align(coordinate_ref, consensus)
            if score > max_score:
                max_score = score
                best_alignment = (reading_frame, consensus)
        report_aminos, index, positions, frame = [], [], [], 0
        if best_alignment is not None:
            frame, consensus = best_alignment
            self.reading_frames[coordinate_name] = frame
            self.consensus[coordinate_name] = consensus
            seed_nuc_seq = self.projects.getReference(self.seed)
            best_seed_alignment = None
            max_seed_score = 0
            for seed_frame in range(3):
                seed_amino_seq = translate(seed_nuc_seq, offset=seed_frame, ambig_char='-')
                aseed, aref, score = self._pair_align(seed_amino_seq, coordinate_ref)
                if score > max_seed_score:
                    max_seed_score = score
                    best_seed_alignment = (seed_amino_seq, aseed, aref)
            seed_amino_seq, aseed, aref = best_seed_alignment
            ref2seed = _index_map(aseed, seed_amino_seq, aref, coordinate_ref)
            aseed, aconseq, _score = self._pair_align(seed_amino_seq, consensus)
            aconseq = aconseq.replace('?', '-')  # gotoh2 pads the left with ?'s
            seed2conseq = _index_map(aconseq, consensus, aseed, seed_amino_seq)
            coordinate_inserts = set(range(len(consensus)))
            self.inserts[coordinate_name] = coordinate_inserts
            empty_seed_amino = SeedAmino(None)
            for ref_index in sorted(ref2seed):
                conseq_index = seed2conseq.get(ref2seed[ref_index])
                if conseq_index is None:
                    index.append(-1)
                    seed_amino = empty_seed_amino
                else:
                    index.append(conseq_index)
                    seed_amino = _LazySeedAmino(self._frames[frame], conseq_index)
                    coordinate_inserts.remove(conseq_index)
                positions.append(ref_index + 1)
                report_aminos.append(ReportAmino(seed_amino, ref_index + 1))
        self.reports[coordinate_name] = report_aminos
        self._report_index[coordinate_name] = (frame, np.array(index, dtype=np.int64),
                                               np.array(positions, dtype=np.int64))

    def _counts_at(self, frame, index, table, shape):
        out = np.zeros((len(index),) + shape, dtype=np.int64)
        hit = index >= 0
        if hit.any():
            out[hit] = table(self._frames[frame])[index[hit]]
        return out

    # ---- writers (:377-579) ----
    def _create_amino_writer(self, amino_file):
        columns = ['seed',
                   'region',
                   'q-cutoff',
                   'query.aa.pos',
                   'refseq.aa.pos']
        columns.extend(AMINO_ALPHABET)
        return csv.DictWriter(amino_file,
                              columns,
                              lineterminator=os.linesep)

    def write_amino_header(self, amino_file):
        self._create_amino_writer(amino_file).writeheader()

    def write_amino_counts(self, amino_file, coverage_summary=None):
        """Amino-acid counts at each coordinate-reference position (:391-433)."""
        writer = csv.writer(amino_file, lineterminator=os.linesep)
        for region in sorted(self.reports):
            frame, index, positions = self._report_index[region]
            n = len(index)
            if not n:
                continue
            counts = self._counts_at(frame, index, lambda fr: fr.aa_cnt, (len(AMINO_ALPHABET),))
            query = [str(i + 1) if i >= 0 else '' for i in index.tolist()]
            writer.writerows([self.seed, region, self.qcut, q, p] + c
                             for q, p, c in zip(query, positions.tolist(), counts.tolist()))
            if coverage_summary is not None:
                region_coverage = float(counts.sum()) / n
                old_coverage = coverage_summary.get('avg_coverage', -1)
                if region_coverage > old_coverage:
                    coverage_summary['avg_coverage'] = region_coverage
                    coverage_summary['coverage_region'] = region
                    coverage_summary['region_width'] = n

    def _create_nuc_writer(self, nuc_file):
        return csv.DictWriter(nuc_file,
                              ['seed',
                               'region',
                               'q-cutoff',
                               'query.nuc.pos',
                               'refseq.nuc.pos',
                               'A',
                               'C',
                               'G',
                               'T'],
                              lineterminator=os.linesep)

    def write_nuc_header(self, nuc_file):
        self._create_nuc_writer(nuc_file).writeheader()

    def write_nuc_counts(self, nuc_file):
        """Nucleotide counts (:451-476)."""
        writer = csv.writer(nuc_file, lineterminator=os.linesep)
        if not self.coordinate_refs:
            n = len(self.seed_aminos[0])       # KeyError without reads, as the reference
            frame = self._frames[0]
            counts = np.zeros((n, 3, 4), dtype=np.int64)
            counts[:frame.ncod] = frame.nt_cnt[:, :, :4]
            rows = []
            for j, codon in enumerate(counts.tolist()):
                for i in range(3):
                    rows.append([self.seed, self.seed, self.qcut, i + 3 * j + 1, ''] + codon[i])
            writer.writerows(rows)
            return
        for region in self.reports:
            frame, index, positions = self._report_index[region]
            counts = self._counts_at(frame, index, lambda fr: fr.nt_cnt[:, :, :4], (3, 4))
            rows = []
            for ci, pos, codon in zip(index.tolist(), positions.tolist(), counts.tolist()):
                for i in range(3):
                    rows.append([self.seed, region, self.qcut, i + 3 * ci + 1 if ci >= 0 else '',
                                 i + 3 * pos - 2] + codon[i])
            writer.writerows(rows)

    def _create_consensus_writer(self, conseq_file):
        return csv.DictWriter(conseq_file,
                              ['region',
                               'q-cutoff',
                               'consensus-percent-cutoff',
                               'offset',
                               'sequence'],
                              lineterminator=os.linesep)

    def write_consensus_header(self, conseq_file):
        self._create_consensus_writer(conseq_file).writeheader()

    def write_consensus(self, conseq_file, min_coverage=100):
        """Nucleotide consensus at each mixture cutoff (:490-522), lower case
        below min_coverage."""
        conseq_writer = self._create_consensus_writer(conseq_file)
        aminos = self.seed_aminos[0]           # KeyError without reads, as the reference
        frame = self._frames[0]
        covered = np.flatnonzero(frame.has[:len(aminos)])
        if not len(covered):
            return
        start = int(covered[0])
        cnt = frame.nt_cnt[start:].reshape(-1, 6)
        first = frame.nt_first[start:].reshape(-1, 6)
        for mixture_cutoff in self.conseq_mixture_cutoffs:
            letters, coverage = _nuc_letters(cnt, first, mixture_cutoff)
            letters = np.where(coverage >= min_coverage, letters, np.char.lower(letters))
            conseq_writer.writerow({
                'region': self.seed,
                'q-cutoff': self.qcut,
                'consensus-percent-cutoff': format_cutoff(mixture_cutoff),
                'offset': start * 3,
                'sequence': ''.join(letters.tolist())
            })

    def _create_nuc_variants_writer(self, nuc_variants_file):
        return csv.DictWriter(nuc_variants_file,
                              ['seed',
                               'qcut',
                               'region',
                               'index',
                               'count',
                               'seq'],
                              lineterminator=os.linesep)

    def write_nuc_variants_header(self, nuc_variants_file):
        self._create_nuc_variants_writer(nuc_variants_file).writeheader()

    def write_nuc_variants(self, nuc_variants_file):
        """:537-549; under Python 3 the reference fails here (dict_keys has
        no sort), and so does this."""
        regions = self.variants.keys()
        regions.sort()

    def _create_failure_writer(self, fail_file):
        return csv.DictWriter(fail_file,
                              ['seed',
                               'region',
                               'qcut',
                               'queryseq',
                               'refseq'],
                              lineterminator=os.linesep)

    def write_failure_header(self, fail_file):
        self._create_failure_writer(fail_file).writeheader()

    def write_failure(self, fail_file):
        """Consensus sequences that did not align to their coordinate
        reference (:563-572)."""
        fail_writer = self._create_failure_writer(fail_file)
        for region, report_aminos in self.reports.items():
            if not report_aminos:
                coordinate_ref = self.projects.getReference(region)
                fail_writer.writerow(dict(seed=self.seed,
                                          region=region,
                                          qcut=self.qcut,
                                          queryseq=self.consensus[region],
                                          refseq=coordinate_ref))

    def write_insertions(self):
        for coordinate_name, coordinate_inserts in self.inserts.items():
            self.insert_writer.write(coordinate_inserts,
                                     coordinate_name,
                                     self.reading_frames[coordinate_name],
                                     self.reports[coordinate_name])


class SeedAmino(object):
    """SeedAmino (:582-626): amino-acid and nucleotide counts of one codon."""

    def __init__(self, consensus_index):
        self.consensus_index = consensus_index
        self.counts = Counter()
        self.nucleotides = [SeedNucleotide() for _ in range(3)]

    def __repr__(self):
        return 'SeedAmino({}): {}'.format(self.consensus_index, self.counts)

    def count_aminos(self, codon_seq, count):
        amino = translate(codon_seq.upper())
        if amino in AMINO_ALPHABET:
            self.counts[amino] += count
        for i in range(3):
            self.nucleotides[i].count_nucleotides(codon_seq[i], count)

    def get_report(self):
        return ','.join([str(self.counts[amino]) for amino in AMINO_ALPHABET])

    def get_consensus(self):
        consensus = self.counts.most_common(1)
        return '-' if not consensus else consensus[0][0]


class SeedNucleotide(object):
    """SeedNucleotide (:628-695): counts of one nucleotide position."""

    def __init__(self):
        self.counts = Counter()

    def count_nucleotides(self, nuc_seq, count):
        if nuc_seq != 'n':     # 'n': the gap between forward and reverse read
            self.counts[nuc_seq] += count

    def get_report(self):
        return ','.join(map(str, [self.counts[nuc] for nuc in 'ACGT']))

    def get_consensus(self, mixture_cutoff):
        if not self.counts:
            return ''
        ranked = self.counts.most_common()
        # gaps and poor quality drop out unless nothing else was read
        kept = [item for item in ranked if item[0] not in ('N', '-')] or ranked[:1]
        total_count = sum(self.counts.values())
        min_count = kept[0][1] if mixture_cutoff == MAX_CUTOFF else total_count * mixture_cutoff
        mixture = sorted(nuc for nuc, count in kept if count >= min_count)
        if len(mixture) > 1:
            return ambig_dict[''.join(mixture)]
        return mixture[0] if mixture else 'N'


class ReportAmino(object):
    def __init__(self, seed_amino, position):
        self.seed_amino = seed_amino
        self.position = position

    def __repr__(self):
        return 'ReportAmino({!r}, {})'.format(self.seed_amino, self.position)


class InsertionWriter(object):
    """InsertionWriter (:711-811).  The read loop of write() runs on the
    device over the group the SequenceReport attached, or over the reads
    given to add_nuc_read."""

    def __init__(self, insert_file):
        self.insert_writer = csv.DictWriter(insert_file,
                                            ['seed',
                                             'region',
                                             'qcut',
                                             'left',
                                             'insert',
                                             'count',
                                             'before'],
                                            lineterminator=os.linesep)
        self.insert_writer.writeheader()
        self._file = insert_file
        self.nuc_seqs = Counter()
        self._source = None

    def start_group(self, seed, qcut):
        self.seed = seed
        self.qcut = qcut
        self.nuc_seqs = Counter()  # {nuc_seq: count}
        self._source = None

    def add_nuc_read(self, offset_sequence, count):
        self.nuc_seqs[offset_sequence] += count

    def _attach(self, ctx, slot, g):
        """The reads of this group are group g of the device table `slot`."""
        self._source = (ctx, slot, g)

    def _insert_counts(self, ranges, reading_frame):
        if self._source is not None:
            ctx, slot, g = self._source
        else:
            if not self.nuc_seqs:
                return []
            ctx, slot, g = session.context(), SLOT_INSERTS, 0
            seqs = list(self.nuc_seqs)
            ctx.a2c_load_rows(slot, seqs, [0] * len(seqs), [self.nuc_seqs[s] for s in seqs],
                              [0, len(seqs)], _CODON_CHARS)
        return ctx.a2c_inserts(slot, g, reading_frame, [r[0] for r in ranges],
                               [r[1] for r in ranges])

    def write(self, inserts, region, reading_frame=0, report_aminos=[]):
        """Insertion ranges with their amino-acid strings and counts
        (:748-811).  Ranges whose rows would be dropped (inserted before
        position 1 or after the end) are not counted."""
        if len(inserts) == 0:
            return
        insert_ranges = []
        for insert in sorted(inserts):
            if not insert_ranges or insert != insert_ranges[-1][1]:
                insert_ranges.append([insert, insert + 1])
            else:
                insert_ranges[-1][1] += 1
        positions = {}
        for report_amino in report_aminos:
            positions.setdefault(report_amino.seed_amino.consensus_index, report_amino.position)
        insert_targets = {left: positions[right] for left, right in insert_ranges
                          if right in positions}
        wanted = [(left, right) for left, right in insert_ranges
                  if not report_aminos or insert_targets.get(left) not in (1, None)]
        if not wanted:
            return
        entries = self._insert_counts(wanted, reading_frame)
        if not entries:
            return
        # DictWriter's row text, built in one pass: the three leading fields
        # through the csv module (quoting), the rest are numbers and amino-acid
        # letters, which never need quotes
        head = io.StringIO()
        csv.writer(head, lineterminator='').writerow([self.seed, region, self.qcut, ''])
        head = head.getvalue()
        tails = {k: (wanted[k][0] + 1, insert_targets.get(wanted[k][0]))
                 for k in range(len(wanted))}
        self._file.write(''.join(
            '{}{},{},{},{}{}'.format(head, tails[k][0], insert_seq, count,
                                     '' if tails[k][1] is None else tails[k][1], os.linesep)
            for k, count, _first, insert_seq in entries))


def format_cutoff(cutoff):
    """ Format the cutoff fraction as a string to use as a name. """
    if cutoff == MAX_CUTOFF:
        return cutoff
    return '{:0.3f}'.format(cutoff)


def _read_all(handle):
    """The rest of an open aligned.csv: the raw bytes of a text file that
    nothing has read from yet (no decode / encode of the whole file), the
    text otherwise."""
    raw = getattr(handle, 'buffer', None)
    if raw is not None:
        try:
            fresh = handle.tell() == 0
        except (OSError, ValueError):
            fresh = False
        if fresh and (handle.encoding or '').lower().replace('-', '') in ('utf8', 'ascii'):
            return raw.read()
    return handle.read()


def aln2counts(aligned_csv,
               nuc_csv,
               amino_csv,
               coord_ins_csv,
               conseq_csv,
               failed_align_csv=None,
               nuc_variants_csv=None,
               callback=None,
               coverage_summary_csv=None,
               json=None):
    """aln2counts.aln2counts (:822-898): the same open files in and out."""
    if json is None:
        projects = project_config.ProjectConfig.loadDefault()
    else:
        projects = project_config.ProjectConfig.loadCustom(json)
    insert_writer = InsertionWriter(coord_ins_csv)
    report = SequenceReport(insert_writer, projects, CONSEQ_MIXTURE_CUTOFFS)
    report.write_nuc_header(nuc_csv)
    report.write_amino_header(amino_csv)
    report.write_consensus_header(conseq_csv)
    if failed_align_csv:
        report.write_failure_header(failed_align_csv)
    if nuc_variants_csv:
        report.write_nuc_variants_header(nuc_variants_csv)
    if coverage_summary_csv is None:
        coverage_summary = None
    else:
        coverage_writer = csv.DictWriter(coverage_summary_csv,
                                         ['avg_coverage',
                                          'coverage_region',
                                          'region_width'],
                                         lineterminator=os.linesep)
        coverage_writer.writeheader()
        coverage_summary = {}
    if callback:
        aligned_filename = getattr(aligned_csv, 'name', None)
        if aligned_filename:
            report.enable_callback(callback, os.stat(aligned_filename).st_size)
    ctx = session.context()
    n_groups = ctx.a2c_load_csv(SLOT_REPORT, _read_all(aligned_csv), _CODON_CHARS)
    for g in range(n_groups):
        report._read_group(ctx, SLOT_REPORT, g)
        report.write_amino_counts(amino_csv, coverage_summary=coverage_summary)
        report.write_consensus(conseq_csv)
        if failed_align_csv:
            report.write_failure(failed_align_csv)
        report.write_insertions()
        report.write_nuc_counts(nuc_csv)
        if nuc_variants_csv:
            report.write_nuc_variants(nuc_variants_csv)
    if coverage_summary_csv is not None:
        if coverage_summary:
            coverage_writer.writerow(coverage_summary)


def parseArgs():
    parser = argparse.ArgumentParser(description='Post-processing of short-read alignments.')
    parser.add_argument('aligned_csv', type=argparse.FileType('r'), help='aligned CSF input')
    parser.add_argument('nuc_csv', type=argparse.FileType('w'),
                        help='CSV containing nucleotide frequencies')
    parser.add_argument('amino_csv', type=argparse.FileType('w'),
                        help='CSV containing amino frequencies')
    parser.add_argument('coord_ins_csv', type=argparse.FileType('w'),
                        help='CSV containing insertions relative to coordinate reference')
    parser.add_argument('conseq_csv', type=argparse.FileType('w'),
                        help='CSV containing consensus sequences')
    parser.add_argument('--failed_align_csv', required=False, type=argparse.FileType('w'),
                        help='CSV containing any consensus that failed to align')
    parser.add_argument('--nuc_variants_csv', required=False, type=argparse.FileType('w'),
                        help='CSV containing top nucleotide variants')
    return parser.parse_args()


def main():
    args = parseArgs()
    aln2counts(args.aligned_csv, args.nuc_csv, args.amino_csv, args.coord_ins_csv,
               args.conseq_csv, args.failed_align_csv, args.nuc_variants_csv)


if __name__ == '__main__':
    main()
