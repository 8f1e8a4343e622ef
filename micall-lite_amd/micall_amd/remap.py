"""
remap stage on the MI355X: the drop-in for micall/core/remap.py's remap().

Same arguments and the same files: remap.csv, and the optional
remap_counts.csv, remap_conseq.csv and unmapped FASTQs, byte-identical to the
reference's on the same input (tests/test_gpu_e2e.py).

Where the reference shells out to bowtie2 and parses SAM text in Python on
every pass, this module drives the device:
  prelim.csv          -> mh_rows_load_csv (parse + matchmaker) and a device
                         pileup of those rows (mh_pileup, source 1)
  each --local pass   -> mh_map over the reads resident in HBM + mh_pileup
                         (RemapPipeline.iterate, the one remap loop)
  distance filter     -> mh_gotoh_align + mh_levenshtein
  mixed-reference     -> split_mixed_references over the device records,
  pairs                  then one more device pass per chosen reference
Every dict order the reference's outputs depend on is reproduced
(remap.py:381-658).
"""
import argparse
import csv
import logging
import os
import re
import sys

import numpy as np

from . import _native, session, sharded_io
from .consensus import Pileup, counts_to_conseqs
from .pipeline import CONSENSUS_Q_CUTOFF, RemapPipeline, write_remap_counts
from .prelim_map import BOWTIE_THREADS, FIELDNAMES, READ_GAP_OPEN, REF_GAP_OPEN, check_fastq
from .projects import ProjectConfig

logger = logging.getLogger(__name__)

REMAP_COUNT_COLUMNS = ['type', 'count', 'filtered_count', 'seed_dist', 'other_dist', 'other_seed']
_IUPAC, _PAIRED = 'ACGTWRKYSMBDHVN*-', 'TGCASYMRWKVHDBN*-'
_PAIRING = str.maketrans(_IUPAC, _PAIRED)
F = {name: i for i, name in enumerate(_native.ALN_FIELDS)}
_FIRST, _UNMAPPED, _MATE_UNMAPPED = 0x40, 0x4, 0x8


def reverse_and_complement(seq):
    """Reverse complement over the IUPAC alphabet (translation.py:36-37);
    a letter outside it raises KeyError as there."""
    unknown = set(seq).difference(_IUPAC)
    if unknown:
        raise KeyError(min(unknown))
    return seq[::-1].translate(_PAIRING)


def is_first_read(flag):
    return bool(int(flag) & _FIRST)


def is_unmapped_read(flag):
    return bool(int(flag) & _UNMAPPED)


def is_short_read(read_row, max_primer_length):
    """True when no M run of the row's CIGAR is longer than
    max_primer_length (remap.py:70-83)."""
    return max(int(n) for n in re.findall(r'(\d+)M', read_row['cigar'])) <= max_primer_length


def _sam_fields(ctx, rows):
    """SAM fields (as printed) of the given resident records."""
    if len(rows) == 0:
        return []
    text = ctx.format_rows(0, order=np.asarray(rows, dtype=np.int64))
    return [line.split('\t') for line in text.split('\n')[:-1]]


def _flags(ctx):
    """(flag, rnext) of the resident records (one strided copy of three
    adjacent fields, not the whole records)."""
    a = ctx.rec_fields(('flag', 'mapq', 'rnext'))
    return a[:, 0], a[:, 2]


def _unmapped_text(ctx):
    """FASTQ text of the unmapped lines of the last pass, R1 and R2 apart
    (remap.py:743-753)."""
    out = ([], [])
    for fields in _sam_fields(ctx, np.nonzero(_flags(ctx)[0] & _UNMAPPED)[0]):
        out[0 if is_first_read(fields[1]) else 1].append('@{0[0]}\n{0[9]}\n+\n{0[10]}\n'.format(fields))
    return ''.join(out[0]).encode(), ''.join(out[1]).encode()


def _write_unmapped(ctx, outs):
    """Append the last pass's unmapped reads to the unmapped FASTQs (every
    rank's, in rank order, in a sharded run).  outs: the SharedOutput of
    unmapped1 and unmapped2 (None where not requested)."""
    if not any(outs):
        return
    texts = _unmapped_text(ctx)
    for out, text in zip(outs, texts):
        if out is not None:
            out.write_bytes([text])


class RemapRun(RemapPipeline):
    """RemapPipeline whose prelim half comes from prelim.csv (the file
    bin/micall hands over) instead of a device prelim pass."""

    def prelim_from_csv(self, prelim_csv, remap_counts_writer=None, callback=None):
        """prelim rows -> per-rname tallies -> seed-group winners -> their
        consensus sequences (remap.py:468-541)."""
        region_seqs = dict(self.seeds)
        refnames = list(region_seqs)                      # temp.sam @SQ order
        rows = self.ctx.rows_load_csv(session.read_text(prelim_csv), refnames)
        info = rows['info']
        groups = []
        if len(info):
            # consecutive rows with one rname id form a group (groupby)
            bounds = np.flatnonzero(np.diff(info[:, 0])) + 1
            for block in np.split(info, bounds):
                nid = int(block[0, 0])
                name = refnames[nid] if nid >= 0 else rows['unknown'][-1 - nid]
                mapped = (block[:, 1] & _UNMAPPED) == 0
                groups.append((name, len(block), int(np.count_nonzero(mapped & (block[:, 2] > 50)))))
        if remap_counts_writer is not None:
            remap_counts_writer.writerows(dict(type='prelim %s' % name, count=count,
                                               filtered_count=filt)
                                          for name, count, filt in groups)
        winners = self.select_seeds(groups)
        # build_conseqs(temp.sam, seeds=seeds) over the prelim rows (remap.py:531)
        present = [refnames[k] for k in rows['present']]
        # every rank of a sharded run parses all of prelim.csv, so this
        # pileup is already global: no exchange
        self.ctx.pileup(1, CONSENSUS_Q_CUTOFF, [len(region_seqs[n]) for n in present])
        pile = Pileup(self.ctx.pileup_fetch(), present)
        built = counts_to_conseqs(pile, pile.refs_with_reads(), seeds=self.seeds)
        chosen = {name: seq for name, seq in built.items() if name in winners}
        return chosen, {name: winners[name] for name in chosen}

    def prelim_from_device(self, remap_counts_writer=None):
        """The same as prelim_from_csv when prelim.csv is the file this
        process's prelim_map() wrote from the records still resident
        (session.prelim_resident): the per-rname tallies and the pileup come
        from those records (all-reduced over the ranks of a sharded run).
        prelim.csv groups rows by rname in first-seen order, so its groups,
        and the order in which its pairs reach each reference, follow the
        tallies' first rows.  Skips the parse of a GB-sized text."""
        self.prelim_names = list(self.seed_set)
        self.prelim_stats = self._counts()
        groups = self.prelim_groups()
        if remap_counts_writer is not None:
            remap_counts_writer.writerows(dict(type='prelim %s' % name, count=count,
                                               filtered_count=filt)
                                          for name, count, filt in groups)
        return self.prelim_conseqs(self.select_seeds(groups))


class MixedReferenceSplit(object):
    """Pairs whose mates mapped to different references
    (MixedReferenceSplitter.split, remap.py:780-828): such a pair leaves
    remap.csv and is assigned to one reference -- the mate with the higher
    MAPQ wins, MAPQ compared as strings ('8' > '44'), then the higher AS:i --
    to be mapped again against that reference alone.

    feed(fields) takes one SAM line's fields and returns True when the line
    stays in remap.csv.  `splits` maps a reference to its (R1 reads, R2
    reads) as (qname, seq, qual); the mate flagged 0x40 of the second line
    seen decides which read is R1, and R2 is reverse-complemented back, as
    the reference writes its split FASTQs.  A mate whose partner never
    comes is dropped."""

    def __init__(self):
        self.splits = {}
        self._waiting = {}

    @staticmethod
    def passes(fields):
        return fields[6] in ('=', '*') or bool(int(fields[1]) & (_UNMAPPED | _MATE_UNMAPPED))

    @staticmethod
    def _score(fields):
        for tag in fields[11:]:
            if tag.startswith('AS:i:'):
                return int(tag[5:])
        return None

    def _winner(self, a, b):
        """Reference of the pair (a: this line, b: its mate seen earlier)."""
        if a[4] != b[4]:
            return a[2] if a[4] > b[4] else b[2]
        return a[2] if self._score(a) > self._score(b) else b[2]

    def feed(self, fields):
        if self.passes(fields):
            return True
        mate = self._waiting.pop(fields[0], None)
        if mate is None:
            self._waiting[fields[0]] = fields
            return False
        r1, r2 = (fields, mate) if int(fields[1]) & _FIRST else (mate, fields)
        reads1, reads2 = self.splits.setdefault(self._winner(fields, mate), ([], []))
        reads1.append((r1[0], r1[9], r1[10]))
        reads2.append((r2[0], reverse_and_complement(r2[9]), r2[10][::-1]))
        return False


def split_mixed_references(ctx):
    """MixedReferenceSplit over the resident records of the last pass:
    returns (record indices that stay in remap.csv -- None when that is every
    record --, splits).  Only records whose RNEXT names another reference
    with both mates mapped are turned into text; every other record passes."""
    flag, rnext = _flags(ctx)
    candidate = (rnext >= 0) & ((flag & (_UNMAPPED | _MATE_UNMAPPED)) == 0)
    rows = np.flatnonzero(candidate)
    if len(rows) == 0:
        return None, {}
    split = MixedReferenceSplit()
    for fields in _sam_fields(ctx, rows):
        split.feed(fields)      # never passes: RNEXT is a name, both mates mapped
    return np.flatnonzero(~candidate), split.splits


def remap(fastq1, fastq2, prelim_csv, remap_csv, remap_counts_csv=None, remap_conseq_csv=None,
          unmapped1=None, unmapped2=None, work_path='', bt2_path='bowtie2',
          bt2build_path='bowtie2-build-s', nthreads=BOWTIE_THREADS, callback=None,
          count_threshold=10, rdgopen=READ_GAP_OPEN, rfgopen=REF_GAP_OPEN, stderr=sys.stderr,
          gzip=False, debug_file_prefix=None, keep=False, json=None):
    """Iterative re-mapping against the sample's own consensus sequences
    (remap.py:381-658).  bt2_path, bt2build_path, nthreads, stderr, gzip and
    debug_file_prefix are accepted for the signature and not used; keep
    writes the last consensus FASTA (there are no other temp files)."""
    check_fastq(fastq1, fastq2)
    rdgopen = READ_GAP_OPEN if rdgopen is None else int(rdgopen)
    rfgopen = REF_GAP_OPEN if rfgopen is None else int(rfgopen)
    projects = ProjectConfig.loadDefault() if json is None else ProjectConfig.loadCustom(json)
    ctx = session.load_fastq(fastq1, fastq2)
    sh = session.shard()
    if sh is not None:
        sh.barrier()
    writer = session.is_writer()
    run = RemapRun(ctx, projects, count_threshold=count_threshold, rdgopen=rdgopen,
                   rfgopen=rfgopen, callback=callback, shard=sh)
    # bowtie2's input lines / 2, also for unpaired input (remap.py:457)
    raw_count = ctx.fastq_line_count / 2

    counts_out = None
    if remap_counts_csv and writer:
        counts_out = csv.DictWriter(remap_counts_csv, REMAP_COUNT_COLUMNS,
                                    lineterminator=os.linesep)
        counts_out.writeheader()
        counts_out.writerow(dict(type='raw', count=raw_count))
    if callback:
        callback(message='... processing preliminary map', progress=0, max_progress=raw_count)

    if session.prelim_resident(ctx, prelim_csv, run.seed_set):
        session.stats['prelim_source'] = 'device'
        conseqs, map_counts = run.prelim_from_device(counts_out)
    else:
        session.stats['prelim_source'] = 'csv'
        conseqs, map_counts = run.prelim_from_csv(prelim_csv, counts_out, callback)

    # Each pass rewrites the unmapped FASTQs (remap.py:552-558), so they hold
    # the unmapped reads of the last pass: written once, after the loop.
    for handle in (unmapped1, unmapped2):
        if handle and writer and conseqs:
            handle.seek(0)
            handle.truncate()
    conseqs, new_counts, unmapped_count = run.iterate(conseqs, map_counts, raw_count,
                                                      remap_counts_writer=counts_out)
    if writer:
        csv.DictWriter(remap_csv, FIELDNAMES, lineterminator=os.linesep).writeheader()
    # every rank writes its own rows / reads (sharded_io.SharedOutput)
    rows_out = sharded_io.SharedOutput(sh, remap_csv)
    unmapped_outs = [sharded_io.SharedOutput(sh, h) if h else None for h in (unmapped1, unmapped2)]
    if run.mapped_to is not None:
        _write_unmapped(ctx, unmapped_outs)
    if new_counts:
        unmapped_count += _write_remap_rows(ctx, run, conseqs, new_counts, rows_out,
                                            unmapped_outs, sh)
    if sh is not None:
        sh.barrier()            # every rank's rows are in the files
    for out in [rows_out] + unmapped_outs:
        if out is not None:
            out.finish()

    if remap_conseq_csv and writer:
        # the sequences the reads were last mapped to (remap.py:637-643)
        remap_conseq_csv.write('region,sequence\n')
        remap_conseq_csv.writelines('%s,%s\n' % (name, conseqs.get(name) or
                                                 projects.getReference(name))
                                    for name in new_counts)
    if counts_out is not None:
        _write_final_counts(counts_out, new_counts, unmapped_count)
    last = getattr(run, 'last_refseqs', None)
    if keep and writer and run.mapped_to is not None and last is not None:
        # the reference set of the last map_to_reference call, a split
        # re-mapping's single reference included (remap.py:624-630, 689-692)
        with open(os.path.join(work_path, 'temp.fasta'), 'w') as f:
            f.writelines('>%s\n%s\n' % item for item in last.items())


def _write_final_counts(writer, new_counts, unmapped_count):
    write_remap_counts(writer, new_counts, title='remap-final')
    writer.writerow(dict(type='unmapped', count=unmapped_count))


def _write_remap_rows(ctx, run, conseqs, new_counts, rows_out, unmapped_outs, shard=None):
    """remap.csv rows of the last pass, then the mixed-reference pairs mapped
    again, one reference at a time (remap.py:612-634).  new_counts gains
    each re-mapping's counts; returns the unmapped lines they add.

    Sharded: mates are resident on one rank, so every rank splits its own
    pairs; the references are re-mapped in their global order of first
    split (rank order, then each rank's order), every rank taking part in
    each one (with its own split pairs, possibly none), and the rows and
    unmapped reads land in rank order."""
    keep_rows, splits = split_mixed_references(ctx)
    n_keep = ctx.reads_count()[0] if keep_rows is None else len(keep_rows)
    rows_out.write_rows(ctx, 1, keep_rows, [0, n_keep])
    order = list(splits)
    if shard is not None:
        order = []
        for text in shard.all_gather_bytes('\n'.join(splits).encode()):
            for name in text.decode().split('\n') if text else []:
                if name not in order:
                    order.append(name)
    extra_unmapped = 0
    for name in order:
        reads1, reads2 = splits.get(name, ([], []))
        names, seqs, quals = [], [], []
        for a, b in zip(reads1, reads2):
            names += [a[0], a[0]]
            seqs += [a[1], b[1]]
            quals += [a[2], b[2]]
        ctx.reads_load(seqs, quals, True, names=names)
        session.invalidate()                 # the FASTQ reads are no longer resident
        counts, unmapped = run.map_to_reference({name: conseqs[name]})
        extra_unmapped += unmapped
        new_counts.update(counts)
        _write_unmapped(ctx, unmapped_outs)
        rows_out.write_rows(ctx, 1, None, [0, len(seqs)])
    return extra_unmapped


def parse_args():
    cli = argparse.ArgumentParser(description='Iterative remapping against sample consensus '
                                              'sequences (MI355X).')
    cli.add_argument('fastq1', help='R1 (or unpaired) FASTQ')
    cli.add_argument('fastq2', nargs='?', help='R2 FASTQ, if paired')
    cli.add_argument('prelim_csv', type=argparse.FileType('r'), help='prelim.csv from prelim_map')
    cli.add_argument('remap_csv', type=argparse.FileType('w'), help='remap.csv to write')
    for name in ('-remap_counts_csv', '-remap_conseq_csv', '-unmapped1', '-unmapped2'):
        cli.add_argument(name, required=False, type=argparse.FileType('w'))
    cli.add_argument('--rdgopen', default=None)
    cli.add_argument('--rfgopen', default=None)
    for flag in ('--gzip', '--verbose', '--keep'):
        cli.add_argument(flag, action='store_true')
    return cli.parse_args()


def main():
    a = parse_args()
    remap(fastq1=a.fastq1, fastq2=a.fastq2, prelim_csv=a.prelim_csv, remap_csv=a.remap_csv,
          remap_counts_csv=a.remap_counts_csv, remap_conseq_csv=a.remap_conseq_csv,
          unmapped1=a.unmapped1, unmapped2=a.unmapped2, gzip=a.gzip, keep=a.keep)


if __name__ == '__main__':
    main()
