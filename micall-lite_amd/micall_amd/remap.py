"""
Drop-in for micall/core/remap.py: remap() with the same arguments, reading
prelim.csv and writing remap.csv (and the optional remap_counts.csv,
remap_conseq.csv and unmapped FASTQ outputs) with the reference's contents.

Per pass, the work the reference does with bowtie2 + Python SAM parsing runs
on the GPU: prelim.csv rows -> device pileup (mh_rows_load_csv, mh_pileup);
each remap pass -> mh_map(--local) over resident reads + mh_pileup; the
consensus-distance filter -> mh_gotoh_align.  Host code keeps the
reference's control flow and every dict order (remap.py:381-658).
"""
import argparse
import csv
import logging
import os
import sys
from collections import Counter

import numpy as np

from . import _native, session
from .consensus import Pileup, counts_to_conseqs
from .pipeline import (CONSENSUS_Q_CUTOFF, MAX_REMAPS, MIN_MAPPING_EFFICIENCY, RemapPipeline,
                       write_remap_counts)
from .prelim_map import (BOWTIE_THREADS, FIELDNAMES, READ_GAP_OPEN, REF_GAP_OPEN, check_fastq)
from .projects import ProjectConfig

logger = logging.getLogger(__name__)

COMPLEMENT = {'A': 'T', 'C': 'G', 'G': 'C', 'T': 'A', 'W': 'S', 'R': 'Y', 'K': 'M', 'Y': 'R',
              'S': 'W', 'M': 'K', 'B': 'V', 'D': 'H', 'H': 'D', 'V': 'B', '*': '*', 'N': 'N',
              '-': '-'}
F = {name: i for i, name in enumerate(_native.ALN_FIELDS)}


def reverse_and_complement(seq):
    """micall/utils/translation.py:36-37."""
    return ''.join(COMPLEMENT[nuc] for nuc in reversed(seq))


def is_first_read(flag):
    return (int(flag) & 0x40) != 0


def is_unmapped_read(flag):
    return (int(flag) & 0x4) != 0


def is_short_read(read_row, max_primer_length):
    """remap.py:70-83."""
    import re
    sizes = re.findall(r'(\d+)M', read_row['cigar'])
    return max(map(int, sizes)) <= max_primer_length


def _sam_fields(ctx, rows):
    """SAM fields of the given resident rows (for the splitter and the
    unmapped FASTQ outputs, which take SEQ/QUAL as printed)."""
    if len(rows) == 0:
        return []
    text = ctx.format_rows(0, order=np.asarray(rows, dtype=np.int64))
    return [line.split('\t') for line in text.split('\n')[:-1]]


def _write_unmapped(ctx, recs, unmapped1, unmapped2):
    """map_to_reference's unmapped FASTQ records (remap.py:743-753)."""
    if not (unmapped1 or unmapped2):
        return
    rows = np.nonzero(recs[:, F['flag']] & 4)[0]
    for fields in _sam_fields(ctx, rows):
        qname, bitflag, seq, qual = fields[0], fields[1], fields[9], fields[10]
        handle = unmapped1 if is_first_read(bitflag) else unmapped2
        if handle:
            handle.write('@%s\n%s\n+\n%s\n' % (qname, seq, qual))


class RemapRun(RemapPipeline):
    """RemapPipeline with the file-level prelim half: the loop starts from
    prelim.csv instead of a device prelim pass."""

    def prelim_from_csv(self, prelim_csv, remap_counts_writer=None, callback=None):
        """remap.py:468-541: prelim rows -> seed selection -> conseqs."""
        conseqs_all = dict(self.seeds)
        refnames = list(conseqs_all)                       # temp.sam @SQ order
        text = prelim_csv.read()
        rows = self.ctx.rows_load_csv(text, refnames)
        info = rows['info']
        refgroups = {}
        # itertools.groupby over rname: runs of equal name ids
        if len(info):
            ids = info[:, 0]
            cut = np.nonzero(np.diff(ids))[0] + 1
            starts = np.concatenate([[0], cut])
            ends = np.concatenate([cut, [len(ids)]])
        else:
            starts = ends = []
        for a, b in zip(starts, ends):
            nid = int(info[a, 0])
            refname = refnames[nid] if nid >= 0 else rows['unknown'][-1 - nid]
            block = info[a:b]
            count = int(b - a)
            mapped = (block[:, 1] & 4) == 0
            filtered_count = int(np.count_nonzero(mapped & (block[:, 2] > 50)))
            if remap_counts_writer is not None:
                remap_counts_writer.writerow(dict(type='prelim %s' % refname, count=count,
                                                  filtered_count=filtered_count))
            if refname == '*':
                continue
            refgroup = self.config.getSeedGroup(refname)
            seed_count_threshold = 1 if refname == 'HIV1B-env-seed' else self.count_threshold
            _best_ref, best_count = refgroups.get(refgroup, (None, seed_count_threshold - 1))
            if filtered_count > best_count:
                refgroups[refgroup] = (refname, filtered_count)
        seed_counts = {best_ref: best_count for best_ref, best_count in refgroups.values()}
        # build_conseqs(temp.sam, seeds=seeds) on the prelim rows (remap.py:531)
        present = [refnames[k] for k in rows['present']]
        self.ctx.pileup(1, CONSENSUS_Q_CUTOFF, [len(conseqs_all[n]) for n in present])
        pile = Pileup(self.ctx.pileup_fetch(), present)
        conseqs = counts_to_conseqs(pile, pile.refs_with_reads(), seeds=self.seeds)
        new_conseqs, map_counts = {}, {}
        for rname, conseq in conseqs.items():
            count = seed_counts.get(rname, None)
            if count is not None:
                map_counts[rname] = count
                new_conseqs[rname] = conseq
        return new_conseqs, map_counts


def remap(fastq1, fastq2, prelim_csv, remap_csv, remap_counts_csv=None,
          remap_conseq_csv=None, unmapped1=None, unmapped2=None, work_path='',
          bt2_path='bowtie2', bt2build_path='bowtie2-build-s',
          nthreads=BOWTIE_THREADS, callback=None, count_threshold=10,
          rdgopen=READ_GAP_OPEN, rfgopen=REF_GAP_OPEN, stderr=sys.stderr,
          gzip=False, debug_file_prefix=None, keep=False, json=None):
    """Iterative re-mapping (remap.py:381-658)."""
    check_fastq(fastq1, fastq2)
    rdgopen = READ_GAP_OPEN if rdgopen is None else int(rdgopen)
    rfgopen = REF_GAP_OPEN if rfgopen is None else int(rfgopen)
    projects = ProjectConfig.loadDefault() if json is None else ProjectConfig.loadCustom(json)
    ctx = session.load_fastq(fastq1, fastq2)
    run = RemapRun(ctx, projects, count_threshold=count_threshold, rdgopen=rdgopen,
                   rfgopen=rfgopen, callback=callback)
    raw_count = ctx.fastq_line_count / 2   # 4 lines per record, paired (remap.py:457)

    remap_counts_writer = None
    if remap_counts_csv:
        remap_counts_writer = csv.DictWriter(
            remap_counts_csv, 'type count filtered_count seed_dist other_dist other_seed'.split(),
            lineterminator=os.linesep)
        remap_counts_writer.writeheader()
        remap_counts_writer.writerow(dict(type='raw', count=raw_count))
    if callback:
        callback(message='... processing preliminary map', progress=0, max_progress=raw_count)

    conseqs, map_counts = run.prelim_from_csv(prelim_csv, remap_counts_writer, callback)

    n_remaps = 0
    new_counts = Counter()
    unmapped_count = raw_count
    mapped_to = None
    while conseqs:
        if callback:
            callback(message='... remap iteration %d' % n_remaps, progress=0)
        if unmapped1:
            unmapped1.seek(0)
            unmapped1.truncate()
        if unmapped2:
            unmapped2.seek(0)
            unmapped2.truncate()
        mapped_to = conseqs
        new_counts, unmapped_count = run.map_to_reference(conseqs)
        _write_unmapped(ctx, ctx.recs(), unmapped1, unmapped2)
        old_seed_names = set(conseqs.keys())
        distance_report = {}
        conseqs = run.build_conseqs_filtered(mapped_to, distance_report)
        new_seed_names = set(conseqs.keys())
        n_remaps += 1
        if remap_counts_writer is not None:
            write_remap_counts(remap_counts_writer, new_counts, title='remap-{}'.format(n_remaps),
                               distance_report=distance_report)
        if new_seed_names == old_seed_names:
            # stopping criterion 1 - none of the regions gained reads
            if all((count <= map_counts[refname]) for refname, count in new_counts.items()):
                break
            # stopping criterion 2 - a sufficient fraction of raw data has been mapped
            mapping_efficiency = sum(new_counts.values()) / float(raw_count)
            if mapping_efficiency > MIN_MAPPING_EFFICIENCY:
                break
            if n_remaps >= MAX_REMAPS:
                break
        map_counts = dict(new_counts)

    # generate SAM CSV output (remap.py:612-634)
    remap_writer = csv.DictWriter(remap_csv, FIELDNAMES, lineterminator=os.linesep)
    remap_writer.writeheader()
    if new_counts:
        recs = ctx.recs()
        keep_rows, splits = split_mixed_references(ctx, recs, run.last_names)
        remap_csv.write(ctx.format_rows(1, order=keep_rows))
        split_counts = Counter()
        for rname, (fwd, rev) in splits.items():
            refseqs = {rname: conseqs[rname]}
            names = []
            seqs, quals = [], []
            for (qname, s1, q1), (_q2, s2, q2) in zip(fwd, rev):
                names += [qname, qname]
                seqs += [s1, s2]
                quals += [q1, q2]
            ctx.reads_load(seqs, quals, True, names=names)
            session.invalidate()
            split_counts.clear()
            cnt, unm = run.map_to_reference(refseqs)
            split_counts.update(cnt)
            unmapped_count += unm
            new_counts.update(split_counts)
            _write_unmapped(ctx, ctx.recs(), unmapped1, unmapped2)
            remap_csv.write(ctx.format_rows(1))

    if remap_conseq_csv:
        remap_conseq_csv.write('region,sequence\n')
        for refname in new_counts.keys():
            # the consensus the reads were mapped to (remap.py:639-643)
            conseq = conseqs.get(refname) or projects.getReference(refname)
            remap_conseq_csv.write('%s,%s\n' % (refname, conseq))

    if remap_counts_writer is not None:
        write_remap_counts(remap_counts_writer, new_counts, title='remap-final')
        remap_counts_writer.writerow(dict(type='unmapped', count=unmapped_count))

    if keep and mapped_to is not None:
        with open(os.path.join(work_path, 'temp.fasta'), 'w') as f:
            for region, conseq in mapped_to.items():
                f.write('>%s\n%s\n' % (region, conseq))


def split_mixed_references(ctx, recs, refnames):
    """MixedReferenceSplitter.split (remap.py:780-828) over the resident
    records: pairs whose mates mapped to different references are taken out
    of remap.csv and assigned to one reference (MAPQ compared as strings,
    then AS); returns (rows to keep, {rname: (fwd reads, rev reads)})."""
    n = len(recs)
    rnext = recs[:, F['rnext']]
    flag = recs[:, F['flag']]
    candidate = (rnext >= 0) & ((flag & 12) == 0)
    keep = np.nonzero(~candidate)[0]
    splits = {}
    rows = np.nonzero(candidate)[0]
    if len(rows) == 0:
        return keep, splits
    fields = dict(zip(rows.tolist(), _sam_fields(ctx, rows)))
    unmatched = {}
    for r in rows.tolist():
        f = fields[r]
        match = unmatched.pop(f[0], None)
        if match is None:
            unmatched[f[0]] = f
            continue
        mapq, match_mapq = f[4], match[4]
        if mapq > match_mapq:
            rname = f[2]
        elif mapq < match_mapq:
            rname = match[2]
        else:
            score = _alignment_score(f)
            match_score = _alignment_score(match)
            rname = f[2] if score > match_score else match[2]
        fwd_list, rev_list = splits.setdefault(rname, ([], []))
        if int(f[1]) & 64:
            fwd_read, rev_read = f, match
        else:
            fwd_read, rev_read = match, f
        fwd_list.append((fwd_read[0], fwd_read[9], fwd_read[10]))
        rev_list.append((rev_read[0], reverse_and_complement(rev_read[9]),
                         ''.join(reversed(rev_read[10]))))
    return keep, splits


def _alignment_score(fields):
    for field in fields[11:]:
        if field.startswith('AS:i:'):
            return int(field[5:])


def parse_args():
    parser = argparse.ArgumentParser(description='Iterative remapping by reference (MI355X).')
    parser.add_argument('fastq1', help='<input> FASTQ containing forward reads')
    parser.add_argument('fastq2', nargs='?', help='<input, optional> FASTQ containing reverse reads')
    parser.add_argument('prelim_csv', type=argparse.FileType('r'),
                        help='<input> CSV containing preliminary map output (modified SAM)')
    parser.add_argument('remap_csv', type=argparse.FileType('w'),
                        help='<output> CSV containing remap output (modified SAM)')
    parser.add_argument('-remap_counts_csv', required=False, type=argparse.FileType('w'))
    parser.add_argument('-remap_conseq_csv', required=False, type=argparse.FileType('w'))
    parser.add_argument('-unmapped1', required=False, type=argparse.FileType('w'))
    parser.add_argument('-unmapped2', required=False, type=argparse.FileType('w'))
    parser.add_argument("--rdgopen", default=None)
    parser.add_argument("--rfgopen", default=None)
    parser.add_argument("--gzip", action='store_true')
    parser.add_argument('--verbose', action='store_true')
    parser.add_argument("--keep", action='store_true')
    return parser.parse_args()


def main():
    args = parse_args()
    remap(fastq1=args.fastq1, fastq2=args.fastq2, prelim_csv=args.prelim_csv,
          remap_csv=args.remap_csv, remap_counts_csv=args.remap_counts_csv,
          remap_conseq_csv=args.remap_conseq_csv, unmapped1=args.unmapped1,
          unmapped2=args.unmapped2, gzip=args.gzip, keep=args.keep)


if __name__ == '__main__':
    main()
