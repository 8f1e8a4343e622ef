"""
Drop-in for micall/core/prelim_map.py: same function, arguments, output file.

prelim_map() maps every read pair end-to-end against every seed reference
of the project file and writes prelim.csv (the SAM columns qname..qual,
rows grouped by rname in first-seen order, prelim_map.py:134-151).  The
bowtie2-build + bowtie2 subprocesses (prelim_map.py:106, :134) are replaced
by the HIP mapper (mh_index_build + mh_map); bt2_path / bt2build_path /
nthreads are accepted for signature compatibility and ignored.
"""
import argparse
import logging
import os
import sys

import numpy as np

from . import _native, session, sharded_io
from .projects import ProjectConfig

# Module constants the reference exports (prelim_map.py:25-33); the bowtie2
# names only describe the command contract the HIP mapper stands in for.
BOWTIE_THREADS, BOWTIE_VERSION = 4, '2.2.8'
BOWTIE_PATH, BOWTIE_BUILD_PATH = 'bowtie2', 'bowtie2-build-s'
READ_GAP_OPEN, READ_GAP_EXTEND = 10, 3      # --rdg
REF_GAP_OPEN, REF_GAP_EXTEND = 10, 3        # --rfg
E2E_SEEDLEN = 22                            # -L of the end-to-end preset
MAXINS = 1200                               # -X

FIELDNAMES = ['qname', 'flag', 'rname', 'pos', 'mapq', 'cigar', 'rnext', 'pnext', 'tlen', 'seq',
              'qual']

logger = logging.getLogger(__name__)


def check_fastq(fastq1, fastq2):
    """prelim_map.py:62-69 / remap.py:415-422: exit(1) on a missing file."""
    for path in (fastq1, fastq2):
        if path is None or os.path.exists(path):
            continue
        logger.error('No FASTQ found at %s', path)
        sys.exit(1)


def grouped_order(sam_ref):
    """Row order of prelim.csv: rows grouped by rname, groups in first-seen
    order, rows in output order within a group (prelim_map.py:137-151)."""
    sam_ref = np.asarray(sam_ref)
    if len(sam_ref) == 0:
        return np.zeros(0, dtype=np.int64)
    values, first = np.unique(sam_ref, return_index=True)
    rank_of_value = np.empty(len(values), dtype=np.int64)
    rank_of_value[np.argsort(first, kind='stable')] = np.arange(len(values))
    ranks = rank_of_value[np.searchsorted(values, sam_ref)]
    return np.argsort(ranks, kind='stable').astype(np.int64)


def prelim_map(fastq1, fastq2, prelim_csv,
               bt2_path='bowtie2', bt2build_path='bowtie2-build-s',
               nthreads=BOWTIE_THREADS, callback=None,
               rdgopen=READ_GAP_OPEN, rfgopen=REF_GAP_OPEN, stderr=sys.stderr,
               gzip=False, work_path='', keep=False, json=None):
    """Run the preliminary mapping step (prelim_map.py:36-161)."""
    check_fastq(fastq1, fastq2)
    rdgopen = READ_GAP_OPEN if rdgopen is None else int(rdgopen)
    rfgopen = REF_GAP_OPEN if rfgopen is None else int(rfgopen)
    ctx = session.load_fastq(fastq1, fastq2)
    sh = session.shard()
    if sh is not None:
        sh.barrier()
    if callback:
        total_reads = ctx.fastq_line_count / 2
        callback(message='... preliminary mapping', progress=0, max_progress=total_reads)
    projects = ProjectConfig.loadDefault() if json is None else ProjectConfig.loadCustom(json)
    seeds = projects.seed_sequences()
    names = list(seeds)
    if keep:
        with open(os.path.join(work_path, 'micall.fasta'), 'w') as ref:
            projects.writeSeedFasta(ref)
    ctx.index_build(names, [seeds[n] for n in names], E2E_SEEDLEN)
    ctx.map(_native.params(_native.E2E, rdg=(rdgopen, READ_GAP_EXTEND),
                           rfg=(rfgopen, REF_GAP_EXTEND), maxins=MAXINS))
    sam_ref = ctx.rec_fields(('sam_ref',))[:, 0]
    header = (','.join(FIELDNAMES) + os.linesep).encode()
    if session.is_writer():
        session.write_bytes(prelim_csv, header)
    out = sharded_io.SharedOutput(sh, prelim_csv)
    order, bounds = grouped_segments(sam_ref, len(names), sh)
    out.write_rows(ctx, 1, order, bounds)
    if sh is not None:
        sh.barrier()            # every rank's rows are in the file
    out.finish()
    session.prelim_written(ctx, prelim_csv, names, out.crc_of_file(header) if out.direct else None)
    if callback:
        callback(progress=ctx.fastq_line_count / 2)


def grouped_segments(sam_ref, n_refs, sh=None):
    """prelim.csv's row order for this rank's records and its segments, one
    per rname group (prelim_map.py:137-151: rows grouped by rname, groups in
    first-seen order, rows in output order within a group).  Sharded, the
    groups are in global first-seen order (the smallest global row index of
    each rname over all ranks, '*' a group of its own) and every rank has
    every group, possibly empty: written segment-major, a group holds the
    rows of rank 0, then rank 1, ... -- the ranks hold consecutive blocks of
    the FASTQ, so that is FASTQ order, as on one GPU."""
    sam_ref = np.asarray(sam_ref)
    # rname ids are small: a stable argsort of int16 keys is numpy's radix sort
    kt = np.int16 if n_refs < np.iinfo(np.int16).max else np.int64
    key = np.where(sam_ref < 0, n_refs, sam_ref).astype(kt)
    by_key = np.argsort(key, kind='stable').astype(np.int64)
    counts = np.bincount(key, minlength=n_refs + 1)
    starts = np.concatenate([[0], np.cumsum(counts)]).astype(np.int64)
    first = np.full(n_refs + 1, -1, dtype=np.int64)
    present = counts > 0
    # a stable sort keeps each key's rows in output order: its first row first
    first[present] = by_key[starts[:-1][present]] + (sh.read_base if sh is not None else 0)
    if sh is not None:
        first = sh.min_i64(first)
    groups = [g for g in np.argsort(np.where(first < 0, np.iinfo(np.int64).max, first),
                                    kind='stable') if first[g] >= 0]
    if len(groups) == 0:
        return np.zeros(0, dtype=np.int64), np.zeros(2, dtype=np.int64)
    order = np.concatenate([by_key[starts[g]:starts[g + 1]] for g in groups]).astype(np.int64)
    bounds = np.concatenate([[0], np.cumsum([counts[g] for g in groups])]).astype(np.int64)
    return order, bounds


_CLI_OPTIONS = (
    ('-fastq1', dict(help='<input> R1 (or unpaired) FASTQ')),
    ('-fastq2', dict(default=None, help='<input, optional> R2 FASTQ of a paired run')),
    ('-prelim_csv', dict(type=argparse.FileType('w'), help='<output> prelim.csv (SAM columns)')),
    ('--rdgopen', dict(default=None, help='<optional> gap open penalty in the read')),
    ('--rfgopen', dict(default=None, help='<optional> gap open penalty in the reference')),
    ('--gzip', dict(action='store_true', help='<optional> the FASTQ files are gzipped')),
    ('--keep', dict(action='store_true', help='<optional> keep the seed FASTA for debugging')),
)


def main():
    parser = argparse.ArgumentParser(
        description='Preliminary end-to-end mapping of a FASTQ pair to the seed references (MI355X).')
    for flag, opts in _CLI_OPTIONS:
        parser.add_argument(flag, **opts)
    args = vars(parser.parse_args())
    prelim_map(**args)


if __name__ == '__main__':
    main()
