"""
Drop-in for micall/core/sam2aln.py: same function, arguments and output files.

sam2aln() reads remap.csv, pairs rows by qname, merges each pair into one
sequence in consensus coordinates (apply_cigar + merge_pairs at q-cutoff 15),
drops pairs with more than half of their bases censored, and writes the
distinct merged sequences with their counts per reference (aligned.csv), the
insertions the merge removed (insert.csv) and the pairs that failed
(failed.csv) -- sam2aln.py:395-478.  The per-pair work and the count of
identical sequences run on the device (mh_sam2aln_csv, mh_sam2aln.hip); the
host parses the CSV and writes the text.  nthreads is accepted for signature
compatibility and ignored.  There is no CPU fallback.

In a sharded job (torchrun) every rank takes its share of remap.csv's rows,
merges its pairs on its GPU, and writes its own insert.csv / failed.csv rows
and its piece of aligned.csv at all-gathered offsets; the distinct merged
sequences are counted by hash owner and sorted across the ranks by a sample
sort (_sam2aln_sharded, mh_s2a_shard.cpp) -- the reference's own pool splits
parse_sam over pairs the same way (sam2aln.py:411-424).
"""
import argparse

import numpy as np

from . import session

SAM2ALN_Q_CUTOFFS = [15]  # sam2aln.py:24
MAX_PROP_N = 0.5          # sam2aln.py:25


SHARD_STATS = {}   # how the last sharded call ran (tests): mode, rows parsed


def sam2aln(remap_csv, aligned_csv, insert_csv=None, failed_csv=None, nthreads=None):
    """sam2aln.sam2aln (sam2aln.py:395-478).  In a sharded job every rank
    does its share (_sam2aln_sharded); when remap.csv cannot be split that
    way, rank 0 computes and writes while the other ranks wait
    (session.writer_stage)."""
    if len(SAM2ALN_Q_CUTOFFS) != 1:
        raise NotImplementedError('the device merge takes one q-cutoff per pass')
    sh = session.shard()
    SHARD_STATS.clear()
    if sh is not None and _sam2aln_sharded(sh, remap_csv, aligned_csv, insert_csv, failed_csv):
        return
    with session.writer_stage(aligned_csv, insert_csv, failed_csv) as stage:
        if not stage.active:
            return
        ctx = session.context()
        fd = session.readable_fd(remap_csv)
        done = None
        if fd is not None:   # the file mmap'd by the library (no '\r' in it)
            done = ctx.sam2aln_file(fd, q_cutoff=SAM2ALN_Q_CUTOFFS[0], max_prop_n=MAX_PROP_N)
            if done is not None:
                remap_csv.seek(0, 2)     # consumed, as the reference's DictReader leaves it
        if done is None:
            text = session.read_text(remap_csv)
            ctx.sam2aln_csv(text, q_cutoff=SAM2ALN_Q_CUTOFFS[0], max_prop_n=MAX_PROP_N)
        for which, handle in (('insert', insert_csv), ('failed', failed_csv), ('aligned', aligned_csv)):
            if handle:
                _write_output(ctx, which, handle)


SAMPLES_PER_NAME = 64   # sample records per reference and rank for the splitters


def _sam2aln_sharded(sh, remap_csv, aligned_csv, insert_csv, failed_csv):
    """This rank's share of sam2aln.  False (on every rank, before any
    output is written) when the job must fall back to rank 0 alone: a
    remap.csv that is not a plain file on every rank, one with quoted fields
    or '\r', or a qname whose rows sit on two ranks."""
    from . import sharded_io
    from .sharded_io import SharedOutput, _agree_ok, _checked
    ctx = session.context()
    fd = session.readable_fd(remap_csv)
    if not _agree_ok(sh, fd is not None):
        return False
    sh.barrier()             # every rank opened (truncated) the outputs
    part = _checked(sh, lambda: ctx.sam2aln_part(fd, sh.rank, sh.world, SAM2ALN_Q_CUTOFFS[0],
                                                  MAX_PROP_N))
    if not _agree_ok(sh, part is not None):
        return False
    hashes, leftover = ctx.sam2aln_part_units(part['units'])
    if sharded_io.qname_conflict(sh, hashes, leftover):
        return False
    remap_csv.seek(0, 2)     # consumed, as the reference's DictReader leaves it
    SHARD_STATS.update(mode='sharded', bytes=part['bytes'], file_bytes=part['file_bytes'],
                       units=part['units'])
    # reference names in the reference's first-seen order over the job's
    # units: every rank's pair units in rank order, then every rank's leftovers
    names, first = ctx.sam2aln_part_names(part['names'])
    texts = sh.all_gather_bytes('\n'.join(names).encode())
    firsts = sh.all_gather_bytes(np.asarray(first, dtype=np.int64).tobytes())
    pairs = sh._gather_sizes([part['pair_units']])[:, 0]
    key = {}
    for r in range(sh.world):
        rn = texts[r].decode().split('\n') if texts[r] else []
        fu = np.frombuffer(firsts[r], dtype=np.int64)
        for n, u in zip(rn, fu.tolist()):
            k = (0, r, u) if u < pairs[r] else (1, r, u)
            if n not in key or k < key[n]:
                key[n] = k
    order = sorted(key, key=key.get)
    gid = {n: i for i, n in enumerate(order)}
    ctx.sam2aln_part_set_names([gid[n] for n in names])
    # aligned.csv: distinct sequences counted by their owner, then sorted
    # across the ranks (sample sort) and written piece by piece
    data, sizes = ctx.sam2aln_records(0, sh.world)
    got = sharded_io.all_to_all_bytes(sh, data, sizes)
    ctx.sam2aln_records_merge(0, got)
    del got
    samples, _ = ctx.sam2aln_records(1, sh.world, SAMPLES_PER_NAME)
    ctx.sam2aln_splitters(np.frombuffer(b''.join(sh.all_gather_bytes(samples.tobytes())), dtype=np.uint8),
                          sh.world)
    data, sizes = ctx.sam2aln_records(2, sh.world)
    got = sharded_io.all_to_all_bytes(sh, data, sizes)
    ctx.sam2aln_records_merge(1, got)
    del got
    counts = sh._gather_sizes(ctx.sam2aln_range_counts(len(order)))     # [rank, name]
    base = counts[:sh.rank].sum(axis=0)
    rows, seg = ctx.sam2aln_range_text(order, base)
    head = b'refname,qcut,rank,count,offset,seq\n' if sh.rank == 0 else b''
    pieces, at = [head], 0
    for n in seg.tolist():
        pieces.append(rows[at:at + n])
        at += n
    out = SharedOutput(sh, aligned_csv)
    out.write_bytes(pieces)
    del rows
    for which, handle in (('insert', insert_csv), ('failed', failed_csv)):
        if handle:
            segs = [ctx.sam2aln_part_text(which, 0, head=sh.rank == 0), ctx.sam2aln_part_text(which, 1)]
            o = SharedOutput(sh, handle)
            o.write_bytes(segs)
            o.finish()
    out.finish()
    sh.barrier()             # every rank's rows are in the files
    for h in (aligned_csv, insert_csv, failed_csv):
        if h and sh.rank == 0:
            h.flush()
    return True


def _write_output(ctx, which, handle):
    """One output: written by the library at the handle's position when it is
    a plain file (pwrite), else through the handle."""
    from .sharded_io import SharedOutput
    out = SharedOutput(None, handle)
    if out.direct:
        # formatted and written together (pwrite from the handle's position)
        out.end += ctx.sam2aln_write(which, out.fd, int(out.end))
        out.finish()
    else:
        handle.write(ctx.sam2aln_output(which))


def parseArgs():
    parser = argparse.ArgumentParser(description='Conversion of SAM data into aligned format.')
    parser.add_argument('remap_csv', type=argparse.FileType('r'),
                        help='<input> SAM output of bowtie2 in CSV format')
    parser.add_argument('aligned_csv', type=argparse.FileType('w'),
                        help='<output> CSV containing cleaned and merged reads')
    parser.add_argument('insert_csv', nargs='?', default=None, type=argparse.FileType('w'),
                        help='<output> CSV containing insertions relative to sample consensus')
    parser.add_argument('failed_csv', nargs='?', default=None, type=argparse.FileType('w'),
                        help='<output> CSV containing reads that failed to merge')
    parser.add_argument('-p', type=int, default=None, help='(optional) number of threads')
    return parser.parse_args()


def main():
    args = parseArgs()
    sam2aln(remap_csv=args.remap_csv, aligned_csv=args.aligned_csv, insert_csv=args.insert_csv,
            failed_csv=args.failed_csv, nthreads=args.p)


if __name__ == '__main__':
    main()
