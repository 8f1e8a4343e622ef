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
"""
import argparse

from . import session

SAM2ALN_Q_CUTOFFS = [15]  # sam2aln.py:24
MAX_PROP_N = 0.5          # sam2aln.py:25


def sam2aln(remap_csv, aligned_csv, insert_csv=None, failed_csv=None, nthreads=None):
    """sam2aln.sam2aln (sam2aln.py:395-478).  In a sharded job rank 0
    computes and writes while the other ranks wait (session.writer_stage)."""
    if len(SAM2ALN_Q_CUTOFFS) != 1:
        raise NotImplementedError('the device merge takes one q-cutoff per pass')
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
