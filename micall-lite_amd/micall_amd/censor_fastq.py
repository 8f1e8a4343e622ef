"""
Drop-in for micall/core/censor_fastq.py:32-102 (censor): same function,
arguments and output.  The per-base Python loop of the reference runs on the
device (mh_censor_fastq, csrc/mh_censor.hip): bases and qualities read in a
bad (tile, cycle) become 'N' / '#', a trailing run of bad cycles is dropped as
the reference drops it, header and '+' lines are copied verbatim.  gzip in
and out as the reference's use_gzip (the output is gzip members compressed
in parallel at level 1: same decompressed bytes, different compressed bytes
than GzipFile's level 9 -- whose header holds a timestamp anyway).  There is
no CPU fallback.

In a sharded job (bin/micall under torchrun: every rank calls censor() with
its own handles on the same files) each rank censors its own block of
records: it reads its share of the source (sharded_io.stage_fastq, strict
four-line records as the reference's zip_longest over lines, :58), censors
it, and writes its gzip members at its offset of the destination, so the
destination is one multi-member gzip stream holding the records in file
order.  The base count and quality sum are summed over the ranks.
"""
import csv
import os

from . import session, sharded_io
from .sharded_io import _binary_fd


def _is_gzip_file(fd):
    try:
        return os.pread(fd, 2, 0) == b'\x1f\x8b'
    except OSError:
        return False


def censor(src, bad_cycles_reader, dest, use_gzip=True, summary_file=None):
    """censor_fastq.censor: src / dest binary file objects (text StringIO
    objects are accepted too and get text back)."""
    bad_cycles = set()
    for cycle in bad_cycles_reader:
        bad_cycles.add((cycle['tile'], int(cycle['cycle'])))
    sh = session.shard()
    if sh is not None:
        sh.barrier()     # every rank has opened (truncated) dest
        fd = _binary_fd(src)
        ok = (fd is not None and _binary_fd(dest) is not None and
              _is_gzip_file(fd) == bool(use_gzip))
        if bool(sh.min_i64([1 if ok else 0])[0]):
            base_count, score_sum = _censor_block(sh, fd, sorted(bad_cycles), dest, use_gzip)
        else:            # rank 0 censors the whole file, the others wait
            base_count = score_sum = 0
            if sh.rank == 0:
                base_count, score_sum = _censor_whole(src, sorted(bad_cycles), dest, use_gzip)
            base_count, score_sum = (int(x) for x in sh.sum_i64([base_count, score_sum]))
        sh.barrier()     # dest is complete on every rank
    else:
        base_count, score_sum = _censor_whole(src, sorted(bad_cycles), dest, use_gzip)
    if summary_file is not None and session.is_writer():
        avg_quality = float(score_sum) / base_count if base_count > 0 else None
        writer = csv.DictWriter(summary_file, ['avg_quality', 'base_count'],
                                lineterminator=os.linesep)
        writer.writeheader()
        writer.writerow(dict(base_count=base_count, avg_quality=avg_quality))


def _censor_whole(src, bad_cycles, dest, use_gzip):
    """The whole file by one process: straight from the source file to the
    destination file when both are plain binary files (the source mmap'd
    and its gzip members inflated in parallel, the output written with
    pwrite at dest's position), else through bytes."""
    import io
    from . import _native
    plain = isinstance(src, (io.BufferedReader, io.FileIO)) and isinstance(dest, (io.BufferedWriter,
                                                                                   io.BufferedRandom,
                                                                                   io.FileIO))
    fd = _binary_fd(src) if plain else None
    out_fd = _binary_fd(dest) if plain else None
    if (fd is not None and out_fd is not None and src.tell() == 0 and
            _is_gzip_file(fd) == bool(use_gzip)):
        ctx = session.context()
        fq = _native.Fastq(fd=fd)
        shared = sharded_io.SharedOutput(None, dest, binary=True)
        try:
            # each gzip member written as soon as it is made
            n, base_count, score_sum = ctx.censor_staged_write(fq, bad_cycles, use_gzip, out_fd,
                                                               int(shared.end))
        finally:
            fq.close()
        shared.end += n
        shared.finish()
        return base_count, score_sum
    data = src.read()
    text_mode = isinstance(data, str)
    if text_mode:
        data = data.encode('utf-8')
    out, base_count, score_sum = session.context().censor_fastq(
        data, bad_cycles, src_gzip=use_gzip, dst_gzip=use_gzip)
    dest.write(out.decode('utf-8') if text_mode else out)
    dest.flush()
    return base_count, score_sum


def _censor_block(sh, fd, bad_cycles, dest, use_gzip):
    """This rank's block of records, censored and written at its offset."""
    st = sharded_io.stage_fastq(sh, [(None, fd)], strict=True)
    fq = st['frames'][0].fq
    ctx = session.context()
    try:
        n, base_count, score_sum = ctx.censor_staged(fq, bad_cycles, use_gzip)
    finally:
        fq.close()
    if sh.rank == 0:
        dest.flush()
    shared = sharded_io.SharedOutput(sh, dest, binary=True)
    if shared.direct:
        off = int(shared.place([n])[0])
        ctx.censor_write(shared.fd, off)
    else:
        shared.write_bytes([ctx.censor_output()])
    shared.finish()
    sums = sh.sum_i64([base_count, score_sum])
    return int(sums[0]), int(sums[1])
