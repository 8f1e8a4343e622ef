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
"""
import csv
import os

from . import session


def censor(src, bad_cycles_reader, dest, use_gzip=True, summary_file=None):
    """censor_fastq.censor: src / dest binary file objects (text StringIO
    objects are accepted too and get text back)."""
    bad_cycles = set()
    for cycle in bad_cycles_reader:
        bad_cycles.add((cycle['tile'], int(cycle['cycle'])))
    data = src.read()
    text_mode = isinstance(data, str)
    if text_mode:
        data = data.encode('utf-8')
    out, base_count, score_sum = session.context().censor_fastq(
        data, sorted(bad_cycles), src_gzip=use_gzip, dst_gzip=use_gzip)
    dest.write(out.decode('utf-8') if text_mode else out)
    if summary_file is not None:
        avg_quality = float(score_sum) / base_count if base_count > 0 else None
        writer = csv.DictWriter(summary_file, ['avg_quality', 'base_count'],
                                lineterminator=os.linesep)
        writer.writeheader()
        writer.writerow(dict(base_count=base_count, avg_quality=avg_quality))
