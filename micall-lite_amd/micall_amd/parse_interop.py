"""
Host-side mirror of micall/core/parse_interop.py: the Illumina InterOp
ErrorMetricsOut.bin reader and the phiX error-rate CSV writer that feed the
censor stage (bin/micall:101-106).  Byte parsing of a few kB; no device work.

    read_records    parse_interop.py:13-38
    read_errors     parse_interop.py:41-69
    write_phix_csv  parse_interop.py:72-139 (with _yield_cycles, :72-91)
"""
import csv
import math
import os
import sys
from itertools import groupby
from struct import unpack


def read_records(data_file, min_version):
    """Fixed-length records after a (version, record length) header byte pair."""
    version, record_length = unpack('!BB', data_file.read(2))
    if version < min_version:
        raise IOError('File version {} is less than minimum version {} in {}.'.format(
            version, min_version, data_file.name))
    while True:
        data = data_file.read(record_length)
        if not data:
            return
        if len(data) < record_length:
            raise IOError('Partial record of length {} found in {}.'.format(len(data),
                                                                           data_file.name))
        yield data


_ERROR_FIELDS = ('lane', 'tile', 'cycle', 'error_rate', 'num_0_errors', 'num_1_error',
                 'num_2_errors', 'num_3_errors', 'num_4_errors')


def read_errors(data_file):
    """Error-metric records (version >= 3): lane, tile, cycle, error_rate and
    the 0-4 error counts."""
    for data in read_records(data_file, min_version=3):
        yield dict(zip(_ERROR_FIELDS, unpack('<HHHfLLLLL', data[:30])))


def _cycles(records, read_lengths):
    """(tile, cycle, error_rate) sorted; reverse-read cycles renumbered
    -1, -2, ... and index-read cycles dropped."""
    rows = sorted((r['tile'], r['cycle'], r['error_rate']) for r in records)
    last_forward = read_lengths[0] if read_lengths else sys.maxsize
    first_reverse = sum(read_lengths[:-1]) + 1 if read_lengths else sys.maxsize
    for tile, cycle, rate in rows:
        if cycle >= first_reverse:
            yield tile, first_reverse - cycle - 1, rate
        elif cycle <= last_forward:
            yield tile, cycle, rate


def write_phix_csv(out_file, records, read_lengths=None, summary=None):
    """tile,cycle,errorrate rows with every missing cycle written blank, per
    tile and direction; optional average error rates in summary.  In a
    sharded job rank 0 writes while the other ranks wait."""
    from . import session
    with session.writer_stage(out_file) as stage:
        if stage.active:
            _write_phix_csv(out_file, records, read_lengths, summary)


def _write_phix_csv(out_file, records, read_lengths, summary):
    writer = csv.writer(out_file, lineterminator=os.linesep)
    writer.writerow(['tile', 'cycle', 'errorrate'])
    sums, counts = [0.0, 0.0], [0, 0]
    for (tile, sign), group in groupby(_cycles(records, read_lengths),
                                       lambda r: (r[0], int(math.copysign(1, r[1])))):
        prev = 0
        last = None
        for last in group:
            prev += sign
            while prev * sign < last[1] * sign:
                writer.writerow((last[0], prev))
                prev += sign
            writer.writerow(last)
            k = (sign + 1) // 2
            sums[k] += last[2]
            counts[k] += 1
        if read_lengths:
            end = read_lengths[0] if sign == 1 else -read_lengths[-1]
            while prev * sign < end * sign:
                prev += sign
                writer.writerow((last[0], prev))
    if counts[1] > 0 and summary is not None:
        summary['error_rate_fwd'] = sums[1] / counts[1]
    if counts[0] > 0 and summary is not None:
        summary['error_rate_rev'] = sums[0] / counts[0]
