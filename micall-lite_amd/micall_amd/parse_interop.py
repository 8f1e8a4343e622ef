"""
Host-side mirror of micall/core/parse_interop.py: the Illumina InterOp
ErrorMetricsOut.bin reader and the phiX error-rate CSV writer that feed the
censor stage (bin/micall:101-106).  Byte parsing of a few kB; no device work.

    read_records    parse_interop.py:14-40
    read_errors     parse_interop.py:43-72
    write_phix_csv  parse_interop.py:98-139 (cycle renumbering :75-95)

write_phix_csv's behaviour, restated: records are ordered by (tile, cycle,
rate).  With read lengths [forward, index..., reverse], cycles up to the
forward length are forward cycles, cycles from sum(lengths[:-1]) + 1 on are
reverse cycles renumbered -1, -2, ..., and the index cycles between are
dropped.  Each (tile, direction) lane is written in order with a blank row
(tile and cycle only) for every cycle the records skip, counted from the
lane's start; a record whose cycle does not advance (a duplicate) still
takes the next slot.  With read lengths, the lane is then padded with blank
rows to the read's length.  summary gets the mean rate of the written
records per direction.
"""
import csv
import os
import sys
from struct import unpack


def read_records(data_file, min_version):
    """Fixed-length records after a (version, record length) header byte pair."""
    version, record_length = unpack('!BB', data_file.read(2))
    if version < min_version:
        raise IOError('File version {} is less than minimum version {} in {}.'.format(
            version, min_version, data_file.name))
    if record_length == 0:     # every read of 0 bytes comes back empty: no records
        return
    body = memoryview(data_file.read())
    whole = len(body) - len(body) % record_length
    for at in range(0, whole, record_length):
        yield bytes(body[at:at + record_length])
    if len(body) > whole:
        raise IOError('Partial record of length {} found in {}.'.format(len(body) - whole,
                                                                       data_file.name))


_ERROR_FIELDS = ('lane', 'tile', 'cycle', 'error_rate', 'num_0_errors', 'num_1_error',
                 'num_2_errors', 'num_3_errors', 'num_4_errors')


def read_errors(data_file):
    """Error-metric records (version >= 3): lane, tile, cycle, error_rate and
    the 0-4 error counts."""
    for data in read_records(data_file, min_version=3):
        yield dict(zip(_ERROR_FIELDS, unpack('<HHHfLLLLL', data[:30])))


def _lanes(records, read_lengths):
    """{(tile, +1 | -1): [(cycle number within the read, rate), ...]} in
    (tile, cycle, rate) order; index-read cycles left out."""
    if read_lengths:
        forward_end, reverse_start = read_lengths[0], sum(read_lengths[:-1]) + 1
    else:
        forward_end = reverse_start = sys.maxsize
    lanes = {}
    for tile, cycle, rate in sorted((r['tile'], r['cycle'], r['error_rate']) for r in records):
        if cycle >= reverse_start:
            lanes.setdefault((tile, -1), []).append((cycle - reverse_start + 1, rate))
        elif cycle <= forward_end:
            lanes.setdefault((tile, 1), []).append((cycle, rate))
    return lanes


def _phix_rows(records, read_lengths, totals):
    """The CSV rows of write_phix_csv; totals[direction] = [sum, count] of
    the record rates written."""
    lanes = _lanes(records, read_lengths)
    rows = []
    for tile, direction in sorted(lanes, key=lambda key: (key[0], -key[1])):
        slot = 0
        acc = totals[direction]
        for number, rate in lanes[tile, direction]:
            rows.extend((tile, direction * blank) for blank in range(slot + 1, number))
            rows.append((tile, direction * number, rate))
            slot = max(slot + 1, number)
            acc[0] += rate
            acc[1] += 1
        if read_lengths:
            length = read_lengths[0] if direction == 1 else read_lengths[-1]
            rows.extend((tile, direction * blank) for blank in range(slot + 1, length + 1))
    return rows


def write_phix_csv(out_file, records, read_lengths=None, summary=None):
    """tile,cycle,errorrate rows with every missing cycle written blank, per
    tile and direction; optional average error rates in summary.  In a
    sharded job rank 0 writes while the other ranks wait."""
    from . import session
    with session.writer_stage(out_file) as stage:
        if stage.active:
            _write_phix_csv(out_file, records, read_lengths, summary)


def _write_phix_csv(out_file, records, read_lengths, summary):
    totals = {1: [0.0, 0], -1: [0.0, 0]}
    rows = _phix_rows(records, read_lengths, totals)
    writer = csv.writer(out_file, lineterminator=os.linesep)
    writer.writerow(['tile', 'cycle', 'errorrate'])
    writer.writerows(rows)
    if summary is not None:
        for direction, key in ((1, 'error_rate_fwd'), (-1, 'error_rate_rev')):
            total, count = totals[direction]
            if count:
                summary[key] = total / count
