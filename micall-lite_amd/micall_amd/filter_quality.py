"""
Host-side mirror of micall/core/filter_quality.py:33-63 (report_bad_cycles):
per tile and read direction, every cycle from the first one whose phiX error
rate is missing, blank or >= 7.5 onwards is a bad cycle.  A few kB of CSV;
no device work.
"""
import csv
import itertools
import math
import os
from operator import itemgetter

BAD_ERROR_RATE = 7.5


def report_bad_cycles(quality_csv, bad_cycles_csv, bad_tiles_csv=None):
    """filter_quality.report_bad_cycles.  In a sharded job rank 0 writes
    while the other ranks wait."""
    from . import session
    with session.writer_stage(bad_cycles_csv, bad_tiles_csv) as stage:
        if stage.active:
            _report_bad_cycles(quality_csv, bad_cycles_csv, bad_tiles_csv)


def _report_bad_cycles(quality_csv, bad_cycles_csv, bad_tiles_csv):
    reader = csv.DictReader(quality_csv)
    writer = csv.DictWriter(bad_cycles_csv, ['tile', 'cycle', 'errorrate'],
                            lineterminator=os.linesep)
    writer.writeheader()
    tile_writer = None
    if bad_tiles_csv is not None:
        tile_writer = csv.DictWriter(bad_tiles_csv, ['tile', 'bad_cycles'],
                                     lineterminator=os.linesep)
        tile_writer.writeheader()
    for tile, rows in itertools.groupby(reader, itemgetter('tile')):
        n_bad = 0
        for _sign, direction in itertools.groupby(
                rows, lambda row: math.copysign(1, int(row['cycle']))):
            bad = False
            for row in direction:
                rate = row['errorrate']
                bad = bad or rate is None or rate == '' or float(rate) >= BAD_ERROR_RATE
                if bad:
                    writer.writerow(row)
                    n_bad += 1
        if tile_writer is not None:
            tile_writer.writerow(dict(tile=tile, bad_cycles=n_bad))
