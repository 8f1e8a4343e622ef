"""
Host-side mirror of micall/core/filter_quality.py:36-63 (report_bad_cycles).

Behaviour (the reference's, restated): the quality CSV is read in file order.
A *run* is a stretch of consecutive rows with the same tile and the same read
direction (the sign of the cycle; cycle 0 counts as forward).  Within a run,
the first row whose error rate is missing, blank or >= 7.5 starts the bad
part, and that row and every later row of the run are written to the
bad-cycles CSV; the rate of a row after that point is not looked at.  With a
bad-tiles CSV, each stretch of consecutive rows of one tile gets a row with
the number of bad cycles it wrote.  A few kB of CSV; no device work.
"""
import csv
import os

BAD_ERROR_RATE = 7.5


def report_bad_cycles(quality_csv, bad_cycles_csv, bad_tiles_csv=None):
    """filter_quality.report_bad_cycles.  In a sharded job rank 0 writes
    while the other ranks wait."""
    from . import session
    with session.writer_stage(bad_cycles_csv, bad_tiles_csv) as stage:
        if stage.active:
            _report_bad_cycles(quality_csv, bad_cycles_csv, bad_tiles_csv)


def _is_bad_rate(rate):
    return rate is None or rate == '' or float(rate) >= BAD_ERROR_RATE


def _report_bad_cycles(quality_csv, bad_cycles_csv, bad_tiles_csv):
    cycles_out = csv.DictWriter(bad_cycles_csv, ['tile', 'cycle', 'errorrate'],
                                lineterminator=os.linesep)
    cycles_out.writeheader()
    tiles_out = None
    if bad_tiles_csv is not None:
        tiles_out = csv.DictWriter(bad_tiles_csv, ['tile', 'bad_cycles'], lineterminator=os.linesep)
        tiles_out.writeheader()

    def close_tile(tile, count):
        if tiles_out is not None:
            tiles_out.writerow({'tile': tile, 'bad_cycles': count})

    run = None            # (tile, reverse?) of the current run
    past_bad = False      # the current run has reached its first bad cycle
    tile_bad = 0          # bad cycles written for the current tile stretch
    for row in csv.DictReader(quality_csv):
        tile = row['tile']
        here = (tile, int(row['cycle']) < 0)
        if here != run:
            if run is not None and run[0] != tile:
                close_tile(run[0], tile_bad)
                tile_bad = 0
            run, past_bad = here, False
        past_bad = past_bad or _is_bad_rate(row['errorrate'])
        if past_bad:
            cycles_out.writerow(row)
            tile_bad += 1
    if run is not None:
        close_tile(run[0], tile_bad)
