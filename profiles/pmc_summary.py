#!/usr/bin/env python3
"""profiles/pmc_summary.py -- per-kernel HBM traffic from two separate
rocprofv3 --pmc passes (FETCH_SIZE, WRITE_SIZE; both in KiB per dispatch).

Correction (MI355X_MICROARCH.md, HBM section): on gfx950 FETCH_SIZE reports
half the bytes of a wide coalesced streaming read, so the read side is
doubled: hbm_bytes = (2 * FETCH_SIZE + WRITE_SIZE) * 1024.  Reads that are
narrower than 16 B/lane are not calibrated by that rule; the doubled figure
is an upper estimate for them.

A k_dp dispatch that follows a k_rescue dispatch is the mate-rescue DP
launch and is reported as k_dp_rescue (same kernel, different work).

usage: pmc_summary.py FETCH_CSV WRITE_CSV PAIRS OUT_JSON
"""
import csv
import json
import sys
from collections import defaultdict


def per_kernel(path, counter):
    rows = {}
    with open(path) as f:
        for row in csv.DictReader(f):
            if row['Counter_Name'] == counter:
                rows[int(row['Dispatch_Id'])] = (row['Kernel_Name'], float(row['Counter_Value']))
    acc = defaultdict(list)
    prev = None
    for d in sorted(rows):
        name, value = rows[d]
        label = 'k_dp_rescue' if name == 'k_dp' and prev == 'k_rescue' else name
        acc[label].append(value)
        prev = name
    return acc


def main(fetch_csv, write_csv, pairs, out):
    fetch = per_kernel(fetch_csv, 'FETCH_SIZE')
    write = per_kernel(write_csv, 'WRITE_SIZE')
    kernels = {}
    for k in sorted(set(fetch) | set(write)):
        f = fetch.get(k, [])
        w = write.get(k, [])
        n = max(len(f), len(w), 1)
        fk = sum(f) / max(len(f), 1)
        wk = sum(w) / max(len(w), 1)
        kernels[k] = {'launches': n, 'fetch_kib_per_launch': round(fk, 1),
                      'write_kib_per_launch': round(wk, 1),
                      'hbm_bytes_per_launch': int(round((2 * fk + wk) * 1024))}
    with open(out, 'w') as f:
        json.dump({'pairs': int(pairs), 'rule': '(2*FETCH_SIZE + WRITE_SIZE) * 1024',
                   'kernel_source_sha': _source_sha(), 'kernels': kernels}, f, indent=1)


def _source_sha():
    """bench.kernel_source_sha() of the tree the passes were collected from
    (bench.py only uses a summary whose fingerprint matches its own)."""
    import os
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    from bench import kernel_source_sha
    return kernel_source_sha()


if __name__ == '__main__':
    main(*sys.argv[1:])
