#!/usr/bin/env python3
"""profiles/sq_summary.py -- per-dispatch issue statistics from one rocprofv3
--pmc pass of SQ counters (profiles/collect_r02.sh, pmc_sq):

  clock_ghz              GRBM_GUI_ACTIVE / 8 (XCDs) / kernel time
  valu_insts             SQ_INSTS_VALU (wave instructions, chip total)
  simd_cycles_per_valu   1024 SIMDs x kernel time x clock / SQ_INSTS_VALU
  wait_any / wait_inst / active: shares of SQ_WAVE_CYCLES in SQ_WAIT_ANY,
                         SQ_WAIT_INST_ANY and SQ_ACTIVE_INST_ANY
plus the VGPR / LDS figures of the dispatch.

usage: sq_summary.py COUNTER_CSV OUT_JSON [kernel ...]
"""
import csv
import json
import sys
from collections import OrderedDict


def main(path, out, *kernels):
    disp = OrderedDict()
    with open(path) as f:
        for row in csv.DictReader(f):
            if kernels and row['Kernel_Name'] not in kernels:
                continue
            d = disp.setdefault(int(row['Dispatch_Id']), {
                'kernel': row['Kernel_Name'], 'dispatch': int(row['Dispatch_Id']),
                'ns': int(row['End_Timestamp']) - int(row['Start_Timestamp']),
                'vgpr': int(row['VGPR_Count']), 'agpr': int(row['Accum_VGPR_Count']),
                'lds_block': int(row['LDS_Block_Size']), 'workgroup': int(row['Workgroup_Size']),
                'c': {}})
            d['c'][row['Counter_Name']] = float(row['Counter_Value'])
    res = []
    for d in disp.values():
        c, ns = d.pop('c'), d.pop('ns')
        if ns <= 0 or 'SQ_INSTS_VALU' not in c:
            continue
        clk = c.get('GRBM_GUI_ACTIVE', 0) / 8 / ns
        wc = max(c.get('SQ_WAVE_CYCLES', 0), 1)
        valu = c['SQ_INSTS_VALU']
        d.update(ms=round(ns / 1e6, 3), clock_ghz=round(clk, 3), valu_insts=valu,
                 salu_insts=c.get('SQ_INSTS_SALU'), waves=c.get('SQ_WAVES'),
                 simd_cycles_per_valu=round(1024 * ns * clk / valu, 2) if valu else None,
                 wait_any_frac=round(c.get('SQ_WAIT_ANY', 0) / wc, 3),
                 wait_inst_frac=round(c.get('SQ_WAIT_INST_ANY', 0) / wc, 3),
                 active_frac=round(c.get('SQ_ACTIVE_INST_ANY', 0) / wc, 3))
        res.append(d)
    with open(out, 'w') as f:
        json.dump({'note': 'rocprofv3 --pmc SQ_* pass (profiles/collect_r02.sh); counters are '
                           'chip totals per dispatch; see profiles/sq_summary.py',
                   'kernel_source_sha': _source_sha(), 'dispatches': res}, f, indent=1)


def _source_sha():
    """bench.kernel_source_sha() of the tree the passes were collected from
    (bench.py only uses a summary whose fingerprint matches its own)."""
    import os
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    from bench import kernel_source_sha
    return kernel_source_sha()


if __name__ == '__main__':
    main(*sys.argv[1:])
