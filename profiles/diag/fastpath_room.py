"""profiles/diag/fastpath_room.py -- how many C2 remap-pass alignments are
ungapped with few mismatches (room for a wider exact ungapped fast path in
k_dp): records of the last (--local) pass by XO (gap opens), XM
(mismatches) and soft clipping.
    python3 profiles/diag/fastpath_room.py [pairs]"""
import collections
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [REPO, os.path.join(REPO, 'micall-lite_amd')]

import numpy as np  # noqa: E402

import bench  # noqa: E402
from micall_amd import _native  # noqa: E402
from micall_amd.pipeline import RemapPipeline  # noqa: E402

pairs = int(sys.argv[1]) if len(sys.argv) > 1 else 1000000
ctx = _native.Context(0)
reads, quals = bench.make_reads(pairs, block=0)
ctx.reads_load_fixed(reads, quals, True)
del reads, quals
RemapPipeline(ctx).run(2.0 * pairs, max_iterations=1)
F = {k: i for i, k in enumerate(_native.ALN_FIELDS)}
r = ctx.recs()
mapped = (r[:, F['flag']] & 4) == 0
xo, xm, ncig = r[:, F['xo']], r[:, F['xm']], r[:, F['n_cigar']]
out = {'records': int(len(r)), 'mapped': int(mapped.sum()),
       'gapped': int((mapped & (xo > 0)).sum()),
       'ungapped_by_xm': {}, 'ungapped_clipped_by_xm': {}}
for k in range(6):
    sel = mapped & (xo == 0) & ((xm == k) if k < 5 else (xm >= 5))
    out['ungapped_by_xm'][str(k) if k < 5 else '5+'] = int((sel & (ncig == 1)).sum())
    out['ungapped_clipped_by_xm'][str(k) if k < 5 else '5+'] = int((sel & (ncig > 1)).sum())
print(json.dumps(out))
