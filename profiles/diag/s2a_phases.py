"""profiles/diag/s2a_phases.py -- the sam2aln drop-in file to file on the
remap.csv of one C2 remap pass: the library's parse phases (MH_S2A_TRACE),
device, formatting, and the Python-side reads and writes.
    python3 profiles/diag/s2a_phases.py [pairs] [repeats]"""
import json
import os
import sys
import tempfile
import time

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [REPO, os.path.join(REPO, 'micall-lite_amd')]

import bench  # noqa: E402
from micall_amd import _native, sam2aln, session  # noqa: E402
from micall_amd.pipeline import RemapPipeline  # noqa: E402

pairs = int(sys.argv[1]) if len(sys.argv) > 1 else 1000000
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 3
ctx = _native.Context(0)
reads, quals = bench.make_reads(pairs, block=0)
ctx.reads_load_fixed(reads, quals, True)
del reads, quals
ctx.set_names(['M00000:1:000000000-AAAAA:1:1101:{}:{}'.format(1000 + i // 1000000, 1000 + i % 1000000)
               for i in range(pairs) for _ in (0, 1)])
RemapPipeline(ctx).run(2.0 * pairs, max_iterations=1)
text = ('qname,flag,rname,pos,mapq,cigar,rnext,pnext,tlen,seq,qual\n' +
        ctx.format_rows(1, 0, 2 * pairs)).encode()
ctx.close()
with tempfile.TemporaryDirectory(dir='/tmp') as d:
    p = os.path.join(d, 'remap.csv')
    with open(p, 'wb') as f:
        f.write(text)
    del text
    for rep in range(reps):
        t0 = time.perf_counter()
        with open(p) as remap, open(os.path.join(d, 'aligned.csv'), 'w') as al, \
                open(os.path.join(d, 'insert.csv'), 'w') as ins, open(os.path.join(d, 'failed.csv'), 'w') as fl:
            sam2aln.sam2aln(remap, al, ins, fl)
        t1 = time.perf_counter()
        tm = session.context().sam2aln_timing()
        sizes = {k: os.path.getsize(os.path.join(d, k + '.csv')) for k in ('aligned', 'insert', 'failed')}
        print(json.dumps({'rep': rep, 'dropin_s': round(t1 - t0, 4), 'lib_ms': [round(x, 1) for x in tm],
                          'bytes': sizes}), flush=True)
