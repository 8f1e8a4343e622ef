"""profiles/diag/a2c_profile.py -- cProfile of one aln2counts drop-in call on
the aligned.csv of one C2 remap pass (as bench.py --stage aln2counts makes
it): where the ~0.4 s of a call go.
    python3 profiles/diag/a2c_profile.py [pairs]"""
import cProfile
import io
import os
import pstats
import sys
import tempfile
import time

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [REPO, os.path.join(REPO, 'micall-lite_amd')]

import bench  # noqa: E402
from micall_amd import aln2counts as a2c, session  # noqa: E402
from micall_amd.pipeline import RemapPipeline  # noqa: E402

pairs = int(sys.argv[1]) if len(sys.argv) > 1 else 1000000
ctx = session.context()
reads, quals = bench.make_reads(pairs, block=0)
ctx.reads_load_fixed(reads, quals, True)
del reads, quals
ctx.set_names(['M00000:1:000000000-AAAAA:1:1101:{}:{}'.format(1000 + i // 1000000, 1000 + i % 1000000)
               for i in range(pairs) for _ in (0, 1)])
RemapPipeline(ctx).run(2.0 * pairs, max_iterations=1)
text = ('qname,flag,rname,pos,mapq,cigar,rnext,pnext,tlen,seq,qual\n' + ctx.format_rows(1, 0, 2 * pairs)).encode()
ctx.sam2aln_csv(text)
del text
aligned = ctx.sam2aln_output('aligned')
d = tempfile.mkdtemp(prefix='a2cprof_')
path = os.path.join(d, 'aligned.csv')
with open(path, 'w') as f:
    f.write(aligned)
del aligned


def step(to_files):
    a2c.aligner.forget()
    if to_files:
        names = ['nuc', 'amino', 'insert', 'conseq', 'failed', 'coverage']
        outs = [open(os.path.join(d, n + '.csv'), 'w') for n in names]
    else:
        outs = [io.StringIO() for _ in range(6)]
    with open(path) as f:
        a2c.aln2counts(f, *outs[:4], failed_align_csv=outs[4], coverage_summary_csv=outs[5])
    for o in outs:
        o.close()


step(False)
for to_files in (False, True):
    t = time.perf_counter()
    step(to_files)
    print('to_files', to_files, round(time.perf_counter() - t, 4), flush=True)
pr = cProfile.Profile()
pr.enable()
step(True)
pr.disable()
pstats.Stats(pr).sort_stats('cumulative').print_stats(35)
pstats.Stats(pr).sort_stats('tottime').print_stats(25)
