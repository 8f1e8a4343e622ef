"""profiles/diag/host_timeline.py -- host wall time of every context call and
consensus step inside C2 bench steps (no synchronisation added: each
native call already returns when its device work is done), per step, to find
the host time between the kernels.
    python3 profiles/diag/host_timeline.py [pairs] [steps]"""
import collections
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [REPO, os.path.join(REPO, 'micall-lite_amd')]

import bench  # noqa: E402
from micall_amd import _native, consensus, pipeline  # noqa: E402
from micall_amd.pipeline import RemapPipeline  # noqa: E402

pairs = int(sys.argv[1]) if len(sys.argv) > 1 else 1000000
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 10
ctx = _native.Context(0)
reads, quals = bench.make_reads(pairs, block=0, genomes='pol')
ctx.reads_load_fixed(reads, quals, True)
del reads, quals
acc = collections.defaultdict(float)
cnt = collections.Counter()


def wrap(obj, name, label):
    f = getattr(obj, name)

    def g(*a, **kw):
        t = time.perf_counter_ns()
        try:
            return f(*a, **kw)
        finally:
            acc[label] += time.perf_counter_ns() - t
            cnt[label] += 1
    setattr(obj, name, g)


for m in ('map', 'map_counts', 'pileup', 'pileup_fetch', 'index_build'):
    wrap(ctx, m, 'ctx.' + m)
wrap(consensus, 'counts_to_conseqs', 'counts_to_conseqs')
pipeline.counts_to_conseqs = consensus.counts_to_conseqs
wrap(pipeline, 'Pileup', 'Pileup()')
pipe = RemapPipeline(ctx)
for _ in range(3):
    pipe.run(2.0 * pairs, max_iterations=1)
ctx.sync()
acc.clear()
cnt.clear()
t = time.perf_counter_ns()
for _ in range(steps):
    pipe.run(2.0 * pairs, max_iterations=1)
ctx.sync()
total = (time.perf_counter_ns() - t) / steps
out = {'us_per_step': round(total / 1e3, 1)}
for k in sorted(acc, key=lambda k: -acc[k]):
    out[k] = {'us_per_step': round(acc[k] / steps / 1e3, 1), 'calls_per_step': cnt[k] / steps}
out['other_us_per_step'] = round((total - sum(acc.values()) / steps) / 1e3, 1)
print(json.dumps(out, indent=1))
