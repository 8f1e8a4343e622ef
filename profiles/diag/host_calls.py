"""profiles/diag/host_calls.py -- wall time of every native call and Python
stage inside one C2 step (after two warm-up steps), synchronising the device
after each native call so a call's time is its own.
    python3 profiles/diag/host_calls.py"""
import collections
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [REPO, os.path.join(REPO, 'micall-lite_amd')]

import torch  # noqa: E402

import bench  # noqa: E402
from micall_amd import _native, pipeline, consensus  # noqa: E402
from micall_amd.pipeline import RemapPipeline  # noqa: E402

pairs = 1000000
ctx = _native.Context(0)
reads, quals = bench.make_reads(pairs, block=0)
ctx.reads_load_fixed(reads, quals, True)
pipe = RemapPipeline(ctx)
acc = collections.OrderedDict()


def timed(name, fn):
    def w(*a, **kw):
        t0 = time.perf_counter()
        r = fn(*a, **kw)
        torch.cuda.synchronize()
        acc[name] = acc.get(name, 0.0) + (time.perf_counter() - t0) * 1e3
        return r
    return w


for name in ('index_build', 'map', 'map_counts', 'map_stats', 'pileup', 'pileup_fetch', 'pileup_scalars',
             'gotoh_align_many'):
    if hasattr(ctx, name):
        setattr(ctx, name, timed('ctx.' + name, getattr(ctx, name)))
for mod, name in ((consensus, 'counts_to_conseqs'), (consensus, 'filter_conseqs'),
                  (pipeline, 'counts_to_conseqs'), (pipeline, 'filter_conseqs')):
    if hasattr(mod, name):
        setattr(mod, name, timed(mod.__name__.split('.')[-1] + '.' + name, getattr(mod, name)))
for _ in range(2):
    pipe.run(2.0 * pairs, max_iterations=1)
torch.cuda.synchronize()
acc.clear()
t0 = time.perf_counter()
pipe.run(2.0 * pairs, max_iterations=1)
torch.cuda.synchronize()
print('step wall ms %.2f' % ((time.perf_counter() - t0) * 1e3))
for k, v in acc.items():
    print('%-34s %8.3f ms' % (k, v))
