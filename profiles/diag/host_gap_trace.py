"""Diagnostics: where the GPU's idle time between the kernels of a C2 bench
step goes on the host.  Every native call of the context and every stage of
RemapPipeline records (name, enter, exit) with time.perf_counter_ns() (no
synchronisation is added), so that, run under
    rocprofv3 --kernel-trace --output-format csv -d DIR -o run -- python3 host_gap_trace.py
the host intervals line up with the kernel trace (both CLOCK_MONOTONIC).
    python3 profiles/diag/host_gap_trace.py [pairs] [steps] [out.json]"""
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
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 4
out = sys.argv[3] if len(sys.argv) > 3 else os.path.join(REPO, 'gpurun_out', 'host_gap.json')
log = []
depth = [0]


def wrap(obj, name, label):
    fn = getattr(obj, name)

    def timed(*a, **kw):
        t = time.perf_counter_ns()
        depth[0] += 1
        try:
            return fn(*a, **kw)
        finally:
            depth[0] -= 1
            log.append((label, t, time.perf_counter_ns(), depth[0]))
    setattr(obj, name, timed)


ctx = _native.Context(0)
reads, quals = bench.make_reads(pairs, block=0)
ctx.reads_load_fixed(reads, quals, True)
del reads, quals
pipe = RemapPipeline(ctx)
for _ in range(2):
    pipe.run(2.0 * pairs, max_iterations=1)
ctx.sync()
for name in ('index_build', 'map', 'map_counts', 'pileup', 'pileup_fetch', 'map_stats', 'reads_count'):
    if hasattr(ctx, name):
        wrap(ctx, name, 'ctx.' + name)
for name in ('prelim', 'prelim_groups', 'select_seeds', 'prelim_conseqs', 'map_to_reference',
             'build_conseqs_filtered', '_counts', '_pileup', 'iterate'):
    wrap(pipe, name, 'pipe.' + name)
for mod, names in ((pipeline, ('Pileup', 'counts_to_conseqs', 'filter_conseqs')),):
    for name in names:
        wrap(mod, name, 'py.' + name)
t0 = time.perf_counter_ns()
for _ in range(steps):
    s = time.perf_counter_ns()
    pipe.run(2.0 * pairs, max_iterations=1)
    log.append(('step', s, time.perf_counter_ns(), 0))
ctx.sync()
print('ms per step', round((time.perf_counter_ns() - t0) / 1e6 / steps, 3))
os.makedirs(os.path.dirname(out), exist_ok=True)
with open(out, 'w') as f:
    json.dump(log, f)
