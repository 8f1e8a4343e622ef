"""Diagnostic: wall time of mh_index_build in isolation and inside the bench
pipeline (1M resident pairs), on the GPU box."""
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(REPO, 'micall-lite_amd'))
sys.path.insert(0, REPO)
from micall_amd import _native, projects  # noqa: E402
from micall_amd.pipeline import RemapPipeline  # noqa: E402
import bench  # noqa: E402

ctx = _native.Context(0)
seeds = projects.load_default().seed_sequences()
names = list(seeds)


def timed_build(ns, ss, sl):
    ctx.sync()
    t = time.perf_counter()
    ctx.index_build(ns, ss, sl)
    return 1e3 * (time.perf_counter() - t)


print('isolated seeds74 %.2f %.2f ms' % (timed_build(names, [seeds[n] for n in names], 22),
                                         timed_build(names, [seeds[n] for n in names], 22)))
reads, quals = bench.make_reads(int(sys.argv[1]) if len(sys.argv) > 1 else 1000000, block=0)
ctx.reads_load_fixed(reads, quals, True)
pipe = RemapPipeline(ctx)
orig = ctx.index_build
log = []


def wrapped(ns, ss, sl):
    ctx.sync()
    t = time.perf_counter()
    orig(ns, ss, sl)
    log.append((len(ns), sum(map(len, ss)), 1e3 * (time.perf_counter() - t)))


ctx.index_build = wrapped
for _ in range(3):
    pipe.run(2e6, max_iterations=1)
for n, total, ms in log:
    print('in pipeline: %d refs, %d nt: %.2f ms' % (n, total, ms))
