"""profiles/diag/step_profile.py -- where the host time of a C2 bench step
goes (the GPU idles ~1.8 ms per step between kernels): cProfile of
RemapPipeline.run over a few steps, device work synchronised as bench.py
does only at the step ends.
    python3 profiles/diag/step_profile.py [pairs] [steps]"""
import cProfile
import os
import pstats
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [REPO, os.path.join(REPO, 'micall-lite_amd')]

import bench  # noqa: E402
from micall_amd import _native  # noqa: E402
from micall_amd.pipeline import RemapPipeline  # noqa: E402

pairs = int(sys.argv[1]) if len(sys.argv) > 1 else 1000000
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 10
genomes = sys.argv[3] if len(sys.argv) > 3 else 'pol'
ctx = _native.Context(0)
reads, quals = bench.make_reads(pairs, block=0, genomes=genomes)
ctx.reads_load_fixed(reads, quals, True)
del reads, quals
pipe = RemapPipeline(ctx)
for _ in range(3):
    pipe.run(2.0 * pairs, max_iterations=1)
ctx.sync()
t = time.perf_counter()
for _ in range(steps):
    pipe.run(2.0 * pairs, max_iterations=1)
ctx.sync()
print('ms per step', round(1e3 * (time.perf_counter() - t) / steps, 3))
pr = cProfile.Profile()
pr.enable()
for _ in range(steps):
    pipe.run(2.0 * pairs, max_iterations=1)
ctx.sync()
pr.disable()
st = pstats.Stats(pr)
st.sort_stats('tottime').print_stats(40)
st.sort_stats('cumulative').print_stats(60)
