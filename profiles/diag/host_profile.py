"""profiles/diag/host_profile.py -- where the host time of one C2 step goes:
cProfile over RemapPipeline.run (after two warm-up steps) on the GPU box.
    python3 profiles/diag/host_profile.py [pairs]"""
import cProfile
import os
import pstats
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [REPO, os.path.join(REPO, 'micall-lite_amd')]

import torch  # noqa: E402

import bench  # noqa: E402
from micall_amd import _native  # noqa: E402
from micall_amd.pipeline import RemapPipeline  # noqa: E402

pairs = int(sys.argv[1]) if len(sys.argv) > 1 else 1000000
ctx = _native.Context(0)
reads, quals = bench.make_reads(pairs, block=0)
ctx.reads_load_fixed(reads, quals, True)
pipe = RemapPipeline(ctx)
for _ in range(2):
    pipe.run(2.0 * pairs, max_iterations=1)
torch.cuda.synchronize()
t0 = time.perf_counter()
prof = cProfile.Profile()
prof.enable()
pipe.run(2.0 * pairs, max_iterations=1)
prof.disable()
print('step wall ms', round((time.perf_counter() - t0) * 1000, 2))
pstats.Stats(prof).sort_stats('tottime').print_stats(25)
