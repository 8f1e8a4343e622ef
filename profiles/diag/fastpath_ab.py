"""A/B of k_dp's exact ungapped fast path (mh_ctx_set_option "dp_fast") on
the bench workload: the --local remap pass against the first and the second
consensus, k_dp device time (HIP events) and the share of extensions the
fast path resolved.  Diagnostics only; run on the GPU box from the repo root:
    python profiles/diag/fastpath_ab.py [pairs]
"""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [REPO, os.path.join(REPO, 'micall-lite_amd')]

import bench  # noqa: E402
from micall_amd import _native  # noqa: E402
from micall_amd.pipeline import RemapPipeline  # noqa: E402


def main():
    pairs = int(sys.argv[1]) if len(sys.argv) > 1 else 1000000
    ctx = _native.Context(0)
    reads, quals = bench.make_reads(pairs, block=0)
    ctx.reads_load_fixed(reads, quals, True)
    pipe = RemapPipeline(ctx)
    pipe.prelim()
    conseqs, _ = pipe.prelim_conseqs(pipe.select_seeds(pipe.prelim_groups()))
    out = []
    for it in (1, 2):
        for fast in (0, 1, 0, 1):
            ctx.set_option('dp_fast', fast)
            ctx.profile(True)
            pipe.map_to_reference(conseqs)
            ctx.sync()
            ms, n = ctx.profile_get('k_dp')
            st = ctx.map_stats()
            out.append(dict(iteration=it, dp_fast=fast, k_dp_ms=round(ms, 3), extensions=st[1],
                            fast=st[3]))
            print(json.dumps(out[-1]), flush=True)
        ctx.set_option('dp_fast', 1)
        conseqs = pipe.build_conseqs_filtered(conseqs)
    ctx.close()


if __name__ == '__main__':
    main()
