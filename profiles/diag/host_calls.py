"""Per-call host wall time of the native context's calls inside a C2 step
(no added synchronisation: a call's time is what the host spends in it,
including the waits it does itself).  Diagnostic only.

    python profiles/diag/host_calls.py [--pairs N] [--steps K]
"""
import argparse
import collections
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, 'micall-lite_amd'))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--pairs', type=int, default=1000000)
    ap.add_argument('--steps', type=int, default=3)
    args = ap.parse_args()
    import torch
    import bench
    from micall_amd import _native
    from micall_amd.pipeline import RemapPipeline
    torch.cuda.set_device(0)
    ctx = _native.Context(0)
    reads, quals = bench.make_reads(args.pairs, block=0)
    ctx.reads_load_fixed(reads, quals, True)
    pipe = RemapPipeline(ctx)
    acc = collections.defaultdict(lambda: [0.0, 0])
    names = [n for n in dir(ctx) if not n.startswith('_') and callable(getattr(ctx, n))]
    for n in names:
        fn = getattr(ctx, n)

        def timed(*a, _fn=fn, _n=n, **kw):
            t = time.perf_counter()
            r = _fn(*a, **kw)
            acc[_n][0] += time.perf_counter() - t
            acc[_n][1] += 1
            return r
        setattr(ctx, n, timed)
    pipe.run(2.0 * args.pairs, max_iterations=1)
    ctx.sync()
    acc.clear()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        pipe.run(2.0 * args.pairs, max_iterations=1)
    ctx.sync()
    wall = (time.perf_counter() - t0) / args.steps * 1e3
    print('step_ms %.3f' % wall)
    for n, (s, k) in sorted(acc.items(), key=lambda kv: -kv[1][0]):
        print('%-24s %8.3f ms/step  %5.1f calls/step' % (n, s / args.steps * 1e3, k / args.steps))


if __name__ == '__main__':
    main()
