"""Child process of tests/test_gpu_shard.py: one rank of a sharded remap run
(or, with --world 1, the unsharded reference run) on cuda:0, results as JSON.

Ranks use the gloo backend on CUDA tensors by default, which runs the same
device export -> all-reduce -> import path that RCCL runs on a multi-GPU
node.  --backend nccl --shard runs that path over RCCL itself with one rank
(RCCL refuses two ranks on one GPU): every collective, dtype and stream
hand-off of the multi-GPU exchange executes, with a world of one."""
import argparse
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, 'micall-lite_amd'))

import numpy as np  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--rank', type=int, default=0)
    ap.add_argument('--world', type=int, default=1)
    ap.add_argument('--pairs', type=int, default=20000)
    ap.add_argument('--out', required=True)
    ap.add_argument('--backend', default='gloo')
    ap.add_argument('--shard', action='store_true', help='use the Shard path even with --world 1')
    args = ap.parse_args()

    import torch
    import torch.distributed as dist
    from micall_amd import _native, projects, synth
    from micall_amd.pipeline import RemapPipeline, Shard

    cfg = projects.load_default()
    seeds = cfg.seed_sequences()
    genomes = {k: seeds[k] for k in ('HIV1B-pol-seed', 'HIV1B-gag-seed')}
    d = synth.make_pairs(args.pairs, genomes, genome_seed=5, read_seed=6, indel_rate=0.005)
    reads = np.stack([d['r1'], d['r2']], axis=1).reshape(2 * args.pairs, -1)
    quals = np.stack([d['q1'], d['q2']], axis=1).reshape(2 * args.pairs, -1)
    per = args.pairs // args.world
    lo, hi = args.rank * per, (args.rank + 1) * per
    device = torch.device('cuda', 0)
    torch.cuda.set_device(device)
    shard = None
    if args.world > 1 or args.shard:
        dist.init_process_group(args.backend, rank=args.rank, world_size=args.world)
        shard = Shard(args.rank, args.world, read_base=2 * lo, device=device)
    ctx = _native.Context(0)
    ctx.reads_load_fixed(reads[2 * lo:2 * hi], quals[2 * lo:2 * hi], True)
    pipe = RemapPipeline(ctx, shard=shard)
    conseqs, counts, unmapped = pipe.run(2.0 * args.pairs)
    st = pipe.prelim_stats
    res = {'conseqs': list(conseqs.items()), 'counts': list(counts.items()),
           'unmapped': unmapped, 'n_remaps': pipe.n_remaps, 'log': pipe.log,
           'groups': pipe.prelim_groups(),
           'prelim': {k: (np.asarray(v).tolist() if hasattr(v, '__len__') else int(v))
                      for k, v in st.items()}}
    with open(args.out, 'w') as f:
        json.dump(res, f)
    ctx.close()
    if shard is not None:
        dist.destroy_process_group()


if __name__ == '__main__':
    main()
