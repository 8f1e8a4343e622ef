"""Child process of tests/test_gpu_shard_dropin.py: one rank of a sharded
bin/micall-style run of the drop-ins, prelim_map() then remap(), on cuda:0.

The rank reads RANK / WORLD_SIZE / MASTER_* from the environment as under
torchrun; micall_amd.session initialises the process group
(MICALL_DIST_BACKEND, gloo here: two ranks share the test box's one GPU) and
keeps this rank's block of read pairs resident.  Every rank opens the same
output paths; rank 0 writes them.  With --fresh-remap the process context is
dropped between the calls, so remap() parses prelim.csv (every rank the whole
file) instead of reusing the resident prelim records."""
import argparse
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, 'micall-lite_amd'))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('r1')
    ap.add_argument('r2', nargs='?')
    ap.add_argument('--out', required=True)
    ap.add_argument('--fresh-remap', action='store_true')
    args = ap.parse_args()

    from micall_amd import prelim_map as pm
    from micall_amd import remap as rm
    from micall_amd import session

    out = args.out
    with open(os.path.join(out, 'prelim.csv'), 'w') as f:
        pm.prelim_map(args.r1, args.r2, f, gzip=True)
    reads = session.context().reads_count()[0]
    if args.fresh_remap:
        session.reset()
    names = ('remap.csv', 'remap_counts.csv', 'remap_conseq.csv', 'unmapped1.fastq',
             'unmapped2.fastq')
    with open(os.path.join(out, 'prelim.csv')) as prelim:
        handles = [open(os.path.join(out, n), 'w+') for n in names]
        rm.remap(args.r1, args.r2, prelim, *handles, gzip=True, work_path=out)
        for h in handles:
            h.close()
    sh = session.shard()
    with open(os.path.join(out, 'rank%d.json' % (sh.rank if sh else 0)), 'w') as f:
        json.dump(dict(prelim_source=session.stats.get('prelim_source'),
                       world=sh.world if sh else 1, read_base=sh.read_base if sh else 0,
                       reads=reads), f)
    if sh is not None:
        import torch.distributed as dist
        dist.destroy_process_group()


if __name__ == '__main__':
    main()
