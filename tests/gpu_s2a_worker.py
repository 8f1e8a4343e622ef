"""Child process of tests/test_gpu_shard_sam2aln.py: one rank of a sharded
sam2aln over many remap.csv files, on cuda:0 (gloo: the ranks share the
test box's one GPU).  For each case directory under --cases it calls the
drop-in as bin/micall does -- every rank opens remap.csv and the three
outputs -- and records how the call ran (micall_amd.sam2aln.SHARD_STATS)."""
import argparse
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, 'micall-lite_amd'))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--cases', required=True)
    args = ap.parse_args()
    from micall_amd import sam2aln as s2a
    from micall_amd import session
    sh = session.shard()
    stats = {}
    for case in sorted(os.listdir(args.cases)):
        d = os.path.join(args.cases, case)
        with open(os.path.join(d, 'remap.csv')) as rc, open(os.path.join(d, 'aligned.csv'), 'w') as al, \
                open(os.path.join(d, 'insert.csv'), 'w') as ins, open(os.path.join(d, 'failed.csv'), 'w') as fa:
            s2a.sam2aln(rc, al, ins, fa)
        stats[case] = dict(s2a.SHARD_STATS)
    with open(os.path.join(args.cases, 'rank%d.json' % sh.rank), 'w') as f:
        json.dump(stats, f)
    import torch.distributed as dist
    dist.destroy_process_group()


if __name__ == '__main__':
    main()
