"""Child process of tests/test_gpu_shard_aln2counts.py: one rank of a
sharded aln2counts over many aligned.csv files, on cuda:0 (gloo: the ranks
share the test box's one GPU).  For each case directory under --cases it
calls the drop-in as bin/micall does (every rank opens aligned.csv and the
outputs; a projects.json beside aligned.csv is passed as json) and records
how the call ran (micall_amd.aln2counts.SHARD_STATS).  For cases named
'single_*' rank 0 first runs the unsharded computation into *.single files,
the expectation of the test."""
import argparse
import io
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, 'micall-lite_amd'))
OUTS = ('nuc', 'amino', 'coord_ins', 'conseq', 'failed', 'coverage')


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--cases', required=True)
    args = ap.parse_args()
    if os.environ.get('MICALL_TEST_STACKS') == '1':
        import faulthandler
        faulthandler.dump_traceback_later(60, repeat=True)
    from micall_amd import aln2counts as a2c
    from micall_amd import session
    sh = session.shard()
    t0 = time.time()
    stats = {}
    for case in sorted(os.listdir(args.cases)):
        d = os.path.join(args.cases, case)
        if not os.path.isdir(d):
            continue
        proj = os.path.join(d, 'projects.json')
        proj = proj if os.path.exists(proj) else None
        if case.startswith('single_') and sh.rank == 0:
            with open(os.path.join(d, 'aligned.csv')) as al:
                outs = {k: io.StringIO() for k in OUTS}
                a2c._aln2counts(al, outs['nuc'], outs['amino'], outs['coord_ins'], outs['conseq'],
                                outs['failed'], None, None, outs['coverage'], proj)
            for k, v in outs.items():
                with open(os.path.join(d, k + '.single'), 'w') as f:
                    f.write(v.getvalue())
        handles = {k: open(os.path.join(d, k + '.csv'), 'w') for k in OUTS}
        with open(os.path.join(d, 'aligned.csv')) as al:
            a2c.aln2counts(al, handles['nuc'], handles['amino'], handles['coord_ins'], handles['conseq'],
                           failed_align_csv=handles['failed'], coverage_summary_csv=handles['coverage'],
                           json=proj)
        for h in handles.values():
            h.close()
        stats[case] = dict(a2c.SHARD_STATS)
        print('rank %d %s %.1f s' % (sh.rank, case, time.time() - t0), file=sys.stderr, flush=True)
    with open(os.path.join(args.cases, 'rank%d.json' % sh.rank), 'w') as f:
        json.dump(stats, f)
    import torch.distributed as dist
    dist.destroy_process_group()


if __name__ == '__main__':
    main()
