"""Child process of tests/test_gpu_shard_chain.py: one rank of a sharded
bin/micall run_sample (/root/reference/bin/micall:91-192) with the drop-ins
in place of micall.core.*.

Every call, every open and every handle is bin/micall's: the InterOp reports
(:104-114), censor of R1 and then R2 with the exhausted bad-cycles reader
(:116-127; the censored files' handles are never closed), prelim_map (:143-154),
remap (:157-169), sam2aln (:172-175) and aln2counts (:178-188, the amino,
insert and conseq handles never closed).  Every rank opens every file, as
every rank of a torchrun job runs the same script.  The cleanup of :190-192
is left out (keep): each rank would remove the same files.

The rank reads RANK / WORLD_SIZE / MASTER_* from the environment as under
torchrun; micall_amd.session initialises the process group (gloo here: the
ranks share the test box's one GPU)."""
import argparse
import csv
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, 'micall-lite_amd'))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('fastq1')
    ap.add_argument('fastq2', nargs='?')
    ap.add_argument('--interop')
    ap.add_argument('--readlen', type=int, default=251)
    ap.add_argument('--index', type=int, default=8)
    ap.add_argument('--outdir', required=True)
    args = ap.parse_args()

    from micall_amd.aln2counts import aln2counts
    from micall_amd.censor_fastq import censor
    from micall_amd.filter_quality import report_bad_cycles
    from micall_amd.parse_interop import read_errors, write_phix_csv
    from micall_amd.prelim_map import prelim_map
    from micall_amd.remap import remap
    from micall_amd.sam2aln import sam2aln
    from micall_amd import session, sharded_io

    prefix = os.path.basename(args.fastq1).replace('.fastq.gz', '')
    fastq1 = open(args.fastq1, 'rb')
    fastq2 = open(args.fastq2, 'rb') if args.fastq2 else None
    stats = {}
    if args.interop:
        # censor_fastqs (bin/micall:91-129)
        lengths = [args.readlen, args.index, args.index, args.readlen]
        records = read_errors(open(args.interop, 'rb'))
        quality_csv = os.path.join(args.outdir, prefix + '.quality.csv')
        with open(quality_csv, 'w') as handle:
            write_phix_csv(out_file=handle, records=records, read_lengths=lengths)
        bad_cycles_csv = os.path.join(args.outdir, prefix + '.bad_cycles.csv')
        with open(quality_csv, 'r') as f1, open(bad_cycles_csv, 'w') as f2:
            report_bad_cycles(f1, f2)
        bad_cycles = csv.DictReader(open(bad_cycles_csv, 'r'))
        sharded_io.reset_stats()
        cfastq1 = fastq1.name.replace('.fastq', '.censor.fastq')
        censor(src=fastq1, bad_cycles_reader=bad_cycles, dest=open(cfastq1, 'wb'), use_gzip=True)
        fastq1 = open(cfastq1, 'rb')
        if fastq2:
            cfastq2 = fastq2.name.replace('.fastq', '.censor.fastq')
            censor(fastq2, bad_cycles, open(cfastq2, 'wb'), True)
            fastq2 = open(cfastq2, 'rb')
        stats['censor'] = dict(sharded_io.IO_STATS)

    sharded_io.reset_stats()
    prelim_csv = os.path.join(args.outdir, prefix + '.prelim.csv')
    with open(prelim_csv, 'w') as handle:
        prelim_map(fastq1=fastq1.name, fastq2=fastq2.name if fastq2 else None, prelim_csv=handle,
                   gzip=True, bt2_path='bowtie2', bt2build_path='bowtie2-build-s', nthreads=4,
                   keep=False, json=None)
    stats['prelim_map'] = dict(sharded_io.IO_STATS)
    sharded_io.reset_stats()
    remap_csv = os.path.join(args.outdir, prefix + '.remap.csv')
    with open(remap_csv, 'w') as handle:
        remap(fastq1=fastq1.name, fastq2=fastq2.name if fastq2 else None,
              prelim_csv=open(prelim_csv), remap_csv=handle, gzip=True, bt2_path='bowtie2',
              bt2build_path='bowtie2-build-s', nthreads=4, keep=False, json=None)
    stats['remap'] = dict(sharded_io.IO_STATS)
    stats['prelim_source'] = session.stats.get('prelim_source')
    align_csv = os.path.join(args.outdir, prefix + '.align.csv')
    with open(align_csv, 'w') as handle:
        sam2aln(remap_csv=open(remap_csv), aligned_csv=handle)
    nuc_csv = os.path.join(args.outdir, prefix + '.nuc.csv')
    amino_csv = os.path.join(args.outdir, prefix + '.amino.csv')
    insert_csv = os.path.join(args.outdir, prefix + '.insert.csv')
    conseq_csv = os.path.join(args.outdir, prefix + '.conseq.csv')
    with open(nuc_csv, 'w') as handle:
        aln2counts(aligned_csv=open(align_csv), nuc_csv=handle, amino_csv=open(amino_csv, 'w'),
                   coord_ins_csv=open(insert_csv, 'w'), conseq_csv=open(conseq_csv, 'w'),
                   json=None)
    sh = session.shard()
    stats.update(rank=sh.rank if sh else 0, world=sh.world if sh else 1,
                 read_base=sh.read_base if sh else 0,
                 reads=session.context().reads_count()[0])
    with open(os.path.join(args.outdir, 'rank%d.json' % stats['rank']), 'w') as f:
        json.dump(stats, f)
    if sh is not None:
        import torch.distributed as dist
        dist.destroy_process_group()


if __name__ == '__main__':
    main()
