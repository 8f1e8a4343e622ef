"""bench.py's FASTQ writer under a job of several ranks (CPU, gloo, world 2
and 3): every rank writes its own block of pairs into the shared files,
which must hold the blocks in rank order -- as many gzip members, or as ONE
gzip member whose deflate stream each rank writes for its block, primed with
the block before's last 32 KiB (bench.write_fastq_gz).  The single-member
file must decode (gzip, CRC-32 and size checked) to the concatenated text and
hold no member start but the first."""
import gzip
import os
import socket
import sys
import zlib

import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def _worker(rank, world, port, d, single):
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port))
    dist.init_process_group('gloo', rank=rank, world_size=world)
    try:
        import bench
        from micall_amd import synth
        from micall_amd.pipeline import Shard
        job = bench.Job(Shard(rank, world, 0))
        pairs = synth.make_pairs(400 + 50 * rank, genomes=bench.bench_genomes('pol'), genome_seed=3,
                                 read_seed=4, block=rank)
        p1, p2 = os.path.join(d, 'R1.fastq.gz'), os.path.join(d, 'R2.fastq.gz')
        bench.write_fastq_gz(pairs, p1, p2, threads=2, single=single, job=job)
        with open(os.path.join(d, 'text%d_1' % rank), 'wb') as f:
            f.write(b''.join(bench._fastq_records(pairs, 1)))
        with open(os.path.join(d, 'text%d_2' % rank), 'wb') as f:
            f.write(b''.join(bench._fastq_records(pairs, 2)))
    finally:
        dist.destroy_process_group()


def _port():
    with socket.socket() as s:
        s.bind(('127.0.0.1', 0))
        return s.getsockname()[1]


@pytest.mark.timeout(300)
@pytest.mark.parametrize('world', [2, 3])
@pytest.mark.parametrize('single', [False, True])
def test_shared_fastq_writer(tmp_path, world, single):
    from micall_amd import _native
    d = str(tmp_path)
    mp.spawn(_worker, args=(world, _port(), d, single), nprocs=world, join=True)
    for mate in (1, 2):
        blob = open(os.path.join(d, 'R%d.fastq.gz' % mate), 'rb').read()
        want = b''.join(open(os.path.join(d, 'text%d_%d' % (r, mate)), 'rb').read()
                        for r in range(world))
        assert gzip.decompress(blob) == want
        if single:
            # one member: a raw inflate of the stream ends exactly at the trailer
            z = zlib.decompressobj(31)
            assert z.decompress(blob) == want and z.eof and z.unused_data == b''
            assert not any(_native.Fastq.scan_part(os.path.join(d, 'R%d.fastq.gz' % mate), -1, r, world)[2]
                           for r in range(world))
        else:
            assert blob.count(b'\x1f\x8b\x08') >= 2 * world
