"""The file assembly of a sharded run on the CPU (gloo, world sizes 2 and 3):
every rank formats the rows of its own contiguous block of reads and rank 0
writes them, and the bytes must be the ones a single GPU writes.

- prelim.csv (prelim_map.py:142-151): rname groups in global first-seen
  order, FASTQ order within a group (micall_amd.prelim_map._write_sharded
  against grouped_order over the whole set);
- remap.csv rows / unmapped FASTQs (remap.py:612-634): rank order
  (micall_amd.remap._emit);
- the split references' global order (Shard.all_gather_bytes).

A fake context stands in for the device: it formats read i as one text line
from the global list, so the test sees exactly which rows went where."""
import io
import os
import socket

import numpy as np
import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

from micall_amd import prelim_map as pm
from micall_amd import remap as rm
from micall_amd import session
from micall_amd.pipeline import Shard

N_READS = 1001          # not a multiple of the world size
N_REFS = 7


def _global_refs():
    rng = np.random.default_rng(3)
    # a few rnames, '*' (-1) among them, first seen at scattered places
    return rng.choice(np.arange(-1, N_REFS), size=N_READS, p=[0.1] + [0.9 / N_REFS] * N_REFS)


def _line(i, ref):
    return ('q%d,%d,ref%d\n' % (i, i % 7, ref)).encode()


class _RowsCtx:
    def __init__(self, refs, lo):
        self.refs, self.lo = refs, lo

    def format_rows_bytes(self, style, first=0, n=None, order=None):
        assert style == 1
        return b''.join(_line(self.lo + int(i), self.refs[self.lo + int(i)]) for i in order)


def _block(rank, world, n):
    return n * rank // world, n * (rank + 1) // world


def _worker(rank, world, port, out_dir):
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port))
    dist.init_process_group('gloo', rank=rank, world_size=world)
    try:
        refs = _global_refs()
        lo, hi = _block(rank, world, N_READS)
        sh = Shard(rank, world, read_base=lo)
        ctx = _RowsCtx(refs, lo)
        # prelim.csv groups
        out = io.StringIO()
        pm._write_sharded(ctx, sh, refs[lo:hi], N_REFS, out)
        # remap.csv rows / unmapped reads in rank order, two outputs at once
        a, b = io.StringIO(), io.StringIO()
        mine = [('r%d\n' % i).encode() for i in range(lo, hi)]
        rm._emit(sh, [(a, b''.join(mine)), (b, b''.join(mine[::2]))])
        # split references: first-split order over the ranks
        names = ['s%d' % ((i * 7) % 5) for i in range(lo, hi, 97)]
        seen = []
        for text in sh.all_gather_bytes('\n'.join(dict.fromkeys(names)).encode()):
            for name in text.decode().split('\n') if text else []:
                if name not in seen:
                    seen.append(name)
        if rank == 0:
            want = b''.join(_line(i, refs[i]) for i in pm.grouped_order(refs)).decode()
            assert out.getvalue() == want
            assert a.getvalue() == ''.join('r%d\n' % i for i in range(N_READS))
            want_b = ''.join(''.join('r%d\n' % i for i in range(*_block(r, world, N_READS))[::2])
                             for r in range(world))
            assert b.getvalue() == want_b
            all_names = ['s%d' % ((i * 7) % 5) for r in range(world)
                         for i in range(_block(r, world, N_READS)[0], _block(r, world, N_READS)[1], 97)]
            assert seen == list(dict.fromkeys(all_names))
            open(os.path.join(out_dir, 'ok'), 'w').close()
        else:
            assert out.getvalue() == '' and a.getvalue() == '' and b.getvalue() == ''
    finally:
        dist.destroy_process_group()


def _free_port():
    with socket.socket() as s:
        s.bind(('127.0.0.1', 0))
        return s.getsockname()[1]


@pytest.mark.timeout(300)
@pytest.mark.parametrize('world', [2, 3])
def test_sharded_outputs_equal_single_gpu_gloo(tmp_path, world):
    mp.spawn(_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True)
    assert (tmp_path / 'ok').exists()


def test_writer_and_block_rule_without_a_group():
    """Outside a process group the drop-ins write everything themselves."""
    assert session.shard() is None
    assert session.is_writer()
