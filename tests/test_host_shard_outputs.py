"""The file assembly of a sharded run on the CPU (gloo, world sizes 2 and 3):
every rank formats the rows of its own contiguous block of reads and writes
them at its offsets of the shared file (sharded_io.SharedOutput: sizes
all-gathered, pwrite), or -- when the handles are not one plain file on every
rank -- sends them to rank 0, which writes them.  The bytes must be the ones
a single GPU writes.

- prelim.csv (prelim_map.py:142-151): rname groups in global first-seen
  order, FASTQ order within a group (prelim_map.grouped_segments over the
  ranks against grouped_order over the whole set), and the crc32 the job
  computes for it without reading it back;
- remap.csv rows / unmapped FASTQs (remap.py:612-634): rank order;
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
from micall_amd import session, sharded_io
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
    """format_rows_bytes / format_segments / write_segments of the device
    context over text lines (the segments API formats, keeps, then writes at
    the given file offsets)."""

    def __init__(self, refs, lo):
        self.refs, self.lo = refs, lo
        self.kept = None

    def _text(self, order):
        return b''.join(_line(self.lo + int(i), self.refs[self.lo + int(i)]) for i in order)

    def format_rows_bytes(self, style, first=0, n=None, order=None):
        assert style == 1
        return self._text(order)

    def format_segments(self, style, order, seg_rows):
        assert style == 1
        self.kept = [self._text(order[a:b]) for a, b in zip(seg_rows[:-1], seg_rows[1:])]
        return np.array([len(t) for t in self.kept], dtype=np.int64)

    def write_segments(self, fd, offsets, crc=True):
        import zlib
        for t, off in zip(self.kept, offsets):
            os.pwrite(fd, t, int(off))
        return np.array([zlib.crc32(t) for t in self.kept], dtype=np.uint32)


def _block(rank, world, n):
    return n * rank // world, n * (rank + 1) // world


def _worker(rank, world, port, out_dir):
    import zlib
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port))
    dist.init_process_group('gloo', rank=rank, world_size=world)
    try:
        refs = _global_refs()
        lo, hi = _block(rank, world, N_READS)
        sh = Shard(rank, world, read_base=lo)
        ctx = _RowsCtx(refs, lo)
        want = b''.join(_line(i, refs[i]) for i in pm.grouped_order(refs))
        head = b'qname,flag,rname\n'
        for direct in (True, False):
            # prelim.csv groups: every rank opened the file, rank 0 wrote the header
            path = os.path.join(out_dir, 'prelim%d.csv' % direct)
            f = open(path, 'w') if direct else io.StringIO()
            sh.barrier()
            if rank == 0:
                f.write(head.decode())
            out = sharded_io.SharedOutput(sh, f)
            assert out.direct == direct
            order, bounds = pm.grouped_segments(refs[lo:hi], N_REFS, sh)
            out.write_rows(ctx, 1, order, bounds)
            sh.barrier()
            out.finish()
            crc = out.crc_of_file(head) if out.direct else None
            if direct:
                f.close()
                text = open(path, 'rb').read()
                assert text == head + want
                assert crc == (zlib.crc32(text), len(text))
            elif rank == 0:
                assert f.getvalue().encode() == head + want
            else:
                assert f.getvalue() == ''
        # remap.csv rows / unmapped reads in rank order, two outputs at once
        a, b = io.StringIO(), io.StringIO()
        pa = os.path.join(out_dir, 'rows.csv')
        fa = open(pa, 'w')
        sh.barrier()
        mine = [('r%d\n' % i).encode() for i in range(lo, hi)]
        outs = [sharded_io.SharedOutput(sh, h) for h in (a, b, fa)]
        outs[0].write_bytes([b''.join(mine)])
        outs[1].write_bytes([b''.join(mine[::2])])
        outs[2].write_bytes([b''.join(mine)])
        outs[2].write_bytes([b''.join(mine[::3])])
        sh.barrier()
        for o in outs:
            o.finish()
        fa.close()
        # split references: first-split order over the ranks
        names = ['s%d' % ((i * 7) % 5) for i in range(lo, hi, 97)]
        seen = []
        for text in sh.all_gather_bytes('\n'.join(dict.fromkeys(names)).encode()):
            for name in text.decode().split('\n') if text else []:
                if name not in seen:
                    seen.append(name)
        if rank == 0:
            assert a.getvalue() == ''.join('r%d\n' % i for i in range(N_READS))
            want_b = ''.join(''.join('r%d\n' % i for i in range(*_block(r, world, N_READS))[::2])
                             for r in range(world))
            assert b.getvalue() == want_b
            want_rows = ''.join('r%d\n' % i for i in range(N_READS)) + ''.join(
                ''.join('r%d\n' % i for i in range(*_block(r, world, N_READS))[::3])
                for r in range(world))
            assert open(pa).read() == want_rows
            all_names = ['s%d' % ((i * 7) % 5) for r in range(world)
                         for i in range(_block(r, world, N_READS)[0], _block(r, world, N_READS)[1], 97)]
            assert seen == list(dict.fromkeys(all_names))
            open(os.path.join(out_dir, 'ok'), 'w').close()
        else:
            assert a.getvalue() == '' and b.getvalue() == ''
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


def _stage_worker(rank, world, port, out_dir):
    """session.writer_stage under gloo: rank 0 writes, the others wait and
    see the complete file after the stage; a failure on rank 0 is raised on
    every rank."""
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port), WORLD_SIZE=str(world),
                      RANK=str(rank), LOCAL_RANK=str(rank), MICALL_DIST_BACKEND='gloo')
    dist.init_process_group('gloo', rank=rank, world_size=world)
    try:
        session._shard_checked = False
        session._shard = None
        sh = Shard(rank, world, 0)
        session._shard, session._shard_checked = sh, True
        path = os.path.join(out_dir, 'stage.csv')
        with open(path, 'w') as f:
            with session.writer_stage(f) as st:
                assert st.active == (rank == 0)
                if st.active:
                    f.write('a,b\n' * 1000)
            assert open(path).read() == 'a,b\n' * 1000      # complete on every rank
        raised = None
        try:
            with session.writer_stage() as st:
                if st.active:
                    raise ValueError('rank 0 fails')
        except Exception as ex:
            raised = type(ex).__name__
        assert raised == ('ValueError' if rank == 0 else 'RuntimeError'), raised
        open(os.path.join(out_dir, 'ok%d' % rank), 'w').close()
    finally:
        session._shard, session._shard_checked = None, False
        dist.destroy_process_group()


@pytest.mark.timeout(300)
@pytest.mark.parametrize('world', [2, 3])
def test_writer_stage_barriers_and_failures_gloo(tmp_path, world):
    mp.spawn(_stage_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True)
    assert all((tmp_path / ('ok%d' % r)).exists() for r in range(world))
