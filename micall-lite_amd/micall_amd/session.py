"""
Process-wide device context and resident-read cache.

bin/micall calls prelim_map() and then remap() on the same FASTQ files
(bin/micall:142-169); the reference re-reads and re-decompresses them in
bowtie2 on every pass.  Here the first call ingests them into HBM and later
calls on the same (unchanged) files reuse the resident reads.

Sharded runs.  When the process is one rank of a torch.distributed job with
more than one rank (a process group already initialised, or torchrun's
WORLD_SIZE > 1 in the environment, in which case the group is initialised
here over MICALL_DIST_BACKEND, default nccl = RCCL), every rank keeps its
own contiguous block of read pairs resident (mh_reads_load_fastq_part) and
the drop-ins exchange counters through pipeline.Shard.  Every rank opens the
same paths and then calls the drop-ins with the same arguments.  The large
outputs (prelim.csv, remap.csv, the censored FASTQs, the unmapped FASTQs)
are written by every rank: each `pwrite`s its own rows at offsets
all-gathered from every rank's byte counts, so the file holds the rows in
the order a single GPU writes them (sharded_io.py).  The small reports
(remap_counts.csv, remap_conseq.csv, the InterOp CSVs) are written by rank
0 (writer_stage).  Each drop-in starts with a barrier, so no rank's open can
truncate what another rank wrote.
"""
import os
import sys
import time

from . import _native

_ctx = None
_key = None
_shard = None
_shard_checked = False
_prelim = None     # what the last prelim_map() of this process wrote (prelim_written)
stats = {}         # how the last calls ran (remap: 'prelim_source' = 'device' or 'csv')


def _device_index():
    if 'MICALL_HIP_DEVICE' in os.environ:
        return int(os.environ['MICALL_HIP_DEVICE'])
    if int(os.environ.get('WORLD_SIZE', '1')) > 1:
        return int(os.environ.get('LOCAL_RANK', '0'))
    return 0


def context():
    global _ctx
    if _ctx is None:
        _ctx = _native.Context(_device_index())
    return _ctx


def shard():
    """This rank's pipeline.Shard in a sharded job, None otherwise."""
    global _shard, _shard_checked
    if _shard_checked:
        return _shard
    _shard_checked = True
    import sys
    if 'torch' not in sys.modules and int(os.environ.get('WORLD_SIZE', '1')) <= 1:
        return None          # no process group can exist: skip importing torch
    try:
        import torch
        import torch.distributed as dist
    except ImportError:
        return None
    if not dist.is_available():
        return None
    if not dist.is_initialized():
        if int(os.environ.get('WORLD_SIZE', '1')) <= 1:
            return None
        torch.cuda.set_device(_device_index())
        dist.init_process_group(os.environ.get('MICALL_DIST_BACKEND', 'nccl'))
    if dist.get_world_size() <= 1:
        return None
    from .pipeline import Shard
    # torch's HIP runtime must come up before this library's context does
    # (load_fastq asks for the shard first); device buffers then carry the
    # pileup exchange
    torch.cuda.set_device(_device_index())
    _shard = Shard(dist.get_rank(), dist.get_world_size(), 0,
                   device=torch.device('cuda', _device_index()))
    return _shard


def is_writer():
    """True on the process that writes the output files (rank 0)."""
    sh = shard()
    return sh is None or sh.rank == 0


def _file_key(*paths):
    out = []
    for p in paths:
        if p is None:
            out.append(None)
        else:
            st = os.stat(p)
            out.append((os.path.abspath(p), st.st_mtime_ns, st.st_size))
    return tuple(out)


def load_fastq(fastq1, fastq2=None):
    """The context with these FASTQ files resident (loaded once).  In a
    sharded job only this rank's block of units is resident (read from its
    share of the files, sharded_io.load_reads), and the shard's read_base is
    the block's first read."""
    global _key
    sh = shard()
    ctx = context()
    key = _file_key(fastq1, fastq2)
    if key != _key:
        if sh is None:
            ctx.reads_load_fastq(fastq1, fastq2)
        else:
            from . import sharded_io
            first_unit = sharded_io.load_reads(ctx, sh, fastq1, fastq2)
            sh.read_base = 2 * first_unit if fastq2 else first_unit
        _key = key
        ctx.fastq_line_count = ctx.fastq_lines()
    return ctx


class writer_stage:
    """A stage that one process computes and writes while the other ranks of
    a sharded job wait (sam2aln, aln2counts, the InterOp reports).  Every rank
    opened (and so truncated) the stage's output files before the call,
    as bin/micall does on every rank: the entry barrier keeps rank 0 from
    writing before the last of those opens; on exit rank 0 flushes the given
    handles and the barrier holds the others until the files are complete.
    A failure on rank 0 is raised on every rank.  `active` is True on the
    process that does the work.

        with session.writer_stage(out1, out2) as st:
            if st.active:
                ...compute and write..."""

    def __init__(self, *handles):
        self.handles = handles
        self.sh = shard()
        self.active = self.sh is None or self.sh.rank == 0

    def __enter__(self):
        if self.sh is not None:
            self.sh.barrier()
        return self

    def __exit__(self, exc_type, exc, tb):
        if self.active:
            for h in self.handles:
                flush = getattr(h, 'flush', None)
                if flush is not None and not getattr(h, 'closed', False):
                    flush()
        if self.sh is not None:
            if exc_type is not None:
                # shown here: a rank that fails between the stage's
                # collectives leaves the others waiting in one of them
                import traceback
                sys.stderr.write('rank {}: the stage failed\n{}'.format(
                    self.sh.rank, ''.join(traceback.format_exception(exc_type, exc, tb))))
                sys.stderr.flush()
            failed = int(self.sh.sum_i64([1 if exc_type is not None else 0])[0])
            if failed and exc_type is None:
                raise RuntimeError('the stage failed on rank 0 of the sharded job')
        return False


def read_text(handle):
    """The rest of an open CSV/SAM text file for the native parsers: the raw
    bytes when nothing has read from it yet and it is UTF-8 / ASCII (no
    decode / encode round trip of a GB-sized file), with the newline
    translation text mode would have made ('\r\n' and '\r' -> '\n');
    otherwise handle.read()."""
    raw = getattr(handle, 'buffer', None)
    enc = (getattr(handle, 'encoding', '') or '').lower().replace('-', '')
    if raw is not None and enc in ('utf8', 'ascii') and getattr(handle, 'newlines', None) is None:
        try:
            fresh = handle.tell() == 0
        except (OSError, ValueError):
            fresh = False
        if fresh:
            data = raw.read()
            if b'\r' in data:
                data = data.replace(b'\r\n', b'\n').replace(b'\r', b'\n')
            return data
    return handle.read()


def readable_fd(handle):
    """The descriptor of an open text file whose whole content the native
    parsers may read straight from the file: nothing read from it yet,
    UTF-8 / ASCII, a regular file (what read_text would hand over as raw
    bytes); else None."""
    import stat
    raw = getattr(handle, 'buffer', None)
    enc = (getattr(handle, 'encoding', '') or '').lower().replace('-', '')
    if raw is None or enc not in ('utf8', 'ascii') or getattr(handle, 'newlines', None) is not None:
        return None
    try:
        if handle.tell() != 0:
            return None
        fd = handle.fileno()
        return fd if stat.S_ISREG(os.fstat(fd).st_mode) else None
    except (OSError, ValueError, AttributeError):
        return None


def write_bytes(handle, data):
    """Write ASCII bytes to an open text file (through its binary buffer when
    it is a UTF-8 / ASCII file that writes '\n' as is), or to a binary one."""
    import io
    if not isinstance(handle, io.TextIOBase) and 'b' in getattr(handle, 'mode', 'b'):
        handle.write(bytes(data))
        return
    raw = getattr(handle, 'buffer', None)
    enc = (getattr(handle, 'encoding', '') or '').lower().replace('-', '')
    if (raw is not None and enc in ('utf8', 'ascii') and os.linesep == '\n' and
            getattr(handle, '_writenl', None) in (None, '\n')):
        handle.flush()
        raw.write(data)
    else:
        handle.write(bytes(data).decode())


def _file_identity(handle):
    """(device, inode, size, mtime, ctime) of the file behind an open
    handle, None for a non-file stream.  ctime cannot be set from user
    space: any later write to the file changes it."""
    try:
        st = os.fstat(handle.fileno())
    except (AttributeError, OSError, ValueError):
        return None
    return st.st_dev, st.st_ino, st.st_size, st.st_mtime_ns, st.st_ctime_ns


def _wait_past(ctime_ns, limit_s=0.05):
    """Return once the kernel's coarse clock, which stamps file changes, has
    moved past `ctime_ns` (at most one timer tick, a few ms).  A later
    rewrite of the file then gets a newer ctime, so an unchanged identity
    proves unchanged content: a same-size rewrite inside the tick of our
    last write cannot pass for our file.  False when that could not be
    established (the identity alone is then not trusted)."""
    clock = getattr(time, 'CLOCK_REALTIME_COARSE', None)
    if clock is None:
        return False
    deadline = time.monotonic() + limit_s
    while time.clock_gettime_ns(clock) <= ctime_ns:
        if time.monotonic() >= deadline:
            return False
        time.sleep(0.0005)
    return True


def prelim_written(ctx, handle, seed_names, checksum=None):
    """Record that prelim_map() wrote `handle` from the device records that
    are resident now (ctx.map_serial) for these seeds: the file's identity
    after the last write and, when known, (crc32, size) of its content as
    formatted (no read-back)."""
    global _prelim
    ident = None
    settled = False
    if is_writer():
        try:
            handle.flush()
        except (AttributeError, OSError, ValueError):
            pass
        ident = _file_identity(handle)
        settled = ident is not None and _wait_past(ident[4])
    _prelim = dict(identity=ident, settled=settled, checksum=checksum, serial=ctx.map_serial, key=_key,
                   seeds=list(seed_names))


def prelim_resident(ctx, handle, seed_names):
    """True when `handle` is the prelim.csv this process's last prelim_map()
    wrote, unchanged, and that pass's records are still resident: remap()
    then takes the prelim rows from the device instead of parsing them
    again.  Unchanged: the same file identity (device, inode, size, mtime,
    ctime); failing that, the same size and crc32 as the rows formatted (a
    file rewritten with the same bytes; read back only then).  In a sharded
    job rank 0 checks the file and every rank its own records."""
    p = _prelim
    ok = (p is not None and p['serial'] == ctx.map_serial and p['key'] == _key and
          p['key'] is not None and p['seeds'] == list(seed_names))
    if ok and is_writer():
        ident = _file_identity(handle)
        ok = ident is not None and p['identity'] is not None
        if ok and (ident != p['identity'] or not p['settled']):
            ok = False
            want = p['checksum']
            if want is not None and ident[2] == want[1] and ident[:2] == p['identity'][:2]:
                try:
                    ok = _native.file_crc32(handle.fileno()) == (want[1], want[0])
                except (OSError, ValueError, _native.NativeError):
                    ok = False
        if ok:
            try:
                ok = handle.tell() == 0
            except (OSError, ValueError):
                ok = False
    sh = shard()
    if sh is not None:
        ok = bool(sh.min_i64([1 if ok else 0])[0])
    return ok


def invalidate():
    """The resident reads were replaced (e.g. by split re-mapping)."""
    global _key, _prelim
    _key = None
    _prelim = None


def reset():
    """Close the process-wide context (the next call creates a new one)."""
    global _ctx, _key, _prelim
    if _ctx is not None:
        _ctx.close()
    _ctx = None
    _key = None
    _prelim = None
