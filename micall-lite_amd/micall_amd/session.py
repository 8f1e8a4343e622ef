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
same paths and then calls the drop-ins with the same arguments; rank 0
writes the output files, in the order a single GPU writes them (each drop-in
starts with a barrier, so no rank's open can truncate what rank 0 wrote).
"""
import os

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
    sharded job only this rank's block of units is resident, and the
    shard's read_base is the block's first read."""
    global _key
    sh = shard()
    ctx = context()
    key = _file_key(fastq1, fastq2)
    if key != _key:
        if sh is None:
            ctx.reads_load_fastq(fastq1, fastq2)
        else:
            _n, first_unit = ctx.reads_load_fastq_part(fastq1, fastq2, sh.rank, sh.world)
            sh.read_base = 2 * first_unit if fastq2 else first_unit
        _key = key
        ctx.fastq_line_count = ctx.fastq_lines()
    return ctx


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


def _identity(handle):
    """(device, inode, size) of an open file, None for a non-file stream."""
    try:
        handle.flush()
        st = os.fstat(handle.fileno())
    except (AttributeError, OSError, ValueError):
        return None
    return st.st_dev, st.st_ino, st.st_size


def write_bytes(handle, data):
    """Write ASCII bytes to an open text file (through its binary buffer when
    it is a UTF-8 / ASCII file that writes '\n' as is)."""
    raw = getattr(handle, 'buffer', None)
    enc = (getattr(handle, 'encoding', '') or '').lower().replace('-', '')
    if (raw is not None and enc in ('utf8', 'ascii') and os.linesep == '\n' and
            getattr(handle, '_writenl', None) in (None, '\n')):
        handle.flush()
        raw.write(data)
    else:
        handle.write(bytes(data).decode())


def _written_checksum(handle):
    """Checksum of the file behind a handle opened for writing (read back
    through its path, after checking that the path is still that file)."""
    ident = _identity(handle)
    name = getattr(handle, 'name', None)
    if ident is None or not isinstance(name, str):
        return None, None
    try:
        fd = os.open(name, os.O_RDONLY)
    except OSError:
        return None, None
    try:
        st = os.fstat(fd)
        if (st.st_dev, st.st_ino) != ident[:2]:
            return None, None
        return ident, _native.file_checksum(fd)
    finally:
        os.close(fd)


def prelim_written(ctx, handle, seed_names):
    """Record that prelim_map() wrote `handle` from the device records that
    are resident now (ctx.map_serial) for these seeds."""
    global _prelim
    ident, sums = _written_checksum(handle) if is_writer() else (None, None)
    _prelim = dict(identity=ident, checksum=sums, serial=ctx.map_serial, key=_key,
                   seeds=list(seed_names))


def prelim_resident(ctx, handle, seed_names):
    """True when `handle` is the prelim.csv this process's last prelim_map()
    wrote, unchanged (the same file, size and crc32 / adler32 of its
    content), and that pass's records are still resident: remap() then
    takes the prelim rows from the device instead of parsing them again.  In
    a sharded job rank 0 checks the file and every rank its own records."""
    p = _prelim
    ok = (p is not None and p['serial'] == ctx.map_serial and p['key'] == _key and
          p['key'] is not None and p['seeds'] == list(seed_names))
    if ok and is_writer():
        ok = p['identity'] is not None and _identity(handle) == p['identity']
        if ok:
            try:
                ok = _native.file_checksum(handle.fileno()) == p['checksum']
            except (OSError, ValueError, _native.NativeError):
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
