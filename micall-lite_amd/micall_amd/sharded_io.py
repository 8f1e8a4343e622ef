"""
File input and output of a sharded job (one process per GPU under torchrun).

The reference reads each FASTQ once per bowtie2 pass and writes every output
file from its one process (prelim_map.py:114-151, remap.py:612-658,
censor_fastq.py:58-96).  In a job of W ranks each rank here

  * reads its 1/W share of every FASTQ file (`stage_fastq`): the gzip members
    that start in its byte range (a plain file: the byte range; a file that is
    one gzip member, as bcl2fastq writes it: the deflate blocks that start in
    its share of the compressed bytes, `_open_members`), frames the text into
    four-line records from the line counts of the ranks before it, passes the
    bytes in front of its first record to the rank before, and, for a pair of
    files, exchanges whole records so that its R1 and R2 blocks hold the same
    reads.  A file that cannot be split (a blank line where a record starts;
    a member with no block start in some rank's share) is decoded whole by
    every rank, which keeps its records by count;
  * writes its own rows of every output file (`SharedOutput`) with pwrite at
    offsets computed from the all-gathered segment sizes, so the file holds
    the rows in single-GPU order (segment 0 of rank 0, rank 1, ..., then
    segment 1, ...) and no rank's text travels to another.

Counters (bytes decoded, bytes written) go to `IO_STATS` so a test can check
that each rank did about 1/W of the work.
"""
import os
from concurrent.futures import ThreadPoolExecutor

import numpy as np

from . import _native

IO_STATS = dict(fastq_file_bytes=0, fastq_text_bytes=0, fastq_mode=None, written_bytes=0)


def reset_stats():
    IO_STATS.update(fastq_file_bytes=0, fastq_text_bytes=0, fastq_mode=None, written_bytes=0)


# ---- collective helpers ------------------------------------------------------
def _agree_ok(sh, ok):
    """True on every rank when `ok` holds on every rank."""
    return bool(sh.min_i64([1 if ok else 0])[0])


def _checked(sh, fn):
    """Run fn() on every rank; if it raises on any rank, raise on all of them
    (so no rank waits in a collective for one that failed)."""
    err = None
    try:
        out = fn()
    except Exception as ex:    # re-raised below, after the agreement
        err, out = ex, None
    if not _agree_ok(sh, err is None):
        if err is not None:
            raise err
        raise _native.NativeError('the call failed on another rank of the job')
    return out


def _p2p(sh, sends, recv_sizes):
    """Point-to-point exchange of byte blocks: sends = {peer: uint8 array},
    recv_sizes = {peer: bytes}; returns {peer: bytes received}."""
    torch, dist = sh.torch, sh.dist
    dev = sh._text_device()
    ops, bufs, keep = [], {}, []
    for peer, n in sorted(recv_sizes.items()):
        if n > 0:
            t = torch.empty(int(n), dtype=torch.uint8, device=dev)
            bufs[peer] = t
            ops.append(dist.P2POp(dist.irecv, t, peer))
    for peer, data in sorted(sends.items()):
        if len(data) > 0:
            t = torch.from_numpy(np.array(data, dtype=np.uint8, copy=True)).to(dev)
            keep.append(t)
            ops.append(dist.P2POp(dist.isend, t, peer))
    if ops:
        for req in dist.batch_isend_irecv(ops):
            req.wait()
    return {peer: t.cpu().numpy().tobytes() for peer, t in bufs.items()}


def all_to_all_bytes(sh, data, sizes):
    """Every rank sends sizes[d] bytes of data (laid out by destination) to
    rank d; returns the bytes received, in source-rank order (uint8)."""
    torch, dist = sh.torch, sh.dist
    sizes = np.asarray(sizes, dtype=np.int64)
    matrix = sh._gather_sizes(sizes)                     # [sender, receiver]
    recv = [int(matrix[s, sh.rank]) for s in range(sh.world)]
    if int(matrix.sum()) == 0:
        return np.zeros(0, dtype=np.uint8)
    dev = sh._text_device()
    src = np.ascontiguousarray(data, dtype=np.uint8)
    inp = torch.from_numpy(src) if dev.type == 'cpu' else torch.from_numpy(src).to(dev)
    out = torch.empty(sum(recv), dtype=torch.uint8, device=dev)
    dist.all_to_all_single(out, inp, recv, [int(x) for x in sizes])
    return out.cpu().numpy()


def qname_conflict(sh, hashes, leftover):
    """True on every rank when some qname that is left unpaired on one rank
    also has rows on another (then the ranks' matchmaker order is not the
    reference's over the whole file).  Each (qname hash, rank, leftover)
    goes to the rank that owns the hash, which looks for hashes held by two
    ranks with a leftover among them."""
    W = sh.world
    h = np.asarray(hashes, dtype=np.uint64)
    owner = (h % np.uint64(W)).astype(np.int64)
    order = np.argsort(owner, kind='stable')
    rec = np.empty((len(h), 2), dtype=np.int64)
    rec[:, 0] = h.view(np.int64)
    rec[:, 1] = (sh.rank << 1) | np.asarray(leftover, dtype=np.int64)
    rec = np.ascontiguousarray(rec[order])
    sizes = np.bincount(owner, minlength=W).astype(np.int64) * 16
    got = all_to_all_bytes(sh, rec.view(np.uint8).reshape(-1), sizes).view(np.int64).reshape(-1, 2)
    bad = False
    if len(got):
        o = np.lexsort((got[:, 1], got[:, 0]))
        hv, fl = got[o, 0], got[o, 1]
        start = np.r_[True, hv[1:] != hv[:-1]]
        gid = np.cumsum(start) - 1
        ng = int(gid[-1]) + 1
        rk = fl >> 1
        rmin = np.full(ng, np.iinfo(np.int64).max)
        rmax = np.full(ng, -1)
        np.minimum.at(rmin, gid, rk)
        np.maximum.at(rmax, gid, rk)
        left = np.zeros(ng, dtype=bool)
        np.logical_or.at(left, gid, (fl & 1) == 1)
        bad = bool(np.any((rmin != rmax) & left))
    return bool(sh.sum_i64([1 if bad else 0])[0])


# ---- FASTQ staging -------------------------------------------------------------
class _Frame:
    """One file's framing on this rank after the boundary exchange."""

    def __init__(self, fq, first, count, total, lines):
        self.fq, self.first, self.count, self.total, self.lines = fq, first, count, total, lines


def _open_members(sh, sources):
    """Each source file one gzip member: this rank's part of each, decoded
    from its own share of the compressed bytes (mh_fastq_member_*).

    1. every rank finds the first deflate block start in its share (rank 0:
       the stream's start) and the ranks all-gather them: rank r decodes up
       to rank r + 1's start, on its threads, with the window it lacks (the
       last 32 KiB of rank r - 1's text) left symbolic;
    2. the windows travel in rank order: rank r receives rank r - 1's
       resolved last 32 KiB of every file (one message), resolves its own
       last 32 KiB with it and sends them on to rank r + 1 (W - 1 messages
       of 32 KiB per file in all);
    3. every rank resolves the rest of its text in parallel and all-gathers
       the CRC-32 and size of its text: combined in rank order they must
       equal the gzip trailer's.

    Returns [Fastq or None] per source; None (on every rank) for a file that
    cannot be split this way (the caller then decodes it whole)."""
    W, r = sh.world, sh.rank
    n = len(sources)

    def each(fn, items):
        if len(items) <= 1:
            return [fn(x) for x in items]
        with ThreadPoolExecutor(len(items)) as ex:
            return list(ex.map(fn, items))
    fqs = _checked(sh, lambda: each(lambda src: _native.Fastq(src[0], src[1] if src[1] is not None
                                                               else -1, r, W, member=True), sources))
    starts = sh._gather_sizes([fq.info['first_bit'] for fq in fqs])        # [rank, source]
    ok = [bool((starts[:, k] >= 0).all()) and bool((np.diff(starts[:, k]) > 0).all()) for k in range(n)]

    def decode(k):
        if not ok[k]:
            return -1
        end = int(starts[r + 1, k]) if r + 1 < W else fqs[k].info['end_bit']
        return fqs[k].member_decode(end)
    sizes = _checked(sh, lambda: each(decode, list(range(n))))
    good = sh._gather_sizes([1 if sz >= 0 else 0 for sz in sizes]).min(axis=0)
    live = [k for k in range(n) if ok[k] and good[k]]
    windows = {k: None for k in live}
    resolved = {k: True for k in live}
    if live:
        torch, dist = sh.torch, sh.dist
        dev = sh._text_device()
        win = _native.Fastq.MEMBER_WINDOW
        if r > 0:
            t = torch.empty(win * len(live), dtype=torch.uint8, device=dev)
            dist.recv(t, src=r - 1)
            got = t.cpu().numpy()
            for j, k in enumerate(live):
                windows[k] = got[j * win:(j + 1) * win].tobytes()
        # Whatever goes wrong on this rank, rank r + 1 is blocked in recv
        # until a window arrives: a failed tail (any exception, not only the
        # library's) is sent on as zeros and marked unresolved, so the CRC
        # agreement below fails on every rank and the file is decoded whole.
        tails = []
        for k in live:
            try:
                tail = fqs[k].member_tail(windows[k])
                if tail is not None:
                    tail = np.asarray(tail, dtype=np.uint8).reshape(-1)
            except Exception:   # noqa: BLE001 -- the chain must not stall
                tail = None
            if tail is None or len(tail) != win:
                resolved[k] = False
                tail = np.zeros(win, dtype=np.uint8)
            tails.append(tail)
        if r + 1 < W:
            try:
                msg = np.concatenate(tails)
            except Exception:   # noqa: BLE001
                for k in live:
                    resolved[k] = False
                msg = np.zeros(win * len(live), dtype=np.uint8)
            dist.send(torch.from_numpy(msg).to(dev), dst=r + 1)

    def finish(k):
        if k not in resolved or not resolved[k]:
            return False
        c0 = 0 if r == 0 else int(starts[r, k]) // 8
        c1 = fqs[k].info['file_size'] if r + 1 == W else int(starts[r + 1, k]) // 8
        return fqs[k].member_finish(windows[k], c0, c1)
    done = _checked(sh, lambda: each(finish, list(range(n))))
    rows = sh._gather_sizes([v for k in range(n) for v in (
        1 if done[k] else 0, fqs[k].info.get('crc', 0) if done[k] else 0,
        fqs[k].info.get('bytes', 0) if done[k] else 0)]).reshape(W, n, 3)
    out = []
    for k in range(n):
        fine = bool(rows[:, k, 0].all())
        if fine:
            crc, total = 0, 0
            for q in range(W):
                crc = _native.crc32_combine(crc, int(rows[q, k, 1]), int(rows[q, k, 2]))
                total += int(rows[q, k, 2])
            fine = crc == fqs[k].info_member['crc'] and (total & 0xffffffff) == fqs[k].info_member['isize']
        if not fine:
            fqs[k].close()
            out.append(None)
        else:
            out.append(fqs[k])
    return out


def _open_all(sh, sources, part, parts):
    def one(src):
        path, fd = src
        return _native.Fastq(path, fd if fd is not None else -1, part, parts)
    if len(sources) == 1:
        return [one(sources[0])]
    with ThreadPoolExecutor(len(sources)) as ex:
        return list(ex.map(one, sources))


def _frame_sharded(sh, fq, strict):
    """Frame this rank's share of a file split by member / byte range and
    move the bytes before its first record to the rank before.  Returns a
    _Frame, or None when the split cannot be used (then no rank uses it)."""
    W, r = sh.world, sh.rank
    inf = fq.info
    rows = sh._gather_sizes([inf['mode'], inf['c0'], inf['c1'], inf['bytes'], inf['newlines'],
                             inf['ends_nl'], inf['starts_nl'], inf['file_size']])
    mode, c0, c1, nbytes, nl, ends_nl, starts_nl, size = (rows[:, k] for k in range(8))
    chain = (all(m in (1, 2, 3) for m in mode) and c0[0] == 0 and c1[W - 1] == size[0] and
             all(c1[k] == c0[k + 1] for k in range(W - 1)))
    if not chain:
        return None
    line0 = int(nl[:r].sum())
    starts_line = True
    for s in range(r - 1, -1, -1):     # the last non-empty part before this one
        if nbytes[s] > 0:
            starts_line = bool(ends_nl[s])
            break
    first_off, count, first_line, blank, tail_cr = fq.frame(line0, starts_line)
    fr = sh._gather_sizes([first_off, count, first_line, blank, tail_cr])
    counts, first_lines = fr[:, 1], fr[:, 2]
    blank_any = bool(fr[:, 3].any())
    for k in range(W - 1):   # a '\r'-only record-start line finished by the next part's '\n'
        if fr[k, 4] and starts_nl[k + 1]:
            blank_any = True
    mean = float(nbytes.sum()) / W
    usable = (all(counts > 0) and (strict or not blank_any) and
              float(nbytes.min()) >= 0.5 * mean and
              all(first_lines[k] == 4 * int(counts[:k].sum()) for k in range(W)))
    if not usable:
        return None
    prefix = fq.view(0, first_off).tobytes()
    prefixes = sh.all_gather_bytes(prefix)
    back = prefixes[r + 1] if r + 1 < W else b''
    fq.splice(first_off, fq.size(), back=back)
    fq.frame(0, True)   # local record offsets of the records now held
    return _Frame(fq, int(counts[:r].sum()), int(counts[r]), int(counts.sum()), int(nl.sum()))


def _frame_whole(fq, strict):
    """A whole file held by every rank: its records by four-line framing.
    None when a blank line sits where a record starts and the caller parses
    records as the ingest does (strict=False)."""
    _off, count, _line, blank, _tail = fq.frame(0, True)
    if blank and not strict:
        return None
    return _Frame(fq, 0, count, count, fq.info['newlines'])


def _keep_records(fr, lo, hi):
    """Cut a framed text down to its global records [lo, hi)."""
    a = fr.fq.record_offset(lo - fr.first)
    b = fr.fq.record_offset(hi - fr.first)
    fr.fq.splice(a, b)
    fr.fq.frame(0, True)
    fr.first, fr.count = lo, hi - lo


def _realign(sh, fr, target):
    """Exchange whole records so that this rank holds records target[rank]
    of a file whose ranks hold contiguous blocks in rank order."""
    W, r = sh.world, sh.rank
    held = sh._gather_sizes([fr.first, fr.first + fr.count])
    sends, send_sizes = {}, np.zeros(W, dtype=np.int64)
    for s in range(W):
        if s == r:
            continue
        o0, o1 = max(fr.first, target[s][0]), min(fr.first + fr.count, target[s][1])
        if o1 > o0:
            a, b = fr.fq.record_offset(o0 - fr.first), fr.fq.record_offset(o1 - fr.first)
            sends[s] = fr.fq.view(a, b)
            send_sizes[s] = b - a
    matrix = sh._gather_sizes(send_sizes)            # [sender, receiver]
    got = _p2p(sh, sends, {s: int(matrix[s, r]) for s in range(W) if s != r})
    t0, t1 = target[r]
    o0, o1 = max(fr.first, t0), min(fr.first + fr.count, t1)
    if o1 > o0:
        a, b = fr.fq.record_offset(o0 - fr.first), fr.fq.record_offset(o1 - fr.first)
    else:
        a = b = 0
    front = b''.join(got[s] for s in range(W) if s != r and held[s, 0] < fr.first and s in got)
    back = b''.join(got[s] for s in range(W) if s != r and held[s, 0] > fr.first and s in got)
    if o1 <= o0:   # nothing of our own: everything came from the others, in rank order
        front = b''.join(got[s] for s in range(W) if s in got)
        back = b''
    fr.fq.splice(a, b, front=front, back=back)
    fr.fq.frame(0, True)
    fr.first, fr.count = t0, t1 - t0


def stage_fastq(sh, sources, strict=False):
    """This rank's block of FASTQ records from every source file.

    sources: [(path, fd)] of one file (unpaired, or the censor's one file) or
    two (R1, R2; their blocks hold the same records).  strict=True frames
    every four lines as a record (the censor's zip_longest over lines,
    censor_fastq.py:58); otherwise a blank record-start line (which the
    ingest's parser skips) makes the files be read whole.

    Returns dict(frames=[_Frame per source], first=first record of the
    block, units=records in the block, total=records in the file,
    lines=newlines of source 0 (raw_count), mode='members'|'whole'); None
    when the ingest should fall back to the whole-file loader
    (mh_reads_load_fastq_part)."""
    W, r = sh.world, sh.rank
    n = len(sources)
    # which files are one gzip member: no rank finds a member start in its
    # byte range (each scans 1/W of the file)
    scans = _checked(sh, lambda: [_native.Fastq.scan_part(p, fd if fd is not None else -1, r, W)
                                  for p, fd in sources])
    flags = sh._gather_sizes([v for gz, _size, found in scans for v in (int(gz), int(found))])
    single = [bool(flags[0, 2 * k]) and not flags[:, 2 * k + 1].any() for k in range(n)]
    fqs = [None] * n
    tried_member = [k for k in range(n) if single[k]]
    if tried_member:
        for k, fq in zip(tried_member, _open_members(sh, [sources[k] for k in tried_member])):
            fqs[k] = fq
            if fq is not None:
                IO_STATS['fastq_file_bytes'] += fq.info['file_bytes_read']
    split = [k for k in range(n) if not single[k]]
    if split:
        opened = _checked(sh, lambda: _open_all(sh, [sources[k] for k in split], r, W))
        for k, fq in zip(split, opened):
            fqs[k] = fq
            IO_STATS['fastq_file_bytes'] += fq.info['file_bytes_read']
    # a single member that could not be split is read whole below (no
    # member-range decode first)
    frames = [None if fq is None else _checked(sh, lambda fq=fq: _frame_sharded(sh, fq, strict))
              for fq in fqs]
    member_split = any(f is not None and single[k] for k, f in enumerate(frames))
    if all(f is None for f in frames):
        for fq in fqs:
            if fq is not None:
                fq.close()
        if not strict:
            return None            # every rank reads the files whole (the part loader)
        fqs = _checked(sh, lambda: _open_all(sh, sources, 0, 1))
        IO_STATS['fastq_file_bytes'] += sum(fq.info['file_bytes_read'] for fq in fqs)
        frames = [_frame_whole(fq, strict) for fq in fqs]
        mode = 'whole'
    else:
        for k, f in enumerate(frames):
            if f is None:          # this one is read whole, its partner split
                if fqs[k] is not None:
                    fqs[k].close()
                whole = _checked(sh, lambda k=k: _open_all(sh, [sources[k]], 0, 1)[0])
                IO_STATS['fastq_file_bytes'] += whole.info['file_bytes_read']
                frames[k] = _frame_whole(whole, strict)
                if frames[k] is None:
                    for f2 in frames:
                        if f2 is not None:
                            f2.fq.close()
                    return None
        mode = 'member-part' if member_split else 'members'
    totals = [f.total for f in frames]
    if len(set(totals)) != 1:
        raise _native.NativeError('paired FASTQ files hold {} and {} reads'.format(*totals))
    total = totals[0]
    # the block of this rank: the first split file's, or the floor split
    lead = next((f for f in frames if f.total == total and f.count != f.total), None)
    if lead is not None:
        blocks = sh._gather_sizes([lead.first, lead.first + lead.count])
        target = [(int(a), int(b)) for a, b in blocks]
    else:
        target = [(total * k // W, total * (k + 1) // W) for k in range(W)]
    for f in frames:
        if f is lead:
            continue
        if f.count == f.total and W > 1:
            _keep_records(f, *target[r])       # held whole: keep the block
        else:
            _realign(sh, f, target)
    IO_STATS['fastq_text_bytes'] += sum(f.fq.size() for f in frames)
    IO_STATS['fastq_mode'] = mode
    return dict(frames=frames, first=target[r][0], units=target[r][1] - target[r][0], total=total,
                lines=frames[0].lines, mode=mode)


def load_reads(ctx, sh, path1, path2=None):
    """The sharded ingest of prelim_map / remap: this rank's block of pairs
    (or reads) resident in ctx.  Returns the first unit of the block."""
    st = stage_fastq(sh, [(path1, None)] + ([(path2, None)] if path2 else []))
    if st is None:
        _n, first_unit = ctx.reads_load_fastq_part(path1, path2, sh.rank, sh.world)
        IO_STATS['fastq_mode'] = 'part-loader'
        return first_unit
    fr = st['frames']
    ctx.reads_load_staged(fr[0].fq, fr[1].fq if len(fr) > 1 else None, (-1, -1, -1, -1),
                          st['lines'])
    for f in fr:
        f.fq.close()
    return st['first']


# ---- output ----------------------------------------------------------------------
def _binary_fd(handle):
    """Descriptor of a seekable binary file handle (not appending), else None."""
    import io
    try:
        if isinstance(handle, io.TextIOBase) or not handle.seekable():
            return None
        if 'a' in getattr(handle, 'mode', ''):
            return None
        return handle.fileno()
    except (AttributeError, OSError, ValueError, io.UnsupportedOperation):
        return None


class SharedOutput:
    """One output file, written by every rank of a sharded job (sh) or by
    the one process (sh None).

    Every rank opened the same path (bin/micall opens its outputs on every
    rank).  place(lens) all-gathers each rank's segment sizes and returns
    this rank's file offsets, segment-major (segment 0 of rank 0, 1, ...,
    then segment 1 ...); the ranks then pwrite their own bytes there.  When
    the handles are not one plain file on every rank (a StringIO, a pipe),
    `direct` is False and the bytes go to rank 0, which writes them through
    its handle (Shard.gather_segments)."""

    def __init__(self, sh, handle, binary=False):
        self.sh, self.handle = sh, handle
        if not handle:
            fd = None
        elif binary:
            fd = _binary_fd(handle)
        else:
            fd = _native._plain_fd(handle)
        ident = (0, 0)
        pos = 0
        if fd is not None:
            handle.flush()
            st = os.fstat(fd)
            ident = (st.st_dev, st.st_ino)
            pos = os.lseek(fd, 0, os.SEEK_CUR)
        self.fd = fd
        self.written = []     # (offset, length, crc) of this rank's segments
        if sh is None:
            self.direct = fd is not None
            self.end = pos
            return
        rows = sh._gather_sizes([1 if fd is not None else 0, ident[0], ident[1]])
        self.direct = bool(rows[:, 0].all()) and len({(a, b) for _f, a, b in rows}) == 1
        self.end = int(sh.sum_i64([pos if sh.rank == 0 else 0])[0]) if self.direct else None

    @property
    def rank(self):
        return 0 if self.sh is None else self.sh.rank

    def place(self, lens):
        """File offsets of this rank's segments (lens: bytes per segment)."""
        lens = np.asarray(lens, dtype=np.int64)
        if len(lens) == 0:
            return np.zeros(0, dtype=np.int64)
        if self.sh is None:
            offs = self.end + np.concatenate([[0], np.cumsum(lens)[:-1]])
            self.end += int(lens.sum())
        else:
            all_lens = self.sh._gather_sizes(lens)            # [rank, segment]
            seg_total = all_lens.sum(axis=0)
            seg_base = self.end + np.concatenate([[0], np.cumsum(seg_total)[:-1]])
            offs = seg_base + all_lens[:self.sh.rank].sum(axis=0)
            self.end += int(seg_total.sum())
        IO_STATS['written_bytes'] += int(lens.sum())
        return offs

    def write_bytes(self, segments):
        """Write this rank's byte segments (same count on every rank)."""
        from . import session
        if not self.direct:
            if self.sh is None:
                for data in segments:
                    if len(data) and self.handle:
                        session.write_bytes(self.handle, data)
                return
            parts = self.sh.gather_segments(segments)
            if parts is not None and self.handle:
                for g in range(len(segments)):
                    for rr in range(self.sh.world):
                        if len(parts[rr][g]):
                            session.write_bytes(self.handle, parts[rr][g])
            return
        import zlib
        offs = self.place([len(x) for x in segments])
        for off, data in zip(offs, segments):
            mv = memoryview(data).cast('B')
            at = 0
            while at < len(mv):
                at += os.pwrite(self.fd, mv[at:], int(off) + at)
            self.written.append((int(off), len(mv), zlib.crc32(mv)))

    def write_rows(self, ctx, style, order, seg_rows):
        """Format rows order[...] (None: every read) in segments (seg_rows
        bounds) and write them: straight from the formatting threads when
        direct."""
        if not self.direct:
            if order is None:
                order = np.arange(ctx.reads_count()[0], dtype=np.int64)
            segs = [ctx.format_rows_bytes(style, order=np.asarray(order)[a:b]) if b > a else b''
                    for a, b in zip(seg_rows[:-1], seg_rows[1:])]
            self.write_bytes(segs)
            return
        if self.sh is None:
            # one process: the segments are contiguous; one formatting +
            # writing stream
            o = np.asarray(order)[seg_rows[0]:seg_rows[-1]] if order is not None else None
            n, crc = ctx.write_rows_at(self.fd, self.end, style, o)
            self.written.append((self.end, n, crc))
            self.end += n
            IO_STATS['written_bytes'] += n
            return
        lens = ctx.format_segments(style, order, seg_rows)
        offs = self.place(lens)
        crcs = ctx.write_segments(self.fd, offs)
        self.written += [(int(o), int(n), int(c)) for o, n, c in zip(offs, lens, crcs)]

    def finish(self):
        """After every rank's writes (sharded callers end with a barrier):
        rank 0's handle is positioned at the end of what was written."""
        if self.direct and self.rank == 0 and self.handle:
            self.handle.seek(self.end)

    def crc_of_file(self, head=b''):
        """(crc32, size) of the whole file as written, when it starts at
        offset 0 with `head` (rank 0's bytes written through its handle
        before) and this object wrote the rest; None otherwise."""
        import zlib
        mine = np.array(self.written, dtype=np.int64).reshape(-1, 3)
        if self.sh is None:
            segs = sorted(tuple(int(x) for x in row) for row in mine)
        else:
            sh = self.sh
            n = sh._gather_sizes([len(mine)])[:, 0]
            m = max(int(n.max()), 1)
            pad = np.zeros((m, 3), dtype=np.int64)
            pad[:len(mine)] = mine
            t = sh.torch.as_tensor(pad.reshape(-1), device=sh.device)
            allw = sh._gather(t).cpu().numpy().reshape(sh.world, m, 3)
            segs = sorted(tuple(int(x) for x in allw[k, j]) for k in range(sh.world)
                          for j in range(int(n[k])))
        crc, at = zlib.crc32(head), len(head)
        for off, ln, c in segs:
            if off != at:
                return None
            crc = _native.crc32_combine(crc, c, ln)
            at += ln
        return crc, at
