"""Sharded FASTQ ingest on the CPU (gloo, world sizes 2 and 3): every rank
reads only its share of each file (the gzip members starting in its byte
range, or the byte range of a plain file), frames its text into four-line
records from the line counts of the ranks before it, hands the bytes before
its first record to the rank before, and realigns R2 to R1's blocks by
point-to-point exchange (micall_amd.sharded_io.stage_fastq).

The block each rank ends up with must be exactly the records
[first, first + units) of both files, the blocks must tile the file in rank
order, raw_count's line count must be the whole file's, and with many
members a rank must decode only about 1/W of the file.  Files that cannot
be split (one gzip member; a blank line where a record starts) fall back to
the whole-file loader (non-strict) or to a whole read plus a floor split of
the records (strict, the censor's framing).  Reference behaviour: the FASTQ
records bowtie2 reads (prelim_map.py:114-134) and censor's four-line records
(censor_fastq.py:58)."""
import gzip
import os
import socket
import zlib

import numpy as np
import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

from micall_amd import _native, sharded_io
from micall_amd.pipeline import Shard


def _records(n, mate, seed, crlf=False, fake_header_at=None):
    rng = np.random.default_rng(seed)
    out = []
    for i in range(n):
        L = int(rng.integers(30, 120))
        seq = ''.join(rng.choice(list('ACGTN'), size=L))
        qual = ''.join(rng.choice(list('#,:AFG'), size=L))
        name = '@M00:1:FC:1:%d:%d:%d %d:N:0:1' % (1101 + i % 3, i, 7 * i, mate)
        rec = '%s\n%s\n+\n%s\n' % (name, seq, qual)
        if crlf:
            rec = rec.replace('\n', '\r\n')
        rec = rec.encode()
        if fake_header_at is not None and i == fake_header_at:
            # a gzip-member-shaped byte run inside the text (it reaches the
            # compressed stream verbatim in a stored member)
            rec = rec.replace(b' %d:N' % mate, b'\x1f\x8b\x08\x00\x00\x00\x00\x00\x00\x03ZZ %d:N' % mate)
        out.append(rec)
    return out


def _records_fast(n, mate, seed):
    """n FASTQ records of 151 nt (vectorised: the > 8 MB single-member cases)."""
    rng = np.random.default_rng(seed)
    bases = np.frombuffer(b'ACGTN', dtype=np.uint8)[rng.choice(5, size=(n, 151), p=[.3, .2, .2, .29, .01])]
    quals = np.frombuffer(b'#,:AFG', dtype=np.uint8)[rng.choice(6, size=(n, 151),
                                                                 p=[.02, .02, .06, .1, .2, .6])]
    return [b'@M00:1:FC:1:%d:%d:%d %d:N:0:1\n%s\n+\n%s\n' % (1101 + i % 3, i, 7 * i, mate,
                                                              bases[i].tobytes(), quals[i].tobytes())
            for i in range(n)]


MODES = {None: 0, 'members': 1, 'member-part': 2, 'whole': 3}
BIG = 80000


def _gz_members(data, member_bytes, level=1, stored_member=None):
    out, k = [], 0
    for at in range(0, len(data), member_bytes):
        lvl = 0 if (stored_member is not None and k == stored_member) else level
        c = zlib.compressobj(lvl, zlib.DEFLATED, 31)
        out.append(c.compress(data[at:at + member_bytes]) + c.flush())
        k += 1
    return b''.join(out)


def _make_case(d, case):
    """Write the case's files; returns (paths, [records per file])."""
    n = 700
    if case.startswith('big'):
        n = BIG
        recs = [_records_fast(n, 1, 1), _records_fast(n, 2, 2)]
        if case == 'big_unpaired':
            recs = recs[:1]
        paths = []
        for k, rs in enumerate(recs):
            p = os.path.join(d, 'R%d.fastq.gz' % (k + 1))
            with open(p, 'wb') as f:
                # one member, as bcl2fastq writes it; big6: zlib level 6
                # (bigger blocks), else level 1; big_stored: stored blocks only
                # (no block start to find: read whole)
                lvl = 6 if case == 'big6' else 0 if case == 'big_stored' else 1
                f.write(gzip.compress(b''.join(rs), lvl))
            paths.append(p)
        return paths, recs
    recs = [_records(n, 1, 1, crlf=case == 'crlf'), _records(n, 2, 2, crlf=case == 'crlf')]
    if case == 'unpaired':
        recs = recs[:1]
    if case == 'blank':
        recs[0][n // 2] = b'\n' + recs[0][n // 2]
    if case == 'fake_header':
        recs[0] = _records(n, 1, 1, fake_header_at=n // 2)
    paths = []
    for k, rs in enumerate(recs):
        data = b''.join(rs)
        p = os.path.join(d, 'R%d.fastq%s' % (k + 1, '' if case == 'plain' else '.gz'))
        if case == 'plain':
            blob = data
        elif case == 'single' or (case == 'mixed' and k == 1):
            blob = gzip.compress(data, 6)
        elif case == 'fake_header':
            mb = 9000 + 1000 * k
            at = data.find(b'\x1f\x8b')
            blob = _gz_members(data, mb, stored_member=at // mb if at >= 0 else None)
            assert k == 1 or b'\x1f\x8b\x08\x00' in blob
        else:
            blob = _gz_members(data, 7000 + 3100 * k)        # R1 / R2 members do not line up
        with open(p, 'wb') as f:
            f.write(blob)
        paths.append(p)
    return paths, recs


def _worker(rank, world, port, d, case, strict):
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port))
    if case.startswith('big'):
        # spans of 1 MiB: several per rank, so that spans after a rank's
        # first copy window bytes that are still symbolic
        os.environ['MH_PINFLATE_SPAN_MIN'] = str(1 << 20)
    dist.init_process_group('gloo', rank=rank, world_size=world)
    if case == 'big_tail_fail' and rank == 0:
        # any exception while resolving rank 0's tail (not only the
        # library's NativeError): rank 1 must still get its window
        def boom(self, window):
            raise MemoryError('injected')
        _native.Fastq.member_tail = boom
    try:
        paths, recs = _make_case(d, case) if rank == 0 else (None, None)
        dist.barrier()
        if rank != 0:
            paths, recs = _make_case(d + '_r%d' % rank, case)   # same content, own copy of the expectation
            paths = [os.path.join(d, os.path.basename(p)) for p in paths]
        sh = Shard(rank, world, 0)
        sharded_io.reset_stats()
        st = sharded_io.stage_fastq(sh, [(p, None) for p in paths], strict=strict)
        result = dict(rank=rank)
        if st is None:
            result['fallback'] = True
            result['file_bytes'] = sharded_io.IO_STATS['fastq_file_bytes']
        else:
            first, units = st['first'], st['units']
            for k, f in enumerate(st['frames']):
                got = f.fq.view().tobytes()
                want = b''.join(recs[k][first:first + units])
                assert got == want, (rank, k, first, units, len(got), len(want))
                f.fq.close()
            total_nl = sum(r.count(b'\n') for r in recs[0])
            assert st['lines'] == total_nl
            assert st['total'] == len(recs[0])
            result.update(first=first, units=units, mode=st['mode'],
                          file_bytes=sharded_io.IO_STATS['fastq_file_bytes'],
                          file_size=sum(os.path.getsize(p) for p in paths))
        np.save(os.path.join(d, 'rank%d.npy' % rank), np.array([
            result.get('fallback', False), result.get('first', -1), result.get('units', -1),
            MODES[result.get('mode')], result.get('file_bytes', 0),
            result.get('file_size', 0)], dtype=np.int64))
    finally:
        dist.destroy_process_group()


def _free_port():
    with socket.socket() as s:
        s.bind(('127.0.0.1', 0))
        return s.getsockname()[1]


def _run(tmp_path, world, case, strict=False):
    d = str(tmp_path / 'files')
    os.makedirs(d, exist_ok=True)
    for r in range(1, world):
        os.makedirs(d + '_r%d' % r, exist_ok=True)
    mp.spawn(_worker, args=(world, _free_port(), d, case, strict), nprocs=world, join=True)
    return [np.load(os.path.join(d, 'rank%d.npy' % r)) for r in range(world)]


@pytest.mark.timeout(300)
@pytest.mark.parametrize('world', [2, 3])
@pytest.mark.parametrize('case', ['members', 'plain', 'unpaired', 'crlf', 'fake_header'])
def test_split_blocks_tile_the_file(tmp_path, world, case):
    res = _run(tmp_path, world, case)
    assert not any(r[0] for r in res)
    firsts, units = [int(r[1]) for r in res], [int(r[2]) for r in res]
    assert firsts[0] == 0 and all(firsts[k] + units[k] == firsts[k + 1] for k in range(world - 1))
    assert firsts[-1] + units[-1] == 700
    assert all(r[3] == MODES['members'] for r in res)    # split, not read whole
    # each rank decoded about its share of the files (members are whole units)
    size = int(res[0][5])
    for r in res:
        assert r[4] <= size / world * 1.6 + 20000, (r[4], size)


@pytest.mark.timeout(300)
@pytest.mark.parametrize('world', [2, 3])
def test_mixed_split_and_whole_files(tmp_path, world):
    """R1 in many members, R2 one member: R2 is read whole and cut to R1's
    blocks."""
    res = _run(tmp_path, world, 'mixed')
    assert not any(r[0] for r in res)
    assert sum(int(r[2]) for r in res) == 700


@pytest.mark.timeout(300)
@pytest.mark.parametrize('world,case,strict', [(2, 'big', False), (3, 'big', False), (2, 'big6', False),
                                               (3, 'big_unpaired', False), (3, 'big', True)])
def test_single_member_split_by_rank(tmp_path, world, case, strict):
    """Each FASTQ one gzip member of > 8 MB (bcl2fastq's layout): every rank
    decodes only the deflate blocks that start in its share of the
    compressed bytes, the windows it lacks arrive by the rank-order chain,
    and the combined CRC-32 matches the trailer (sharded_io._open_members).
    The blocks tile the file in rank order with the serial decode's bytes
    (checked per record in _worker), and no rank reads more than 3/4 (W=2)
    or 3/5 (W=3) of the compressed bytes."""
    res = _run(tmp_path, world, case, strict=strict)
    assert not any(r[0] for r in res)
    assert all(r[3] == MODES['member-part'] for r in res)
    firsts, units = [int(r[1]) for r in res], [int(r[2]) for r in res]
    assert firsts[0] == 0 and all(firsts[k] + units[k] == firsts[k + 1] for k in range(world - 1))
    assert firsts[-1] + units[-1] == BIG
    size = int(res[0][5])
    assert size > (8 << 20) * (1 if case == 'big_unpaired' else 2)
    for r in res:
        assert 0 < r[4] <= size * (3 / 4 if world == 2 else 3 / 5), (r[4], size)


@pytest.mark.timeout(300)
def test_single_member_without_block_starts_is_read_whole(tmp_path):
    """A member of stored blocks only has no block start to split at: the
    ranks agree to read it whole (strict framing: records split by count),
    having decoded nothing before."""
    res = _run(tmp_path, 2, 'big_stored', strict=True)
    assert not any(r[0] for r in res)
    assert all(r[3] == MODES['whole'] for r in res)
    assert [int(r[2]) for r in res] == [BIG // 2, BIG - BIG // 2]


@pytest.mark.timeout(300)
@pytest.mark.parametrize('case', ['single', 'blank'])
def test_unsplittable_files_fall_back(tmp_path, case):
    res = _run(tmp_path, 2, case)
    assert all(r[0] for r in res)                    # the whole-file part loader


@pytest.mark.timeout(300)
@pytest.mark.parametrize('case', ['single', 'members'])
def test_strict_framing_for_censor(tmp_path, case):
    """The censor's framing: one member is read whole by every rank and its
    records split by count; many members are split."""
    res = _run(tmp_path, 3, case, strict=True)
    assert not any(r[0] for r in res)
    units = [int(r[2]) for r in res]
    assert sum(units) == 700
    if case == 'single':
        assert units == [700 * (k + 1) // 3 - 700 * k // 3 for k in range(3)]


def test_parallel_gunzip_matches_serial(tmp_path):
    """mh_gunzip's member-parallel path (inputs over 4 MiB): a multi-member
    file whose stored member holds gzip-header-shaped bytes (a false member
    candidate: the span is merged with its neighbour), and one whose false
    candidate sits in the last member (the parallel path gives up and the
    file is decoded serially).  Both equal Python's gzip."""
    rng = np.random.default_rng(5)
    body = rng.choice(np.frombuffer(b'ACGT\n', dtype=np.uint8), size=6 << 20).tobytes()
    fake = b'\x1f\x8b\x08\x00\x00\x00\x00\x00\x00\x03' + b'\x00' * 12 + b'\xff\xff\xff\x7f'
    for where in ('middle', 'last'):
        parts = [body[k:k + (1 << 20)] for k in range(0, len(body), 1 << 20)]
        k = 2 if where == 'middle' else len(parts) - 1
        parts[k] = parts[k][:1000] + fake + parts[k][1000:]
        blob = b''.join(_gz_members(p, len(p) + 1, level=0 if j == k else 1)
                        for j, p in enumerate(parts))
        assert fake in blob
        path = tmp_path / ('f_%s.gz' % where)
        path.write_bytes(blob)
        fq = _native.Fastq(str(path))
        assert fq.view().tobytes() == gzip.decompress(blob)
        fq.close()


def _py_reads(text, paired):
    """The loader's reading of FASTQ text (mh_api.cpp index_fastq and
    qname_span): blank lines skipped where a record starts, '\\r' before
    '\\n' dropped, QNAME = header up to the first blank (bowtie2), '/1' '/2'
    dropped for mates, QUAL padded with 'I' / cut to the SEQ length."""
    lines = text.split(b'\n')
    if lines and lines[-1] == b'':
        lines = lines[:-1]
    lines = [ln[:-1] if ln.endswith(b'\r') else ln for ln in lines]
    out, k = [], 0
    while k < len(lines):
        if lines[k] == b'':
            k += 1
            continue
        h, seq, qual = lines[k], lines[k + 1], lines[k + 3]
        a = 1 if h[:1] == b'@' else 0
        while a < len(h) and h[a:a + 1] in (b' ', b'\t'):
            a += 1
        b = a
        while b < len(h) and h[b:b + 1] not in (b' ', b'\t', b'\r'):
            b += 1
        name = h[a:b]
        if paired and len(name) > 2 and name[-2:-1] == b'/' and name[-1:] in (b'1', b'2'):
            name = name[:-2]
        q = (qual + b'I' * len(seq))[:len(seq)]
        out.append((name.decode(), seq, q))
        k += 4
    return out


@pytest.mark.parametrize('variant', ['plain', 'crlf', 'slash', 'blank_and_short_qual'])
def test_host_parse_matches_the_loader_rules(tmp_path, variant):
    """mh_fastq_parse: the host half of the loader (records, bowtie2 QNAMEs,
    SEQ / QUAL, mates interleaved) against a Python restatement, on R1 / R2
    texts with CRLF line ends, '/1' '/2' name suffixes, blank lines between
    records and qualities shorter than the read."""
    r1 = _records(300, 1, 11, crlf=variant == 'crlf')
    r2 = _records(300, 2, 12, crlf=variant == 'crlf')
    if variant == 'slash':
        r1 = [r.replace(b' 1:N', b'/1 1:N') for r in r1]
        r2 = [r.replace(b' 2:N', b'/2 2:N') for r in r2]
    if variant == 'blank_and_short_qual':
        r1[10] = b'\n' + r1[10]
        parts = r2[20].split(b'\n')
        parts[3] = parts[3][:-5]
        r2[20] = b'\n'.join(parts)
    paths = []
    for k, rs in enumerate((r1, r2)):
        p = tmp_path / ('R%d.fastq.gz' % (k + 1))
        p.write_bytes(_gz_members(b''.join(rs), 5000))
        paths.append(str(p))
    a, b = _native.Fastq(paths[0]), _native.Fastq(paths[1])
    names, seqs, quals = a.parse(b)
    want1, want2 = _py_reads(b''.join(r1), True), _py_reads(b''.join(r2), True)
    want = [x for pair in zip(want1, want2) for x in pair]
    assert names == [w[0] for w in want]
    assert seqs == [w[1] for w in want]
    assert quals == [w[2] for w in want]
    un_names, un_seqs, _ = a.parse()
    assert un_names[:3] == [w[0] for w in _py_reads(b''.join(r1), False)][:3]
    assert len(un_seqs) == 300
    a.close()
    b.close()


def _pinflate_run(path, env_extra):
    """Stage a FASTQ in a child process with MH_PINFLATE_TRACE: (text sha, stderr)."""
    import subprocess
    import sys
    code = ('import hashlib, sys; sys.path[:0] = [%r]\n'
            'from micall_amd import _native\n'
            'fq = _native.Fastq(path=%r)\n'
            'print(hashlib.sha256(fq.view().tobytes()).hexdigest())\n'
            % (os.path.dirname(os.path.dirname(os.path.abspath(_native.__file__))), path))
    env = dict(os.environ, MH_PINFLATE_TRACE='1', OMP_NUM_THREADS='4', **env_extra)
    out = subprocess.run([sys.executable, '-c', code], capture_output=True, text=True, env=env, timeout=300)
    assert out.returncode == 0, out.stderr
    return out.stdout.strip(), out.stderr


@pytest.mark.parametrize('level,nul', [(1, False), (6, False), (9, True)])
def test_single_member_parallel_inflate(tmp_path, level, nul):
    """One gzip member (as bcl2fastq writes it) of > 8 MB is inflated by
    several threads (mh_pinflate.cpp: block starts found by header search,
    spans decoded with a zero window, window-derived bytes resolved from
    base-255 offset windows, CRC-32 checked) and gives the bytes of a plain
    inflate; a file holding NUL bytes (which the zero window cannot tell from
    window bytes) too."""
    import hashlib
    import numpy as np
    rng = np.random.default_rng(level)
    n = 90000 if level == 1 else 60000
    bases = np.frombuffer(b'ACGT', dtype=np.uint8)[rng.integers(0, 4, (n, 151))]
    quals = (rng.integers(0, 40, (n, 151)) + 33).astype(np.uint8)
    if nul:
        quals[::997, 7] = 0
    lines = []
    for i in range(n):
        lines.append(b'@M01:1:FC:1:%d:%d:%d 1:N:0:1\n' % (1101 + i % 4, i, i))
        lines.append(bases[i].tobytes() + b'\n+\n' + quals[i].tobytes() + b'\n')
    text = b''.join(lines)
    path = str(tmp_path / 'R1.fastq.gz')
    with gzip.GzipFile(path, 'wb', compresslevel=level) as f:    # FNAME in the header
        f.write(text)
    assert os.path.getsize(path) > (8 << 20)
    want = hashlib.sha256(text).hexdigest()
    got, err = _pinflate_run(path, {})
    assert got == want
    assert 'pinflate crc' in err, err[-2000:]
    got, err = _pinflate_run(path, {'MICALL_SERIAL_INFLATE': '1'})
    assert got == want and 'pinflate' not in err


def test_single_member_parallel_inflate_high_ratio(tmp_path):
    """A member that compresses ~7:1 (reads drawn from a small pool): each
    span's decode outgrows the output size first guessed for it and is run
    again with a larger buffer; the bytes still equal a plain inflate's, and
    the zlib span decode (MICALL_ZLIB_SPANS=1) gives the same."""
    import hashlib
    import numpy as np
    rng = np.random.default_rng(3)
    pool_b = np.frombuffer(b'ACGT', dtype=np.uint8)[rng.integers(0, 4, (64, 151))]
    pool_q = (rng.integers(30, 41, (64, 151)) + 33).astype(np.uint8)
    n = 190000
    pick_b, pick_q = rng.integers(0, 64, n), rng.integers(0, 64, n)
    lines = []
    for i in range(n):
        lines.append(b'@M01:1:FC:1:%d:%d:%d 1:N:0:1\n' % (1101 + i % 4, i % 50, i % 70))
        lines.append(pool_b[pick_b[i]].tobytes() + b'\n+\n' + pool_q[pick_q[i]].tobytes() + b'\n')
    text = b''.join(lines)
    path = str(tmp_path / 'R1.fastq.gz')
    with gzip.GzipFile(path, 'wb', compresslevel=6) as f:
        f.write(text)
    assert os.path.getsize(path) > (8 << 20)
    assert len(text) > 6 * os.path.getsize(path)
    want = hashlib.sha256(text).hexdigest()
    for extra in ({}, {'MICALL_ZLIB_SPANS': '1'}):
        got, err = _pinflate_run(path, extra)
        assert got == want
        assert 'pinflate crc' in err, err[-2000:]


@pytest.mark.parametrize('tail,ok', [(b'', True), (b'\n', True), (b'\n\n', True), (b'\r\n', True),
                                     (b'@extra\n', False), (b'@extra', False)])
def test_host_parse_record_framing_tail(tmp_path, tail, ok):
    """index_fastq's framing at the end of the text: trailing empty lines
    (or '\\r' alone) are skipped, a partial record is an error, whichever of
    its two paths (every fourth line when no line is empty, else the
    line-by-line walk) runs."""
    text = b''.join(_records(40, 1, 5)) + tail
    p = tmp_path / 'R1.fastq'
    p.write_bytes(text)
    if ok:
        fq = _native.Fastq(str(p))
        names, seqs, _ = fq.parse()
        assert len(seqs) == 40 and names[0] == _py_reads(text, False)[0][0]
        fq.close()
    else:
        with pytest.raises(Exception, match='truncated'):
            fq = _native.Fastq(str(p))
            fq.parse()


def test_member_scan_near_range_ends(tmp_path):
    """mh_fastq_scan_part: a member that starts just before the end of a
    part's byte range is found (its header probe reads past the range), so a
    file of one member per rank -- the censor's output -- is split by
    member, not taken for a single member."""
    rng = np.random.default_rng(9)
    data = rng.integers(0, 256, 300000, dtype=np.uint8).tobytes()
    blob = b''.join(_gz_members(data[a:b], b - a + 1) for a, b in ((0, 99000), (99000, 199000),
                                                                   (199000, 300000)))
    path = tmp_path / 'three.gz'
    path.write_bytes(blob)
    found = [_native.Fastq.scan_part(str(path), -1, r, 3)[2] for r in range(3)]
    assert found[:2] == [True, True] and found[2] is False
    single = tmp_path / 'one.gz'
    single.write_bytes(gzip.compress(data, 1))
    assert not any(_native.Fastq.scan_part(str(single), -1, r, 3)[2] for r in range(3))


@pytest.mark.timeout(300)
def test_member_tail_failure_does_not_stall_the_chain(tmp_path):
    """an exception other than NativeError in rank 0's
    member_tail used to skip the send, leaving rank 1 in recv forever.  Now
    the window goes on as zeros marked unresolved, the CRC agreement fails on
    every rank and every rank falls back to reading the files whole."""
    res = _run(tmp_path, 2, 'big_tail_fail')
    assert all(r[0] for r in res) or all(r[3] == MODES['whole'] for r in res), res
