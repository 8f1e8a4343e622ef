"""bin/micall's whole per-sample chain as ONE sharded job (VERDICT r03, next
round item 1): 2 and 3 ranks on the test box's one GPU (gloo; the driver's
nodes use RCCL through the same calls) run tests/gpu_chain_worker.py, which
is bin/micall:91-192 call for call with the drop-ins in place of
micall.core.*:

    read_errors -> write_phix_csv -> report_bad_cycles -> censor (R1, then
    R2 with the exhausted reader) -> prelim_map -> remap -> sam2aln ->
    aln2counts

Every rank opens every file; censor, prelim_map and remap split their work
by rank (each rank reads its share of the FASTQ and writes its own rows at
its offsets), the InterOp reports, sam2aln and aln2counts run on rank 0
while the others wait.  Every intermediate and output file must be
byte-equal to what the stock reference wrote on the same inputs
(tests/golden/chain/, tests/golden/e2e/c1_example; the censored FASTQs are
compared decompressed).  c1_members is C1 written as many gzip members of
different sizes in R1 and R2, so the ingest splits the files by member and
realigns R2's records to R1's blocks.  c1_example's FASTQs are one gzip
member each, split by deflate block (each rank decodes its share of the
compressed bytes).  3 ranks split 600 / 800 / 9,600 units unevenly."""
import gzip
import json
import os
import shutil
import socket
import subprocess
import sys
import zlib

import pytest

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))
WORKER = os.path.join(HERE, 'gpu_chain_worker.py')
CHAIN = os.path.join(HERE, 'golden', 'chain')
E2E = os.path.join(HERE, 'golden', 'e2e')


def _port():
    with socket.socket() as s:
        s.bind(('127.0.0.1', 0))
        return s.getsockname()[1]


def _run_ranks(world, args, out):
    base = dict(os.environ, MASTER_ADDR='127.0.0.1', MASTER_PORT=str(_port()),
                WORLD_SIZE=str(world), MICALL_DIST_BACKEND='gloo', MICALL_HIP_DEVICE='0')
    procs = [subprocess.Popen([sys.executable, WORKER] + args + ['--outdir', str(out)],
                              env=dict(base, RANK=str(r), LOCAL_RANK=str(r)))
             for r in range(world)]
    codes = []
    for p in procs:
        try:
            codes.append(p.wait(timeout=300))
        except subprocess.TimeoutExpired:
            for q in procs:
                q.kill()
            raise
    assert codes == [0] * world, codes
    return [json.load(open(os.path.join(str(out), 'rank%d.json' % r))) for r in range(world)]


def _gz_text(path, mode='rt'):
    with gzip.open(path, mode) as f:
        return f.read()


def _members(data, size):
    out = []
    for at in range(0, len(data), size):
        c = zlib.compressobj(1, zlib.DEFLATED, 31)
        out.append(c.compress(data[at:at + size]) + c.flush())
    return b''.join(out)


def _inputs(case, work):
    """Copy the case's inputs into the work directory: (worker args, golden
    file for each output name)."""
    if case.startswith('c5_'):
        d = os.path.join(CHAIN, case)
        lengths = json.load(open(os.path.join(d, 'read_lengths.json')))
        args = []
        for mate in (1, 2):
            src = os.path.join(d, 'R%d.fastq.gz' % mate)
            if os.path.exists(src):
                shutil.copyfile(src, os.path.join(work, 'R%d.fastq.gz' % mate))
                args.append(os.path.join(work, 'R%d.fastq.gz' % mate))
        args += ['--interop', os.path.join(d, 'ErrorMetricsOut.bin'), '--readlen', str(lengths[0]),
                 '--index', str(lengths[1])]
        want = {'R1.quality.csv': 'quality.csv', 'R1.bad_cycles.csv': 'bad_cycles.csv',
                'R1.prelim.csv': 'prelim.csv', 'R1.remap.csv': 'remap.csv',
                'R1.align.csv': 'align.csv', 'R1.nuc.csv': 'nuc.csv', 'R1.amino.csv': 'amino.csv',
                'R1.insert.csv': 'insert.csv', 'R1.conseq.csv': 'conseq.csv'}
        return args, {k: os.path.join(d, v + '.gz') for k, v in want.items()}, d
    d = os.path.join(E2E, 'c1_example')
    args = []
    for mate, size in ((1, 150000), (2, 97000)):
        src = os.path.join(d, 'R%d.fastq.gz' % mate)
        dst = os.path.join(work, 'R%d.fastq.gz' % mate)
        if case == 'c1_members':
            with open(dst, 'wb') as f:
                f.write(_members(_gz_text(src, 'rb'), size))
        else:
            shutil.copyfile(src, dst)
        args.append(dst)
    want = {'R1.prelim.csv': 'prelim.csv', 'R1.remap.csv': 'remap.csv',
            'R1.align.csv': 'aligned.csv', 'R1.nuc.csv': 'a2c_nuc.csv',
            'R1.amino.csv': 'a2c_amino.csv', 'R1.insert.csv': 'a2c_coord_ins.csv',
            'R1.conseq.csv': 'a2c_conseq.csv'}
    return args, {k: os.path.join(d, v + '.gz') for k, v in want.items()}, d


@pytest.mark.timeout(900)
@pytest.mark.parametrize('world', [2, 3])
@pytest.mark.parametrize('case', ['c5_unpaired300', 'c5_paired251', 'c1_example', 'c1_members'])
def test_sharded_bin_micall_chain_matches_reference(tmp_path, case, world):
    work = tmp_path / 'work'
    work.mkdir()
    args, want, gold = _inputs(case, str(work))
    info = _run_ranks(world, args, work)
    assert [i['rank'] for i in info] == list(range(world))
    assert all(i['prelim_source'] == 'device' for i in info)
    for name, golden in sorted(want.items()):
        got = (work / name).read_text()
        assert got == _gz_text(golden), name
    if case.startswith('c5_'):
        for mate in (1, 2):
            got = work / ('R%d.censor.fastq.gz' % mate)
            if not got.exists():
                continue
            assert _gz_text(str(got), 'rb') == _gz_text(os.path.join(gold, 'R%d.censor.fastq.gz' % mate),
                                                        'rb'), mate
    # every rank read a share of the FASTQ and wrote a share of the rows
    prelim = [i['prelim_map'] for i in info]
    written = [p['written_bytes'] for p in prelim]
    assert all(w > 0 for w in written)
    assert max(written) <= 0.75 * sum(written) if world == 2 else max(written) <= 0.6 * sum(written)
    if case in ('c5_unpaired300', 'c5_paired251', 'c1_members'):
        # the censored files (one gzip member per rank) and c1_members are split by member
        assert all(p['fastq_mode'] == 'members' for p in prelim), prelim
        decoded = [p['fastq_file_bytes'] for p in prelim]
        assert max(decoded) <= 0.75 * sum(decoded), decoded
    if case == 'c1_example':
        # C1's FASTQs are one gzip member each (bcl2fastq's layout): every
        # rank decodes the deflate blocks in its share of the compressed
        # bytes (sharded_io._open_members), none the whole file
        assert all(p['fastq_mode'] == 'member-part' for p in prelim), prelim
        decoded = [p['fastq_file_bytes'] for p in prelim]
        assert max(decoded) <= (0.75 if world == 2 else 0.6) * sum(decoded), decoded
    if case.startswith('c5_'):
        censor = [i['censor']['written_bytes'] for i in info]
        assert all(w > 0 for w in censor) and max(censor) <= 0.75 * sum(censor)
