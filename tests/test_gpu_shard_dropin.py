"""The drop-ins in a sharded run write the single-GPU files (VERDICT r02,
next-round item 3): two ranks on the test box's one GPU (gloo; the
driver's multi-GPU nodes use RCCL through the same calls) each keep their
block of the FASTQ pairs resident, and prelim.csv, remap.csv,
remap_counts.csv, remap_conseq.csv and the unmapped FASTQs must be byte-equal
to the reference-generated goldens -- with remap() taking the prelim rows from
the resident records, and again parsing prelim.csv in a fresh context.
Reference: prelim_map.py:142-151 (grouped rows), remap.py:612-658 (remap.csv
of the last pass, then the split pairs re-mapped)."""
import gzip
import json
import os
import socket
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))
WORKER = os.path.join(HERE, 'gpu_dropin_worker.py')
FILES = ('prelim.csv', 'remap.csv', 'remap_counts.csv', 'remap_conseq.csv', 'unmapped1.fastq',
         'unmapped2.fastq')


def _port():
    with socket.socket() as s:
        s.bind(('127.0.0.1', 0))
        return s.getsockname()[1]


def _run_ranks(world, args, out):
    base = dict(os.environ, MASTER_ADDR='127.0.0.1', MASTER_PORT=str(_port()),
                WORLD_SIZE=str(world), MICALL_DIST_BACKEND='gloo', MICALL_HIP_DEVICE='0')
    procs = [subprocess.Popen([sys.executable, WORKER] + args + ['--out', str(out)],
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
    return [json.load(open(out / ('rank%d.json' % r))) for r in range(world)]


@pytest.mark.timeout(900)
@pytest.mark.parametrize('case', ['syn_pol', 'syn_chimera', 'c1_example', 'syn_unpaired300'])
@pytest.mark.parametrize('fresh', [False, True])
def test_two_rank_dropins_write_the_golden_files(golden_dir, tmp_path, case, fresh):
    d = os.path.join(golden_dir, 'e2e', case)
    r1 = os.path.join(d, 'R1.fastq.gz')
    r2 = os.path.join(d, 'R2.fastq.gz')
    args = [r1] + ([r2] if os.path.exists(r2) else []) + (['--fresh-remap'] if fresh else [])
    info = _run_ranks(2, args, tmp_path)
    assert [i['prelim_source'] for i in info] == ['csv' if fresh else 'device'] * 2
    assert info[1]['read_base'] > 0 and all(i['reads'] > 0 for i in info)
    for name in FILES:
        with gzip.open(os.path.join(d, name + '.gz'), 'rt') as f:
            want = f.read()
        got = open(tmp_path / name).read()
        assert got == want, name
