"""aln2counts' counting split over the ranks of a job (VERDICT r04, next-round
item 4): 2 and 3 ranks on the test box's one GPU (gloo; RCCL on the driver's
nodes through the same calls) each count the rows in their share of
aligned.csv on the device, the counters (sums) and their first rows (minima,
over the job's row numbers within a group) are all-reduced, every rank
builds the reports from the job's counters and rank 0 writes them; the
insertion strings are added up the same way (micall_amd.aln2counts
_load_sharded, InsertionWriter.write; csrc/mh_a2c.hip mh_a2c_part_*,
mh_a2c_insert_export / _merge).  Every output must be byte-equal to the
reference's aln2counts() on the same aligned.csv: every e2e case
(tests/golden/e2e/*/a2c_*.csv) and every edge-case text of
tests/golden/aln2counts_edge.json; and a synthetic aligned.csv of several
groups (two qcuts, runs crossing the ranks' cuts) equal to the unsharded
run.  Reference: aln2counts.py:115-172 (the counting), :786-795 (insertions)."""
import gzip
import json
import os
import random
import socket
import subprocess
import sys

import pytest

from micall_amd import projects

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))
GOLDEN = os.path.join(HERE, 'golden')
WORKER = os.path.join(HERE, 'gpu_a2c_worker.py')
OUTS = ('nuc', 'amino', 'coord_ins', 'conseq', 'failed', 'coverage')


def _port():
    with socket.socket() as s:
        s.bind(('127.0.0.1', 0))
        return s.getsockname()[1]


def _gz(path):
    with gzip.open(path, 'rt') as f:
        return f.read()


def _synthetic(n_rows=6000, seed=5):
    rng = random.Random(seed)
    pol = projects.load_default().seed_sequences()['HIV1B-pol-seed']
    sample = pol[:1500] + 'GGA' + pol[1500:]
    rows = []
    for qcut in ('15', '20'):
        seen = set()
        for rank in range(n_rows // 2):
            off = rng.randrange(0, len(sample) - 120)
            s = list(sample[off:off + rng.randint(60, 420)])
            for i in range(len(s)):
                r = rng.random()
                if r < 0.02:
                    s[i] = rng.choice('ACGT')
                elif r < 0.03:
                    s[i] = 'N'
            if rng.random() < 0.2:
                i = rng.randrange(10, len(s) - 20)
                s[i:i + 5] = ['n'] * 5
            s = ''.join(s).strip('-')
            if (off, s) in seen:
                continue
            seen.add((off, s))
            rows.append('HIV1B-pol-seed,{},{},{},{},{}\n'.format(qcut, len(rows), rng.choice([1, 2, 3, 7]),
                                                                   off, s))
    return 'refname,qcut,rank,count,offset,seq\n' + ''.join(rows)


def _cases(root):
    want = {}

    def put(name, text, outs, proj=None):
        os.makedirs(os.path.join(root, name))
        with open(os.path.join(root, name, 'aligned.csv'), 'w') as f:
            f.write(text)
        if proj is not None:
            with open(os.path.join(root, name, 'projects.json'), 'w') as f:
                json.dump(proj, f)
        want[name] = outs
    for case in sorted(os.listdir(os.path.join(GOLDEN, 'e2e'))):
        d = os.path.join(GOLDEN, 'e2e', case)
        put('e2e_' + case, _gz(os.path.join(d, 'aligned.csv.gz')),
            {k: _gz(os.path.join(d, 'a2c_%s.csv.gz' % k)) for k in OUTS})
    edge = json.load(open(os.path.join(GOLDEN, 'aln2counts_edge.json')))
    for k, case in enumerate(edge['cases']):
        put('edge%02d' % k, case['text'], case['outputs'], edge['config'])
    put('single_synthetic', _synthetic(), None)
    return want


@pytest.mark.timeout(900)
@pytest.mark.parametrize('world', [2, 3])
def test_sharded_aln2counts_matches_reference(tmp_path, world):
    root = str(tmp_path / 'cases')
    os.makedirs(root)
    want = _cases(root)
    env = dict(os.environ, MASTER_ADDR='127.0.0.1', MASTER_PORT=str(_port()), WORLD_SIZE=str(world),
               MICALL_DIST_BACKEND='gloo', MICALL_HIP_DEVICE='0')
    procs = [subprocess.Popen([sys.executable, WORKER, '--cases', root],
                              env=dict(env, RANK=str(r), LOCAL_RANK=str(r))) for r in range(world)]
    try:
        codes = [p.wait(timeout=800) for p in procs]
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
    assert codes == [0] * world, codes
    stats = [json.load(open(os.path.join(root, 'rank%d.json' % r))) for r in range(world)]
    for name, outs in want.items():
        for k in OUTS:
            got = open(os.path.join(root, name, k + '.csv')).read()
            exp = outs[k] if outs is not None else open(os.path.join(root, name, k + '.single')).read()
            assert got == exp, (name, k)
    # the e2e cases and the synthetic one count split: every rank counted a
    # share of the rows, none all of them
    for name in want:
        if not (name.startswith('e2e_') or name.startswith('single_')):
            continue
        modes = [s[name].get('mode') for s in stats]
        assert modes == ['sharded'] * world, (name, modes)
        rows = [s[name]['rows'] for s in stats]
        if sum(rows) >= 3 * world:
            assert max(rows) < sum(rows), (name, rows)
