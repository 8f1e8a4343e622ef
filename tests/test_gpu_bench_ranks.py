"""bench.py's multi-rank path (what the driver runs at N = 2..8 over RCCL),
rehearsed with two ranks on the one GPU of the test box over gloo
(MICALL_BENCH_BACKEND=gloo): per-rank read blocks, the all-reduced tallies
and pileup, max-over-ranks timing and the single JSON line of rank 0."""
import json
import os
import socket
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    with socket.socket() as s:
        s.bind(('127.0.0.1', 0))
        return s.getsockname()[1]


@pytest.mark.gpu
def test_bench_two_ranks_gloo():
    pairs = 20000
    env = dict(os.environ, MICALL_BENCH_BACKEND='gloo')
    cmd = [sys.executable, '-m', 'torch.distributed.run', '--nnodes=1', '--nproc-per-node', '2',
           '--master-addr', '127.0.0.1', '--master-port', str(_free_port()),
           os.path.join(REPO, 'bench.py'), '--gpus', '2', '--pairs', str(pairs),
           '--steps', '1', '--warmup', '1', '--no-cpu-baseline']
    out = subprocess.run(cmd, env=env, cwd=REPO, capture_output=True, text=True, timeout=100)
    assert out.returncode == 0, out.stderr[-2000:]
    lines = [ln for ln in out.stdout.splitlines() if ln.startswith('{"metric"')]
    assert len(lines) == 1, out.stdout[-2000:]
    d = json.loads(lines[0])
    assert d['n_gpus'] == 2 and d['scaling'] == 'weak'
    assert d['value'] > 0 and d['ms_per_step'] > 0
    # every read of both ranks' blocks maps to the pol consensus; the tallies
    # are the all-reduced sums over the two ranks
    assert sum(d['result']['mapped_lines'].values()) == 2 * 2 * pairs
    assert list(d['result']['conseqs']) == ['HIV1B-pol-seed']
