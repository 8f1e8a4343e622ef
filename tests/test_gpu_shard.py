"""Sharded remap on the GPU: two ranks (child processes on cuda:0, gloo on
CUDA tensors, the same device export/all-reduce/import as RCCL) must produce
exactly the unsharded run's seed tallies, consensus sequences, mapped counts
and loop decisions."""
import json
import os
import socket
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))
WORKER = os.path.join(HERE, 'gpu_shard_worker.py')


def _port():
    with socket.socket() as s:
        s.bind(('127.0.0.1', 0))
        return s.getsockname()[1]


def _run(cmds, env):
    procs = [subprocess.Popen(c, env=env) for c in cmds]
    codes = []
    for p in procs:
        try:
            codes.append(p.wait(timeout=400))
        except subprocess.TimeoutExpired:
            for q in procs:
                q.kill()
            raise
    assert codes == [0] * len(cmds), codes


@pytest.mark.timeout(900)
def test_two_rank_remap_matches_single_rank(tmp_path):
    env = dict(os.environ, MASTER_ADDR='127.0.0.1', MASTER_PORT=str(_port()))
    single = tmp_path / 'single.json'
    _run([[sys.executable, WORKER, '--world', '1', '--out', str(single)]], env)
    outs = [tmp_path / ('rank%d.json' % r) for r in range(2)]
    _run([[sys.executable, WORKER, '--world', '2', '--rank', str(r), '--out', str(outs[r])]
          for r in range(2)], env)
    ref = json.load(open(single))
    assert ref['conseqs'], 'the unsharded run built no consensus'
    for out in outs:
        got = json.load(open(out))
        for key in ('groups', 'prelim', 'conseqs', 'counts', 'unmapped', 'n_remaps', 'log'):
            assert got[key] == ref[key], key


@pytest.mark.timeout(600)
def test_rccl_shard_path_matches_unsharded(tmp_path):
    """The Shard exchange over the nccl backend (RCCL), one rank: the
    collectives the driver's multi-GPU runs use, on device buffers, must leave
    every result of the unsharded run unchanged."""
    env = dict(os.environ, MASTER_ADDR='127.0.0.1', MASTER_PORT=str(_port()))
    single = tmp_path / 'single.json'
    rccl = tmp_path / 'rccl.json'
    _run([[sys.executable, WORKER, '--world', '1', '--pairs', '8000', '--out', str(single)]], env)
    _run([[sys.executable, WORKER, '--world', '1', '--pairs', '8000', '--backend', 'nccl', '--shard',
           '--out', str(rccl)]], env)
    ref = json.load(open(single))
    got = json.load(open(rccl))
    assert ref['conseqs']
    for key in ('groups', 'prelim', 'conseqs', 'counts', 'unmapped', 'n_remaps', 'log'):
        assert got[key] == ref[key], key
