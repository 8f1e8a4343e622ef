"""bench.py's multi-rank paths (what the driver runs at N = 2..8 over RCCL),
rehearsed with two ranks on the one GPU of the test box over gloo
(MICALL_BENCH_BACKEND=gloo): per-rank read blocks, the all-reduced tallies
and pileup, max-over-ranks timing and the single JSON line of rank 0; the
file-to-file legs (end_to_end with many gzip members and with one member)
and the --stage chain leg run the sharded drop-ins over files that hold
both ranks' blocks."""
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


def _bench(args, timeout=400, launcher=True):
    env = dict(os.environ, MICALL_BENCH_BACKEND='gloo')
    for k in ('WORLD_SIZE', 'RANK', 'LOCAL_RANK'):
        env.pop(k, None)
    pre = ([sys.executable, '-m', 'torch.distributed.run', '--nnodes=1', '--nproc-per-node', '2',
            '--master-addr', '127.0.0.1', '--master-port', str(_free_port())] if launcher
           else [sys.executable])
    cmd = pre + [os.path.join(REPO, 'bench.py'), '--gpus', '2'] + args
    out = subprocess.run(cmd, env=env, cwd=REPO, capture_output=True, text=True, timeout=timeout)
    assert out.returncode == 0, out.stderr[-3000:]
    lines = [ln for ln in out.stdout.splitlines() if ln.startswith('{"metric"')]
    assert len(lines) == 1, out.stdout[-2000:]
    return json.loads(lines[0])


@pytest.mark.gpu
@pytest.mark.timeout(600)
def test_bench_two_ranks_gloo():
    pairs = 20000
    d = _bench(['--pairs', str(pairs), '--steps', '1', '--warmup', '1', '--no-cpu-baseline'])
    assert d['n_gpus'] == 2 and d['scaling'] == 'weak'
    assert d['value'] > 0 and d['ms_per_step'] > 0
    # every read of both ranks' blocks maps to the pol consensus; the tallies
    # are the all-reduced sums over the two ranks
    assert sum(d['result']['mapped_lines'].values()) == 2 * 2 * pairs
    assert list(d['result']['conseqs']) == ['HIV1B-pol-seed']
    # rank 0's records of its first pairs equal the oracle's
    assert d['parity']['record_mismatches'] == 0 and d['parity']['units_checked'] == pairs
    # the file-to-file legs over both ranks' blocks: each rank read about
    # half of the files and wrote about half of the rows
    for key, mode in (('end_to_end', 'members'), ('end_to_end_single_member', 'member-part')):
        e = d[key]
        assert e['n_gpus'] == 2 and e['value'] > 0, e
        io = e['per_rank_io']
        assert io['fastq_mode'] == mode, (key, io)
        for k in ('fastq_file_bytes', 'written_bytes'):
            assert max(io[k]) <= 0.75 * sum(io[k]), (key, k, io)


@pytest.mark.gpu
@pytest.mark.timeout(600)
def test_bench_chain_two_ranks_gloo():
    """--stage chain under torchrun: censor (one-member input split by rank),
    prelim_map, remap, sam2aln, aln2counts on the shared files; one line with
    the median run and the per-rank I/O of the sharded stages."""
    d = _bench(['--stage', 'chain', '--pairs', '20000', '--steps', '3', '--warmup', '0'])
    assert d['n_gpus'] == 2 and d['config']['pairs'] == 40000
    assert len(d['all_runs_s']) == 3
    assert abs(sorted(d['all_runs_s'])[1] - d['ms_per_step'] / 1e3) < 0.002     # the median run
    io = d['per_rank_io_last_run']
    assert io['censor']['fastq_mode'] == 'member-part', io
    assert io['prelim_map']['fastq_mode'] == 'members', io
    for stage in ('censor', 'prelim_map', 'remap'):
        w = io[stage]['written_bytes']
        assert min(w) > 0 and max(w) <= 0.75 * sum(w), (stage, w)


@pytest.mark.gpu
@pytest.mark.timeout(600)
def test_bench_gpus_2_launches_its_own_ranks():
    """Plain `bench.py --gpus 2` (no torchrun around it, as the driver may
    call it): bench.py starts the two ranks itself as a child
    torch.distributed.run and relays rank 0's line, which reports the world
    the process group really had."""
    pairs = 10000
    d = _bench(['--pairs', str(pairs), '--steps', '1', '--warmup', '1', '--no-cpu-baseline',
                '--no-e2e'], launcher=False)
    assert d['n_gpus'] == 2
    c = d['config']
    assert c['dist_world'] == 2 and c['dist_backend'] == 'gloo' and len(c['rank_devices']) == 2, c
    assert sum(d['result']['mapped_lines'].values()) == 2 * 2 * pairs
