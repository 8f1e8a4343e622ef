"""bench.py's launch guards (host logic, no GPU): a line is never printed
for a world other than --gpus, and single-GPU stages refuse --gpus N."""
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(args, **env):
    e = dict(os.environ)
    for k in ('WORLD_SIZE', 'RANK', 'LOCAL_RANK'):
        e.pop(k, None)
    e.update(env)
    return subprocess.run([sys.executable, os.path.join(REPO, 'bench.py')] + args, env=e,
                          capture_output=True, text=True, timeout=120)


def test_world_mismatch_is_refused():
    out = _run(['--gpus', '2'], WORLD_SIZE='1', RANK='0', LOCAL_RANK='0')
    assert out.returncode != 0
    assert 'refusing' in out.stderr and '{"metric"' not in out.stdout


def test_single_gpu_stage_refuses_gpus_n():
    out = _run(['--gpus', '2', '--stage', 'sam2aln'])
    assert out.returncode != 0 and 'one GPU' in out.stderr


def test_self_launch_refuses_more_ranks_than_devices():
    # no GPU in the CPU suite's container: zero devices, so --gpus 2 over
    # RCCL is refused before any rank starts
    import torch
    if torch.cuda.device_count() >= 2:
        import pytest
        pytest.skip('node has GPUs')
    out = _run(['--gpus', '2'])
    assert out.returncode != 0 and 'GPU(s)' in out.stderr
