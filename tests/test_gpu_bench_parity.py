"""bench.py's parity legs at small size (the configuration-size runs are in
profiles/r06/): the consensus leg with the consensus-distance filter on
mixed HIV-1 regions (several consensuses, so the oracle step's filter runs),
and --parity-full over the whole input in chunks that do not divide it."""
import json
import os
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

pytestmark = pytest.mark.gpu


def _bench(args, timeout=500):
    env = dict(os.environ)
    for k in ('WORLD_SIZE', 'RANK', 'LOCAL_RANK'):
        env.pop(k, None)
    out = subprocess.run([sys.executable, os.path.join(REPO, 'bench.py')] + args, env=env, cwd=REPO,
                         capture_output=True, text=True, timeout=timeout)
    assert out.returncode == 0, out.stderr[-3000:]
    lines = [ln for ln in out.stdout.splitlines() if ln.startswith('{"metric"')]
    assert len(lines) == 1, out.stdout[-2000:]
    return json.loads(lines[0])


@pytest.mark.timeout(600)
def test_consensus_leg_with_the_filter():
    d = _bench(['--genomes', 'hiv', '--pairs', '30000', '--steps', '1', '--warmup', '0', '--no-e2e',
                '--no-cpu-baseline', '--cpu-sample', '30000'])
    p = d['parity']
    assert p['record_mismatches'] == 0
    c = p['consensus']
    assert len(c['unfiltered_per_pass'][0]) >= 2, c      # the filter ran
    assert c['prelim_equal'] and c['passes_equal'] and c['final_equal'], c
    assert p['consensus_equal'] is True


@pytest.mark.timeout(600)
def test_parity_full_in_uneven_chunks():
    d = _bench(['--pairs', '20000', '--steps', '1', '--warmup', '0', '--no-e2e', '--no-cpu-baseline',
                '--iterations', '2', '--force-iterations', '--parity-full', '7000'])
    w = d['parity']['whole_input']
    assert w['units_checked'] == 20000 and w['chunk_units'] == 7000
    assert [p['pass'] for p in w['passes']] == ['prelim', 'remap-1', 'remap-2']
    assert all(p['reads'] == 40000 for p in w['passes'])
    assert w['record_mismatches'] == 0
