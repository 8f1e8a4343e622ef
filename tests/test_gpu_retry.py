"""The grow-and-retry paths of the HIP library under forced overflows.

Three device buffers are sized by a guess and grown when a launch asks for
more, with the launch run again:

- the CIGAR pool of a mapping pass (`mh_map.hip` run_map: the pass restarts
  from k_seed, since k_rescue rewrote the candidates of the mates it rescued
  and their slots point into the replaced pool: the bug fixed in d40a5b9);
- the pileup's insertion-token events and their bytes (`mh_pileup.hip`
  run_pileup);
- the distinct-token bytes of the token aggregation (run_token_aggregate).

`mh_test_set_capacities` starts each of them tiny, so every pass of the
parity tests below goes through its retry; `mh_retry_counts` proves the
retry was taken, and the results must stay bit-exact with the oracle (the
reference behaviour these preserve: remap.py:141-306 for the pileup,
bowtie2's SAM for the mapper)."""
import numpy as np
import pytest

import oracle
import test_gpu_parity as par
from micall_amd import _native

pytestmark = pytest.mark.gpu


@pytest.fixture
def tiny():
    c = _native.Context(0)
    c.test_set_capacities(cigar_pool_words=300, pileup_events=3, pileup_event_bytes=8,
                          token_bytes=2)
    yield c
    c.close()


@pytest.mark.parametrize('mode', [oracle.E2E, oracle.LOCAL])
def test_map_pol_through_pool_retry(tiny, mode):
    par.test_map_pol_vs_oracle(tiny, mode)
    assert tiny.retry_counts()['cigar_pool'] == 1


@pytest.mark.parametrize('mode', [oracle.E2E, oracle.LOCAL])
def test_mate_rescue_through_pool_retry(tiny, mode):
    """d40a5b9's scenario: rescued mates' candidates and a replaced pool."""
    par.test_mate_rescue_vs_oracle(tiny, mode)
    assert tiny.retry_counts()['cigar_pool'] == 1
    assert tiny.map_stats()[4] > 150          # the rescue launch ran in the retried pass


@pytest.mark.parametrize('mode,q', [(oracle.LOCAL, 20), (oracle.E2E, 0)])
def test_pileup_through_event_and_token_retries(tiny, mode, q):
    par.test_pileup_vs_oracle(tiny, mode, q)
    r = tiny.retry_counts()
    assert r['cigar_pool'] == 1
    assert r['pileup_events'] == 1
    assert r['token_bytes'] == 1


@pytest.mark.parametrize('q', [0, 20])
def test_pileup_rows_through_event_retry(tiny, q):
    """Source 1 (rows read back from text) with leading-gap CIGARs."""
    rng = np.random.default_rng(41 + q)
    par._rows_case_vs_oracle(tiny, par._random_cigar_sam(rng, 300), q)
    raw_events = sum(count for _, _, _, count in tiny.pileup_fetch()['events'])
    assert raw_events >= 3                   # > 3 events or > 8 bytes: past the imposed buffers
    assert tiny.retry_counts()['pileup_events'] == 1


def test_pool_grows_with_a_larger_batch():
    """A small paired batch, then a 40x larger one with mate rescues on the
    same context and no imposed capacity: the pool is sized again for the
    larger pass up front (no retry), and the records match the oracle."""
    c = _native.Context(0)
    try:
        names, seqs, quals = par._reads(40, 3)
        ref = par._oracle_alns([par.POL], oracle.LOCAL, seqs, quals, True)
        par._assert_same(par._gpu_alns(c, ['HIV1B-pol-seed'], [par.POL], oracle.LOCAL, seqs, quals,
                                       True), ref, seqs)
        par.test_mate_rescue_vs_oracle(c, oracle.LOCAL)
        par.test_map_pol_vs_oracle(c, oracle.E2E)
        assert c.retry_counts() == dict(cigar_pool=0, pileup_events=0, token_bytes=0, gotoh_wait=0)
    finally:
        c.close()


def test_caps_reset_to_library_sizing(tiny):
    """Capacity 0 returns to the library's own sizing: no retries after."""
    names, seqs, quals = par._reads(300, 9, indel_rate=0.01)
    par._gpu_alns(tiny, ['HIV1B-pol-seed'], [par.POL], oracle.LOCAL, seqs, quals, True)
    assert tiny.retry_counts()['cigar_pool'] == 1
    tiny.test_set_capacities()
    par._gpu_alns(tiny, ['HIV1B-pol-seed'], [par.POL], oracle.LOCAL, seqs, quals, True)
    tiny.pileup(0, 20, [len(par.POL)])
    tiny.pileup_fetch()
    assert tiny.retry_counts() == dict(cigar_pool=1, pileup_events=0, token_bytes=0, gotoh_wait=0)


def test_gotoh_wait_timeout_is_retried():
    """k_gotoh's strips wait for the strip above by polling its boundary
    cells; a wait past its real-time limit fails the launch (-4) and the
    batch runs once more with the default 20 s limit.  With a first-attempt
    limit of 1 tick (10 ns) some strip of a 3 kb alignment gives up, the retry
    runs, and the result still equals the oracle (_gotoh2.c:442-541)."""
    c = _native.Context(0)
    try:
        c.test_set_gotoh_wait(1)
        rng = np.random.default_rng(3)
        conseq = par.synth.sample_genome(par.POL, rng, 0.1, 0.004).tobytes().decode()[100:3000]
        mat, alpha = [5, -4, -4, -4, 0, -4, 5, -4, -4, 0, -4, -4, 5, -4, 0, -4, -4, -4, 5, 0,
                      0, 0, 0, 0, 0], 'ACGT?'
        want = oracle.gotoh_align(par.POL, conseq, 15, 3, True, alpha, mat)
        assert c.gotoh_align(par.POL, conseq, 15, 3, True, alpha, mat) == want
        assert c.retry_counts()['gotoh_wait'] == 1
    finally:
        c.close()
