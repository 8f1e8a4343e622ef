"""The device index cache (mh_api.cpp mh_index_build) keys large reference
sets by a 64-bit signature; a hit is used only when the cached reference
bytes compare equal.  MH_INDEX_FORCE_COLLISION=1 gives every set the same
signature: the second set must then be built, not served from the cache."""
import os

import numpy as np
import pytest

import oracle
from micall_amd import _native

pytestmark = pytest.mark.gpu


def _refs(seed):
    rng = np.random.default_rng(seed)
    return [''.join('ACGT'[x] for x in rng.integers(0, 4, 40000)) for _ in range(2)]


def test_signature_collision_rebuilds():
    a, b = _refs(1), _refs(2)
    seqs = [b[i % 2][300 * i:300 * i + 251] for i in range(64)]
    quals = ['I' * 251] * len(seqs)
    mode = oracle.E2E
    os.environ['MH_INDEX_FORCE_COLLISION'] = '1'
    ctx = _native.Context(0)
    try:
        for refs in (a, b, a, b):     # every build after the first is a signature hit
            ctx.index_build(['r0', 'r1'], refs, oracle.seed_len(mode))
            ctx.reads_load(seqs, quals, False)
            ctx.map(_native.params(mode))
            got = ctx.fetch()
            ix = oracle.Index(refs, oracle.seed_len(mode))
            want = np.frombuffer(bytes(oracle.map_reads(ix, oracle.params(mode), seqs, quals, False)),
                                 dtype=_native.ALN_DTYPE)[:len(seqs)]
            assert (got['ref'] == want['ref']).all() and (got['pos'] == want['pos']).all()
            if refs is b:     # reads drawn from set b map exactly where they were drawn
                assert (got['ref'] == np.arange(64) % 2).all() and (got['pos'] == 300 * np.arange(64)).all()
            else:
                assert (got['ref'] < 0).all()
    finally:
        ctx.close()
        del os.environ['MH_INDEX_FORCE_COLLISION']
