"""The C-ABI library builds for gfx950, loads, and exports every entry point
include/micall_hip.h declares (no compute calls: runs without a GPU)."""
import os
import re
import subprocess

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _declared():
    with open(os.path.join(REPO, 'include', 'micall_hip.h')) as f:
        text = f.read()
    return sorted(set(re.findall(r'^int (mh_\w+)\(', text, re.M)))


@pytest.fixture(scope='module')
def native():
    so = os.path.join(REPO, 'micall-lite_amd', 'micall_amd', 'libmicall_hip.so')
    if not os.path.exists(so):
        subprocess.run(['make', '-s', '-j8', '-C', os.path.join(REPO, 'micall-lite_amd', 'csrc')],
                       check=True)
    from micall_amd import _native
    return _native


def test_every_declared_symbol_is_exported(native):
    L = native.lib()
    names = _declared()
    assert len(names) >= 25
    for name in names:
        assert hasattr(L, name), name
    # and the binding declares a signature for every one of them
    assert set(names) <= set(native.EXPORTED)


def test_version_and_errors(native):
    assert native.lib().mh_version() == 1
    assert native.levenshtein('kitten', 'sitting') == 3


def test_no_cpu_fallback_without_gpu(native):
    """On a host without a GPU the context refuses to start (no fallback)."""
    if native.device_count() > 0:
        pytest.skip('a GPU is visible')
    with pytest.raises(native.NativeUnavailable):
        native.Context(0)


def test_levenshtein_bit_parallel_matches_dp(native):
    """mh_levenshtein (bit-vector, 64-row blocks) against the oracle's
    cell-by-cell DP, across block boundaries and with the consensus alphabet."""
    import random

    import oracle
    rng = random.Random(7)
    alphabet = 'ACGTN-'
    lengths = [0, 1, 2, 63, 64, 65, 127, 128, 129, 300, 701]
    for la in lengths:
        for lb in (0, 1, 64, 65, la, la + 3, max(la - 5, 0), 500):
            a = ''.join(rng.choice(alphabet) for _ in range(la))
            # b: a mutated copy half the time (small distances), random otherwise
            if rng.random() < 0.5 and la:
                b = list(a)
                for _ in range(rng.randint(0, 8)):
                    op, p = rng.randint(0, 2), rng.randrange(len(b) + 1)
                    if op == 0 and p < len(b):
                        b[p] = rng.choice(alphabet)
                    elif op == 1:
                        b.insert(p, rng.choice(alphabet))
                    elif b and p < len(b):
                        del b[p]
                b = ''.join(b)
            else:
                b = ''.join(rng.choice(alphabet) for _ in range(lb))
            assert native.levenshtein(a, b) == oracle.levenshtein(a, b), (la, len(b))
            assert native.levenshtein(b, a) == oracle.levenshtein(a, b), (la, len(b))


def test_levenshtein_batch_keeps_pair_order():
    """mh_levenshtein_batch runs its pairs longest first over host threads;
    each result still lands at its pair's index, and characters of b that a
    does not hold (mapped to one no-match symbol) count as mismatches."""
    import random

    from micall_amd import _native
    rng = random.Random(11)
    pairs = []
    for _ in range(40):
        la, lb = rng.randint(0, 400), rng.randint(0, 400)
        pairs.append((''.join(rng.choice('ACGT') for _ in range(la)),
                      ''.join(rng.choice('ACGTNxyz-') for _ in range(lb))))
    got = _native.levenshtein_many(pairs)
    assert got == [_native.levenshtein(a, b) for a, b in pairs]
    import oracle
    assert got[:8] == [oracle.levenshtein(a, b) for a, b in pairs[:8]]


def test_crc32_combine_matches_zlib(native):
    """mh_crc32_combine (the CRC-32 of A ++ B from crc(A), crc(B), |B|; the
    shift by |B| bytes as products of precomputed x^(2^k) mod P) equals
    zlib.crc32 of the concatenation, empty and odd lengths included."""
    import random
    import zlib
    rng = random.Random(5)
    for _ in range(300):
        a = rng.randbytes(rng.randint(0, 3000))
        b = rng.randbytes(rng.choice([0, 1, 2, 7, 8, 100, 4095, 70000]))
        got = native.crc32_combine(zlib.crc32(a), zlib.crc32(b), len(b))
        assert got == zlib.crc32(a + b)
