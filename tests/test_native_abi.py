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
