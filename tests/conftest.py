"""Shared pytest setup: the `gpu` marker and import paths.

CPU tests (-m "not gpu") check the oracle against the committed golden
vectors and the host logic; GPU tests (-m gpu) call the HIP path through the
C-ABI and compare it with the oracle."""
import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (os.path.join(REPO, 'oracle'), os.path.join(REPO, 'micall-lite_amd'),
          os.path.join(REPO, 'tests')):
    if p not in sys.path:
        sys.path.insert(0, p)

GOLDEN = os.path.join(REPO, 'tests', 'golden')


def pytest_configure(config):
    config.addinivalue_line('markers', 'gpu: needs an MI355X (runs the HIP path)')


@pytest.fixture(scope='session')
def golden_dir():
    return GOLDEN
