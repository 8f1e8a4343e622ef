"""
tests/golden/refharness.py -- fixture-generation helper, runs in the dev
container only (needs /root/reference; nothing under tests/ imports it at
test time).

Makes the read-only reference importable under Python 3.10:
  * `StringIO` / `cStringIO` (Python 2 names used by the reference tests)
    alias io.StringIO;
  * `Levenshtein` (python-Levenshtein, not installed) is replaced by a plain
    unit-cost edit distance -- the only function remap.py uses (:250);
  * `micall.alignment._gotoh2` is the reference's own C extension compiled
    from its source by `make -C oracle ref` into oracle/_ref/.
"""
import glob
import importlib.util
import io
import os
import sys
import types

REF = os.environ.get('MICALL_REFERENCE', '/root/reference')
REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def _edit_distance(a, b):
    prev = list(range(len(b) + 1))
    for i, ca in enumerate(a, 1):
        cur = [i]
        for j, cb in enumerate(b, 1):
            cur.append(min(prev[j] + 1, cur[j - 1] + 1, prev[j - 1] + (ca != cb)))
        prev = cur
    return prev[-1]


def setup():
    if REF not in sys.path:
        sys.path.insert(0, REF)
    for name in ('StringIO', 'cStringIO'):
        mod = types.ModuleType(name)
        mod.StringIO = io.StringIO
        sys.modules.setdefault(name, mod)
    lev = types.ModuleType('Levenshtein')
    lev.distance = _edit_distance
    sys.modules.setdefault('Levenshtein', lev)
    built = glob.glob(os.path.join(REPO, 'oracle', '_ref', '_gotoh2*.so'))
    if not built:
        import subprocess
        subprocess.run(['make', '-s', '-C', os.path.join(REPO, 'oracle'), 'ref'], check=True)
        built = glob.glob(os.path.join(REPO, 'oracle', '_ref', '_gotoh2*.so'))
    spec = importlib.util.spec_from_file_location('micall.alignment._gotoh2', built[0])
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    sys.modules['micall.alignment._gotoh2'] = mod
    import micall.alignment
    micall.alignment._gotoh2 = mod
    import micall.alignment.gotoh2 as g2
    sys.modules.setdefault('gotoh2', g2)
    return mod
