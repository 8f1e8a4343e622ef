"""micall_amd.run_micall: the reference's bin/micall run unchanged with its
micall.core / micall.utils imports bound to the drop-ins (bin/micall:10-17).

A stand-in script with bin/micall's import block must see the drop-in
modules and bowtie2's path/version check must pass without a bowtie2
executable.  When the reference tree is present (the dev container), every
name its bin/micall imports must resolve through the launcher."""
import os
import re
import subprocess
import sys

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
PKG = os.path.join(REPO, 'micall-lite_amd')
IMPORTS = '''from micall.core.parse_interop import read_errors, write_phix_csv
from micall.core.filter_quality import report_bad_cycles
from micall.core.censor_fastq import censor
from micall.core.prelim_map import prelim_map
from micall.core.remap import remap
from micall.core.sam2aln import sam2aln
from micall.core.aln2counts import aln2counts
from micall.utils.externals import Bowtie2
'''


def _run(script_text, tmp_path):
    script = tmp_path / 'micall_script'
    script.write_text(script_text)
    env = dict(os.environ, PYTHONPATH=PKG + os.pathsep + os.environ.get('PYTHONPATH', ''))
    env.pop('WORLD_SIZE', None)
    return subprocess.run([sys.executable, '-m', 'micall_amd.run_micall', str(script), 'a1', 'a2'],
                          capture_output=True, text=True, env=env, timeout=120)


def test_imports_resolve_to_the_dropins(tmp_path):
    body = IMPORTS + '''
import sys
for f in (read_errors, write_phix_csv, report_bad_cycles, censor, prelim_map, remap, sam2aln,
          aln2counts):
    print(f.__module__)
b = Bowtie2(execname='bowtie2')
print('version', b.version, sys.argv[1:])
'''
    out = _run(body, tmp_path)
    assert out.returncode == 0, out.stderr
    mods = out.stdout.split('\n')[:8]
    assert all(m.startswith('micall_amd.') for m in mods), mods
    assert "version 2.2.8 ['a1', 'a2']" in out.stdout


def test_reference_bin_micall_imports_are_covered(tmp_path):
    ref = '/root/reference/bin/micall'
    if not os.path.exists(ref):
        pytest.skip('reference tree absent')
    text = open(ref).read()
    lines = [ln for ln in text.split('\n') if re.match(r'from micall\.', ln)]
    assert lines
    body = '\n'.join(lines) + '\nprint("ok")\n'
    out = _run(body, tmp_path)
    assert out.returncode == 0, out.stderr
    assert out.stdout.strip().endswith('ok')
