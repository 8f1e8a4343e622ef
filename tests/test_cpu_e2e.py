"""The CPU end-to-end restatement that bench.py times as the end-to-end CPU
baseline (oracle/cpu_e2e.py: the reference's prelim_map() + remap() structure
with the oracle C mapper in bowtie2's place) writes the reference's files on
the golden e2e cases -- so the CPU figure is for the same work and the same
outputs as the drop-ins."""
import gzip
import io
import os

import pytest

import cpu_e2e
from micall_amd import projects


def _golden(d, name):
    with gzip.open(os.path.join(d, name + '.gz'), 'rt') as f:
        return f.read()


@pytest.mark.parametrize('case', ['syn_pol', 'syn_chimera', 'syn_unpaired300', 'micro_2090A-HCV',
                                  'syn_maxremaps', 'syn_hiv3', 'c1_example'])
def test_cpu_e2e_writes_the_golden_files(golden_dir, tmp_path, case):
    d = os.path.join(golden_dir, 'e2e', case)
    r1 = os.path.join(d, 'R1.fastq.gz')
    r2 = os.path.join(d, 'R2.fastq.gz')
    r2 = r2 if os.path.exists(r2) else None
    cfg = projects.load_default()
    seeds = cfg.seed_sequences()
    prelim = io.StringIO()
    cpu_e2e.prelim_map(r1, r2, prelim, seeds, 4)
    assert prelim.getvalue() == _golden(d, 'prelim.csv')
    outs = {k: io.StringIO() for k in ('remap.csv', 'remap_counts.csv', 'remap_conseq.csv')}
    un1, un2 = open(tmp_path / 'u1', 'w+'), open(tmp_path / 'u2', 'w+')
    prelim.seek(0)
    cpu_e2e.remap(r1, r2, prelim, outs['remap.csv'], outs['remap_counts.csv'],
                  outs['remap_conseq.csv'], un1, un2, cfg.all_region_sequences(),
                  {k: cfg.getSeedGroup(k) for k in seeds}, str(tmp_path), 4)
    un1.close()
    un2.close()
    for name, buf in outs.items():
        assert buf.getvalue() == _golden(d, name), name
    assert open(tmp_path / 'u1').read() == _golden(d, 'unmapped1.fastq')
    assert open(tmp_path / 'u2').read() == _golden(d, 'unmapped2.fastq')
