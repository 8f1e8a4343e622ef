"""bowtie2 / bowtie2-build-s command contract (micall_amd/bowtie2_cli.py,
micall-lite_amd/bin) on the CPU: --version as externals.py reads it, the six
index names prelim_map.py / remap.py remove, argument checking.  Mapping
through the commands is tests/test_gpu_bowtie2_cli.py."""
import os
import subprocess
import sys

import pytest

from micall_amd import bowtie2_cli

BIN = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), 'micall-lite_amd',
                   'bin')


@pytest.mark.parametrize('cmd', ['bowtie2', 'bowtie2-align-s', 'bowtie2-build', 'bowtie2-build-s'])
def test_version_last_token(cmd):
    out = subprocess.run([sys.executable, os.path.join(BIN, cmd), '--version'], check=True,
                         stdout=subprocess.PIPE, stderr=subprocess.STDOUT, universal_newlines=True).stdout
    # externals.py:164-165: stdout.split('\n')[0].split()[-1]
    assert out.split('\n')[0].split()[-1] == '2.2.8'


def test_build_writes_the_six_index_names(tmp_path):
    fasta = tmp_path / 'micall.fasta'
    fasta.write_text('>HIV1B-pol-seed some description\nACGTNNAC\nGGTT\n>R2\nTTTT\n')
    template = str(tmp_path / 'reference')
    rc = subprocess.run([sys.executable, os.path.join(BIN, 'bowtie2-build-s'), '--wrapper', 'micall-0',
                         '--quiet', '-f', str(fasta), template]).returncode
    assert rc == 0
    for suffix in bowtie2_cli.BT2_SUFFIXES:   # prelim_map.py:158-161, remap.py:656-657
        assert os.path.exists('{}.{}.bt2'.format(template, suffix))
    names, seqs = bowtie2_cli.fasta_records(template + '.1.bt2')
    assert names == ['HIV1B-pol-seed', 'R2']
    assert seqs == ['ACGTNNACGGTT', 'TTTT']


@pytest.mark.parametrize('argv', [
    ['-x', 't', '-1', 'a.fq'],                        # -1 without -2
    ['-x', 't', '-U', 'a.fq', '-1', 'b', '-2', 'c'],  # both
    ['-1', 'a', '-2', 'b'],                           # no -x
    ['-x', 't', '-U', 'a.fq', '--very-fast'],         # not in the contract
    ['-x', 't', '-U'],                                # missing value
])
def test_bad_arguments_are_refused(argv):
    with pytest.raises(bowtie2_cli.UsageError):
        bowtie2_cli.parse_align_args(argv)


def test_reference_arguments_parse():
    # prelim_map.py:114-131 and remap.py:701-721
    opts, sw = bowtie2_cli.parse_align_args(
        ['--wrapper', 'micall-0', '--quiet', '-x', 'ref', '-1', 'r1', '-2', 'r2', '--rdg', '10,3',
         '--rfg', '10,3', '--no-hd', '--local', '-X', '1200', '-p', '4'])
    assert opts['-x'] == 'ref' and opts['-X'] == '1200' and bowtie2_cli.pair_of(opts['--rdg']) == (10, 3)
    assert sw == {'--quiet', '--no-hd', '--local'}


def test_header():
    h = bowtie2_cli.sam_header(['a', 'b'], ['ACGT', 'AC'], ['-x', 'r'])
    assert h.splitlines()[:3] == ['@HD\tVN:1.0\tSO:unsorted', '@SQ\tSN:a\tLN:4', '@SQ\tSN:b\tLN:2']
    assert h.splitlines()[3].startswith('@PG\tID:bowtie2\tPN:bowtie2\tVN:2.2.8')
