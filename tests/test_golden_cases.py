"""The e2e goldens (tests/golden/e2e/, written by the stock reference
pipeline through tests/golden/gen_golden.py e2e) hold the scenarios the GPU
parity tests rely on.  CPU only: this checks the fixtures, not the product."""
import csv
import gzip
import io
import os

import pytest

E2E = os.path.join(os.path.dirname(os.path.abspath(__file__)), 'golden', 'e2e')
MICROTESTS = ['1234A-V3LOOP', '2000A-V3LOOP', '2010A-V3LOOP', '2020A-GP41', '2030A-V3LOOP',
              '2040A-HLA-B', '2050A-V3LOOP', '2060A-V3LOOP', '2070A-PR', '2080A-V3LOOP',
              '2090A-HCV', '2100A-HCV-1337B-V3LOOP']


def _rows(case, name):
    with gzip.open(os.path.join(E2E, case, name + '.gz'), 'rt') as f:
        return list(csv.DictReader(io.StringIO(f.read())))


def _read(path):
    with gzip.open(path, 'rt') as f:
        return f.read()


def _counts(case):
    return {r['type']: r['count'] for r in _rows(case, 'remap_counts.csv')}


def test_every_reference_microtest_is_a_case():
    # micall/tests/microtest/README.md:14-29
    for stem in MICROTESTS:
        assert os.path.isdir(os.path.join(E2E, 'micro_' + stem)), stem


def test_c1_example_uses_slash_suffixed_names():
    # BASELINE config C1: examples/HIV1C-pol (9,600 pairs named CONSENSUS_C-N/1, /2)
    with gzip.open(os.path.join(E2E, 'c1_example', 'R1.fastq.gz'), 'rt') as f:
        head = f.readline()
    assert head.startswith('@CONSENSUS_C-') and head.rstrip().endswith('/1')
    rows = _rows('c1_example', 'remap.csv')
    assert len(rows) == 19200
    # bowtie2 strips /1 /2, so both mates share one qname and pair up
    assert rows[0]['qname'] == rows[1]['qname'] and not rows[0]['qname'].endswith('/1')


def test_chimera_case_splits_mixed_reference_pairs():
    # remap.py:613-634: pairs with RNEXT naming another reference are taken
    # out and mapped again; remap-final then exceeds the last pass's counts
    c = _counts('syn_chimera')
    for ref in ('HIV1B-gag-seed', 'HIV1B-env-seed'):
        assert int(c['remap-final ' + ref]) > int(c['remap-1 ' + ref])
    remap = _rows('syn_chimera', 'remap.csv')
    assert all(r['rnext'] in ('=', '*') for r in remap)


def test_maxremaps_case_stops_on_max_remaps():
    # growing counts every pass, mapped fraction <= 0.95: only MAX_REMAPS
    # (remap.py:602-603) can end the loop, after pass 3
    c = _counts('syn_maxremaps')
    passes = [int(c['remap-%d SARS-CoV-2' % k]) for k in (1, 2, 3)]
    assert passes[0] < passes[1] < passes[2]
    assert passes[2] / float(c['raw']) <= 0.95
    assert 'remap-4 SARS-CoV-2' not in c


@pytest.mark.parametrize('case', ['syn_noseed', 'micro_2030A-V3LOOP'])
def test_no_seed_cases_record_the_reference_failure(case):
    # no seed reaches the threshold: the loop never runs and the reference's
    # cleanup raises (remap.py:653-655); the drop-in completes
    with open(os.path.join(E2E, case, 'reference_raises.txt')) as f:
        assert f.read().startswith('FileNotFoundError temp.fasta')
    c = _counts(case)
    assert not any(k.startswith('remap-') for k in c)
    assert c['unmapped'] == c['raw']


def test_c5_chain_goldens_hold_their_scenarios(golden_dir):
    """tests/golden/chain: bad tile-cycles censored in R1 (trailing bad
    cycles dropped), R2 of the paired case left uncensored by the exhausted
    DictReader (bin/micall:116,126), unpaired 1x300 reads mapped (-U)."""
    import json
    for case, paired in (('c5_unpaired300', False), ('c5_paired251', True)):
        d = os.path.join(golden_dir, 'chain', case)
        bad = _read(os.path.join(d, 'bad_cycles.csv.gz')).splitlines()[1:]
        assert 30 <= len(bad) <= 80
        raw = _read(os.path.join(d, 'R1.fastq.gz')).splitlines()
        cen = _read(os.path.join(d, 'R1.censor.fastq.gz')).splitlines()
        lengths = json.load(open(os.path.join(d, 'read_lengths.json')))
        assert len(raw[1]) == lengths[0]
        shorter = sum(1 for a, b in zip(raw[1::4], cen[1::4]) if len(b) < len(a))
        assert shorter > 0
        if paired:
            assert (_read(os.path.join(d, 'R2.fastq.gz')) ==
                    _read(os.path.join(d, 'R2.censor.fastq.gz')))
        else:
            assert not os.path.exists(os.path.join(d, 'R2.fastq.gz'))
        counts = _read(os.path.join(d, 'remap_counts.csv.gz'))
        assert 'remap-final HIV1B-pol-seed' in counts
