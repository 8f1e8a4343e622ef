"""censor_fastq.censor on the device (micall_amd.censor_fastq, mh_censor.hip)
against outputs of the reference's own censor() (tests/golden/censor/):
the censor_fastq_test.py scenarios (plain text) and a synthetic multi-tile
FASTQ pair with bad cycles derived from a synthetic ErrorMetricsOut.bin,
gzip in and out, chained as bin/micall:90-126 chains them."""
import csv
import gzip
import io
import json
import os

import pytest

import og_censor
from micall_amd import censor_fastq

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))
CDIR = os.path.join(HERE, 'golden', 'censor')
G = json.load(open(os.path.join(CDIR, 'censor_golden.json')))


@pytest.mark.parametrize('k', range(len(G['cases'])))
def test_censor_scenarios_match_reference(k):
    case = G['cases'][k]
    dest, summary = io.BytesIO(), io.StringIO()
    censor_fastq.censor(io.BytesIO(case['fastq'].encode()),
                        [dict(tile=t, cycle=c) for t, c in case['bad_cycles']], dest,
                        use_gzip=False, summary_file=summary)
    assert dest.getvalue().decode() == case['censored']
    assert summary.getvalue() == case['summary']


def test_censor_pair_matches_reference_gzip():
    reader = csv.DictReader(io.StringIO(G['bad_cycles_csv']))
    for mate in (1, 2):
        dest, summary = io.BytesIO(), io.StringIO()
        with open(os.path.join(CDIR, 'R{}.fastq.gz'.format(mate)), 'rb') as src:
            censor_fastq.censor(src, reader, dest, use_gzip=True, summary_file=summary)
        with gzip.open(os.path.join(CDIR, 'R{}.censor.fastq.gz'.format(mate))) as f:
            assert gzip.decompress(dest.getvalue()) == f.read()
        assert summary.getvalue() == G['summary_r{}'.format(mate)]


def test_censor_large_vs_oracle():
    """Many tiles, long reads, CRLF line ends and trailing spaces, random bad
    cycles in both directions."""
    import random
    rng = random.Random(3)
    recs, bad = [], set()
    for t in range(1101, 1121):
        for c in rng.sample(range(1, 301), 12):
            bad.add((str(t), c if rng.random() < 0.5 else -c))
    for i in range(5000):
        n = rng.randint(30, 300)
        seq = ''.join(rng.choice('ACGTN') for _ in range(n))
        qual = ''.join(rng.choice('#+5?AFG') for _ in range(n))
        end = '\r\n' if i % 17 == 0 else ('  \n' if i % 23 == 0 else '\n')
        recs.append('@M1:2:F:1:{}:{}:{} {}:N:0:1\n{}{}+\n{}{}'.format(
            1101 + i % 24, i, i, 1 + i % 2, seq, end, qual, end))
    data = ''.join(recs).encode()
    want, n, total = og_censor.censor_bytes(data, bad)
    dest, summary = io.BytesIO(), io.StringIO()
    censor_fastq.censor(io.BytesIO(gzip.compress(data)),
                        [dict(tile=t, cycle=str(c)) for t, c in sorted(bad)], dest,
                        use_gzip=True, summary_file=summary)
    assert gzip.decompress(dest.getvalue()) == want
    assert summary.getvalue() == 'avg_quality,base_count\n{},{}\n'.format(repr(total / n), n)


@pytest.mark.parametrize('use_gzip', [True, False])
def test_censor_file_to_file_streamed(tmp_path, use_gzip):
    """The drop-in on real files (bin/micall's call): the source mmap'd and
    each output block written with pwrite as it is made
    (mh_censor_staged_write), at the handle's position (bytes already
    written through the handle are kept), for a file large enough to make
    many blocks and for an empty one."""
    import random
    rng = random.Random(11)
    bad = {(str(1101 + t), c) for t in range(4) for c in rng.sample(range(1, 151), 6)}
    recs = []
    for i in range(120000):
        seq = ''.join(rng.choice('ACGT') for _ in range(150))
        recs.append('@M1:2:F:1:{}:{}:{} 1:N:0:1\n{}\n+\n{}\n'.format(1101 + i % 4, i, i, seq, 'F' * 150))
    data = ''.join(recs).encode()
    want, n, total = og_censor.censor_bytes(data, bad)
    for payload, expect in ((data, want), (b'', b'')):
        src_path, dst_path = tmp_path / 'in.fastq', tmp_path / 'out.fastq'
        src_path.write_bytes(gzip.compress(payload, 1) if use_gzip else payload)
        lead = b'lead bytes\n'
        with open(src_path, 'rb') as src, open(dst_path, 'wb') as dst:
            dst.write(lead)
            censor_fastq.censor(src, [dict(tile=t, cycle=str(c)) for t, c in sorted(bad)], dst,
                                use_gzip=use_gzip)
            dst.write(b'tail')
        out = dst_path.read_bytes()
        assert out.startswith(lead) and out.endswith(b'tail')
        body = out[len(lead):-4]
        assert (gzip.decompress(body) if use_gzip else body) == expect
