"""The oracle step's consensus-distance filter (cpu_pipeline.distance_filter,
used by timed_step, bench.py's cpu_baseline and the GPU parity tests at C4
size) against the SAM-level restatement oracle.sam_to_conseqs(is_filtered=
True), which tests/test_oracle_pileup.py pins to the reference's own
remap_test outputs: the same reads, one --local pass against the prelim
consensus set, the same consensus and the same kept set.  Reference:
remap.py:228-268 (filter), :129-138 (extract_relevant_seed)."""
import numpy as np
import pytest

import cpu_e2e
import cpu_pipeline
import oracle
from micall_amd import projects, synth

CFG = projects.load_default()
SEEDS = CFG.seed_sequences()
ALL = CFG.all_region_sequences()
GROUPS = {k: CFG.getSeedGroup(k) for k in SEEDS}


def _sam_path(pairs, conseqs):
    names, seqs, quals = synth.interleave(pairs)
    cn = list(conseqs)
    ix = oracle.Index([conseqs[k] for k in cn], oracle.seed_len(oracle.LOCAL))
    alns = oracle.map_reads(ix, oracle.params(oracle.LOCAL), seqs, quals, True, 8)
    lines = cpu_e2e._header(conseqs)
    for i in range(len(seqs)):
        lines.append('\t'.join(oracle.sam_fields(alns[i], oracle.qname_of(names[i], True), seqs[i],
                                                 quals[i], cn)) + '\n')
    report = {}
    out = oracle.sam_to_conseqs(lines, 20, seeds=ALL, is_filtered=True, filter_coverage=5.0,
                                distance_report=report, nuc_model=cpu_e2e.HYPHY_NUC)
    return out, report


@pytest.mark.parametrize('genomes', [
    ('HIV1B-pol-seed', 'HIV1B-env-seed', 'HIV1B-gag-seed', 'HIV1B-nef-seed'),
    ('HCV-1a', 'HCV-1b', 'HIV1B-pol-seed'),
], ids=['hiv_regions', 'hcv_genotypes'])
def test_step_filter_equals_sam_level_oracle(genomes):
    pairs = synth.make_pairs(2500, genomes={k: SEEDS[k] for k in genomes}, genome_seed=20261015,
                             read_seed=11)
    reads = np.stack([pairs['r1'], pairs['r2']], axis=1).reshape(-1, pairs['r1'].shape[1])
    quals = np.stack([pairs['q1'], pairs['q2']], axis=1).reshape(-1, pairs['q1'].shape[1])
    prep = cpu_pipeline.Prepared.from_arrays(reads, quals, True)
    final, _ = cpu_pipeline.timed_step(SEEDS, ALL, GROUPS, prep, 8, max_iterations=1)
    res = prep.result
    assert len(res['passes'][0]['unfiltered']) >= 2, res['passes']   # the filter ran
    want, report = _sam_path(pairs, res['prelim_conseqs'])
    assert final == want
    assert sorted(final) == res['passes'][0]['kept']
    # every unfiltered consensus was measured against every seed
    assert set(report) == set(res['passes'][0]['unfiltered'])
