"""bench.py's cpu_baseline leg (oracle/cpu_pipeline.timed_step: og_map,
og_rows_from_alns and og_pileup_mt with OpenMP, reads packed before timing)
computes the same consensus as the plain oracle step (run_step: per-read
Python marshalling, serial og_pileup).  CPU only."""
import numpy as np

import cpu_pipeline
import oracle
from micall_amd import projects, synth


def test_timed_step_matches_run_step():
    cfg = projects.load_default()
    seed_set = cfg.seed_sequences()
    groups = {k: cfg.getSeedGroup(k) for k in seed_set}
    pairs = synth.make_pairs(3000, genomes={'HIV1B-pol-seed': seed_set['HIV1B-pol-seed']},
                             genome_seed=5, read_seed=6, indel_rate=0.01)
    _, seqs, quals = synth.interleave(pairs)
    want, _ = cpu_pipeline.run_step(seed_set, cfg.all_region_sequences(), groups, seqs, quals,
                                    True, 4)
    prep = cpu_pipeline.Prepared(seqs, quals, True)
    got, _ = cpu_pipeline.timed_step(seed_set, cfg.all_region_sequences(), groups, prep, 4)
    assert got == want and got
    # the records of both passes stay readable (bench.py's parity leg), and
    # the array-built preparation maps the same
    res = prep.result
    assert res['remap_names'] == list(res['prelim_conseqs'])
    reads = np.stack([pairs['r1'], pairs['r2']], axis=1).reshape(-1, pairs['r1'].shape[1])
    qual = np.stack([pairs['q1'], pairs['q2']], axis=1).reshape(-1, pairs['q1'].shape[1])
    recs = cpu_pipeline.map_arrays([seed_set[k] for k in res['prelim_names']], oracle.E2E,
                                   reads, qual, True, 4)
    assert recs.tobytes() == res['prelim'].tobytes()
    again = cpu_pipeline.Prepared.from_arrays(reads, qual, True)
    got2, _ = cpu_pipeline.timed_step(seed_set, cfg.all_region_sequences(), groups, again, 4)
    assert got2 == got
    assert again.result['remap'].tobytes() == res['remap'].tobytes()


def test_pileup_mt_equals_serial_pileup():
    """Counters, read counts, first units, max positions and the event list
    (in order) of og_pileup_mt equal og_pileup's."""
    seed_set = projects.load_default().seed_sequences()
    pol = seed_set['HIV1B-pol-seed']
    pairs = synth.make_pairs(2000, genomes={'HIV1B-pol-seed': pol}, genome_seed=8, read_seed=9,
                             indel_rate=0.02)
    _, seqs, quals = synth.interleave(pairs)
    prep = cpu_pipeline.Prepared(seqs, quals, True)
    cpu_pipeline._declare_fast(oracle.lib())
    recs = cpu_pipeline._map_fast(prep, oracle.Index([pol], 20), oracle.LOCAL, 4, prep.alns)
    one = cpu_pipeline._pileup_fast(prep, prep.alns, recs, 1, [len(pol)], 1)
    many = cpu_pipeline._pileup_fast(prep, prep.alns, recs, 1, [len(pol)], 7)
    for k in range(4):
        assert np.array_equal(np.asarray(one[k]), np.asarray(many[k])), k
    assert one[5] == many[5] and one[5] > 0
    ev = lambda p: [(e.ref, e.pos, p[6][e.tok_off:e.tok_off + e.tok_len]) for e in p[4][:p[5]]]  # noqa: E731
    assert ev(one) == ev(many)
