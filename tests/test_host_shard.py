"""Host logic on the CPU: the consensus half of the pipeline (consensus.py)
and the multi-GPU shard reduction (pipeline.Shard / RemapPipeline._counts)
over torch.distributed with the gloo backend at world_size 2.

The per-rank inputs are oracle pileups / oracle alignments of each rank's
contiguous block of read pairs; the reduced result must equal the oracle on
the whole set -- the same property the RCCL path relies on (sum of dense
counters, max of flags and max_pos, min of first unit / first row, gathered
insertion events)."""
import ctypes
import os
import socket
from collections import Counter

import numpy as np
import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

import cpu_pipeline
import oracle
from micall_amd import projects, synth
from micall_amd.consensus import Pileup, counts_to_conseqs
from micall_amd.pipeline import RemapPipeline, Shard

REFS = ['HIV1B-gag-seed', 'HIV1B-pol-seed']
N_PAIRS = 300


def _data():
    cfg = projects.load_default()
    seeds = cfg.seed_sequences()
    genomes = {k: seeds[k] for k in REFS}
    d = synth.make_pairs(N_PAIRS, genomes, genome_seed=11, read_seed=12, read_len=251,
                         indel_rate=0.01)
    reads = np.stack([d['r1'], d['r2']], axis=1).reshape(2 * N_PAIRS, 251)
    quals = np.stack([d['q1'], d['q2']], axis=1).reshape(2 * N_PAIRS, 251)
    seqs = [r.tobytes().decode() for r in reads]
    qs = [q.tobytes().decode() for q in quals]
    ix = oracle.Index([seeds[k] for k in REFS], 20)
    alns = oracle.map_reads(ix, oracle.params(oracle.LOCAL), seqs, qs, True, 4)
    return cfg, seeds, seqs, qs, alns


def _fetched(alns, seqs, quals, ref_lens, pair_lo, pair_hi):
    """Oracle pileup of pairs [pair_lo, pair_hi) in Context.pileup_fetch's
    layout, first_unit relative to pair_lo (as a rank would report it)."""
    lo, hi = 2 * pair_lo, 2 * pair_hi
    rows, keep = cpu_pipeline._rows_from_alns(alns[lo:hi], seqs[lo:hi], quals[lo:hi], hi - lo)
    units = []
    for u in range((hi - lo) // 2):
        if alns[lo + 2 * u].sam_ref >= 0 and alns[lo + 2 * u + 1].sam_ref >= 0:
            units += [2 * u, 2 * u + 1]
    n_refs = len(ref_lens)
    cap = max(ref_lens) + 2048
    row_arr = (oracle.OgRow * max(len(rows), 1))(*rows)
    unit_arr = (ctypes.c_int64 * max(len(units), 1))(*units)
    dense = (ctypes.c_int32 * (n_refs * cap * 6))()
    rc = (ctypes.c_int64 * n_refs)()
    fu = (ctypes.c_int64 * n_refs)(*([-1] * n_refs))
    mpos = (ctypes.c_int32 * n_refs)()
    ev_cap = (hi - lo) * 256 + 16
    ev = (oracle.OgEvent * ev_cap)()
    pool = ctypes.create_string_buffer(ev_cap * 4)
    ne, used = ctypes.c_int64(), ctypes.c_int64()
    assert oracle.lib().og_pileup(n_refs, cap, row_arr, len(units) // 2, unit_arr, 20, dense, rc,
                                  fu, mpos, ev, ev_cap, ctypes.byref(ne), pool, len(pool),
                                  ctypes.byref(used)) == 0
    d6 = np.frombuffer(dense, dtype=np.int32).reshape(n_refs, cap, 6)
    raw = pool.raw
    return dict(dense=d6[:, :, :4].copy(), nflag=(d6[:, :, 4] != 0).astype(np.uint8),
                dflag=(d6[:, :, 5] != 0).astype(np.uint8),
                read_counts=np.frombuffer(rc, dtype=np.int64).copy(),
                first_unit=np.frombuffer(fu, dtype=np.int64).copy(),
                max_pos=np.frombuffer(mpos, dtype=np.int32).copy(),
                events=[k + (n,) for k, n in sorted(Counter(
                    (e.ref, e.pos, raw[e.tok_off:e.tok_off + e.tok_len].decode())
                    for e in ev[:ne.value]).items())], cap=cap)


def _map_counts(alns, lo, hi):
    """What mh_map_counts reports for reads [lo, hi) (row indices relative)."""
    k = len(REFS)
    c = dict(lines=np.zeros(k, np.int64), filtered=np.zeros(k, np.int64),
             mapped=np.zeros(k, np.int64), first_row=np.full(k, -1, np.int64),
             first_mapped=np.full(k, -1, np.int64), unmapped=0, star=0, star_first=-1)
    for i in range(lo, hi):
        a, row = alns[i], i - lo
        if a.flag & 4:
            c['unmapped'] += 1
        if a.sam_ref < 0:
            c['star'] += 1
            if c['star_first'] < 0:
                c['star_first'] = row
            continue
        r = a.sam_ref
        c['lines'][r] += 1
        if c['first_row'][r] < 0:
            c['first_row'][r] = row
        if not a.flag & 4:
            c['mapped'][r] += 1
            if c['first_mapped'][r] < 0:
                c['first_mapped'][r] = row
            runs = [op >> 4 for op in a.cigar[:a.n_cigar] if op & 15 == 0]
            if max(runs + [0]) > 50:
                c['filtered'][r] += 1
    return c


def test_host_consensus_matches_oracle():
    """consensus.counts_to_conseqs on fetched counters == the oracle's
    counts_to_conseqs on the same refmap (remap.py:309-333)."""
    cfg, seeds, seqs, qs, alns = _data()
    all_seeds = cfg.all_region_sequences()
    lens = [len(seeds[k]) for k in REFS]
    f = _fetched(alns, seqs, qs, lens, 0, N_PAIRS)
    pile = Pileup(f, REFS)
    order = pile.refs_with_reads()
    assert len(order) == 2
    got = counts_to_conseqs(pile, order, seeds=all_seeds)
    want = cpu_pipeline._conseqs(REFS, all_seeds, cpu_pipeline._pileup(alns, seqs, qs, 2, lens,
                                                                         True), order)
    assert got == want and list(got) == list(want)


class _FakeCtx:
    """Stands in for the device context: returns a rank's oracle results."""

    def __init__(self, fetched, counts):
        self.fetched, self.counts = fetched, counts

    def pileup_fetch(self):
        return self.fetched

    def map_counts(self):
        return self.counts


def _worker(rank, world, port, out_dir):
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port))
    dist.init_process_group('gloo', rank=rank, world_size=world)
    try:
        cfg, seeds, seqs, qs, alns = _data()
        lens = [len(seeds[k]) for k in REFS]
        per = N_PAIRS // world
        lo, hi = rank * per, (rank + 1) * per
        shard = Shard(rank, world, read_base=2 * lo)
        ctx = _FakeCtx(_fetched(alns, seqs, qs, lens, lo, hi), _map_counts(alns, 2 * lo, 2 * hi))
        fetched = shard.pileup(ctx, unit_base=lo)
        pipe = RemapPipeline(ctx, config=cfg, shard=shard)
        counts = pipe._counts()
        if rank == 0:
            full = _fetched(alns, seqs, qs, lens, 0, N_PAIRS)
            for key in ('dense', 'nflag', 'dflag', 'read_counts', 'first_unit', 'max_pos'):
                np.testing.assert_array_equal(fetched[key], full[key], err_msg=key)
            merged = Counter()
            for r, pos, tok, n in fetched['events']:
                merged[r, pos, tok] += n
            assert merged == Counter({(r, pos, tok): n for r, pos, tok, n in full['events']})
            want = _map_counts(alns, 0, 2 * N_PAIRS)
            for key, v in want.items():
                np.testing.assert_array_equal(counts[key], v, err_msg=key)
            all_seeds = cfg.all_region_sequences()
            p1, p2 = Pileup(fetched, REFS), Pileup(full, REFS)
            assert (counts_to_conseqs(p1, p1.refs_with_reads(), all_seeds)
                    == counts_to_conseqs(p2, p2.refs_with_reads(), all_seeds))
            open(os.path.join(out_dir, 'ok'), 'w').close()
    finally:
        dist.destroy_process_group()


def _free_port():
    with socket.socket() as s:
        s.bind(('127.0.0.1', 0))
        return s.getsockname()[1]


@pytest.mark.timeout(300)
def test_shard_reduction_gloo_world2(tmp_path):
    mp.spawn(_worker, args=(2, _free_port(), str(tmp_path)), nprocs=2, join=True)
    assert (tmp_path / 'ok').exists()
