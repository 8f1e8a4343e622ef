"""
oracle/cpu_pipeline.py -- TEST INFRASTRUCTURE ONLY (bench.py's cpu_baseline
leg and tests).

The same step as bench.py's GPU step -- prelim pass (end-to-end over every
seed), seed selection, prelim consensus, one --local remap pass over the
consensus, pileup and consensus again -- run by the CPU oracle: the C
restatement (og_map with OpenMP over read pairs, og_pileup) plus the Python
consensus code of oracle.py.
"""
import ctypes
import time
from collections import Counter

import numpy as np

import oracle


def _rows_from_alns(alns, seqs, quals, n_reads):
    """OgRow per read in SAM orientation (what temp.sam would hold)."""
    comp = str.maketrans('ACGTN', 'TGCAN')
    rows, keep = [], []
    for i in range(n_reads):
        a = alns[i]
        s = oracle.decode_seq(seqs[i])
        q = quals[i]
        if a.ref >= 0 and a.rev:
            s = s.translate(comp)[::-1]
            q = q[::-1]
        sb, qb = s.encode(), q.encode()
        n = a.n_cigar if a.ref >= 0 and not (a.flag & 4) else 0
        arr = (ctypes.c_uint32 * max(n, 1))(*a.cigar[:n])
        keep.append((sb, qb, arr))
        rows.append(oracle.OgRow(a.flag, a.sam_ref, a.sam_pos, n, arr, len(sb), sb, qb))
    return rows, keep


def _pileup(alns, seqs, quals, n_refs, ref_lens, paired, q=20):
    n = len(seqs)
    rows, keep = _rows_from_alns(alns, seqs, quals, n)
    units = []
    if paired:
        for u in range(n // 2):
            a, b = 2 * u, 2 * u + 1
            pa, pb = alns[a].sam_ref >= 0, alns[b].sam_ref >= 0
            if pa and pb:
                units += [a, b]
    else:
        for u in range(n):
            if alns[u].sam_ref >= 0:
                units += [u, -1]
    cap = max(ref_lens) + 2048
    row_arr = (oracle.OgRow * max(n, 1))(*rows)
    unit_arr = (ctypes.c_int64 * max(len(units), 1))(*units)
    dense = (ctypes.c_int32 * (n_refs * cap * 6))()
    rc = (ctypes.c_int64 * n_refs)()
    fu = (ctypes.c_int64 * n_refs)(*([-1] * n_refs))
    mp = (ctypes.c_int32 * n_refs)()
    ev_cap = n * 256 + 16
    ev = (oracle.OgEvent * ev_cap)()
    pool = ctypes.create_string_buffer(ev_cap * 4)
    ne, used = ctypes.c_int64(), ctypes.c_int64()
    st = oracle.lib().og_pileup(n_refs, cap, row_arr, len(units) // 2, unit_arr, q, dense, rc, fu, mp,
                                ev, ev_cap, ctypes.byref(ne), pool, len(pool), ctypes.byref(used))
    if st:
        raise RuntimeError('og_pileup status %d' % st)
    return dense, rc, fu, mp, ev, ne.value, pool.raw, cap


def _conseqs(names, seeds, pile, order):
    dense, rc, fu, mp, ev, ne, pool, cap = pile
    events = {}
    for e in ev[:ne]:
        events.setdefault((e.ref, e.pos), Counter())[pool[e.tok_off:e.tok_off + e.tok_len].decode()] += 1
    refmap = {}
    for r in order:
        pos_nucs = {}
        for pos in range(1, mp[r] + 1):
            base = (r * cap + pos - 1) * 6
            c = Counter()
            for k, tok in enumerate('ACGT'):
                if dense[base + k]:
                    c[tok] = dense[base + k]
            if dense[base + 4]:
                c['N'] = -1
            if dense[base + 5]:
                c['-'] = -2
            c.update(events.get((r, pos), {}))
            if c:
                pos_nucs[pos] = c
        refmap[names[r]] = (pos_nucs, mp[r])
    return oracle.counts_to_conseqs(refmap, seeds)[0]


def run_step(seed_set, all_seeds, seed_groups, seqs, quals, paired=True, nthreads=0,
             count_threshold=10):
    """prelim + one remap iteration on the CPU oracle; returns (conseqs, seconds)."""
    t0 = time.perf_counter()
    names = list(seed_set)
    ix = oracle.Index([seed_set[n] for n in names], 22)
    alns = oracle.map_reads(ix, oracle.params(oracle.E2E), seqs, quals, paired, nthreads)
    n = len(seqs)
    lines, filt, first = Counter(), Counter(), {}
    for i in range(n):
        a = alns[i]
        if a.sam_ref < 0:
            continue
        name = names[a.sam_ref]
        lines[name] += 1
        first.setdefault(name, i)
        if not (a.flag & 4):
            mx = max([c >> 4 for c in a.cigar[:a.n_cigar] if (c & 15) == 0] or [0])
            if mx > 50:
                filt[name] += 1
    refgroups = {}
    for name in sorted(first, key=first.get):
        thr = 1 if name == 'HIV1B-env-seed' else count_threshold
        _b, best = refgroups.get(seed_groups[name], (None, thr - 1))
        if filt[name] > best:
            refgroups[seed_groups[name]] = (name, filt[name])
    seed_counts = {r: c for r, c in refgroups.values()}
    pile = _pileup(alns, seqs, quals, len(names), [len(seed_set[k]) for k in names], paired)
    order = sorted((r for r in range(len(names)) if pile[2][r] >= 0), key=lambda r: first[names[r]])
    conseqs = {k: v for k, v in _conseqs(names, all_seeds, pile, order).items() if k in seed_counts}
    if conseqs:
        cn = list(conseqs)
        ix2 = oracle.Index([conseqs[k] for k in cn], 20)
        alns2 = oracle.map_reads(ix2, oracle.params(oracle.LOCAL), seqs, quals, paired, nthreads)
        pile2 = _pileup(alns2, seqs, quals, len(cn), [len(conseqs[k]) for k in cn], paired)
        order2 = sorted((r for r in range(len(cn)) if pile2[2][r] >= 0), key=lambda r: pile2[2][r])
        conseqs = _conseqs(cn, all_seeds, pile2, order2)
    return conseqs, time.perf_counter() - t0


# ---------------------------------------------------------------------------
# bench.py's cpu_baseline: the same step with every per-read loop in C
# (OpenMP over read pairs on all the cores given) and the inputs marshalled
# before the clock starts.
# ---------------------------------------------------------------------------
class Prepared:
    """Reads packed once into the buffers og_map / og_rows_from_alns take.
    Each mapping pass of timed_step has its own record buffer (alns: the
    prelim pass, alns2: the remap pass), so both stay readable afterwards
    (bench.py's parity leg compares them with the device's records)."""

    def __init__(self, seqs, quals, paired):
        self.n = len(seqs)
        self.paired = paired
        self.offs = (ctypes.c_int64 * max(self.n, 1))()
        self.lens = (ctypes.c_int32 * max(self.n, 1))()
        pos = 0
        for i, s in enumerate(seqs):
            self.offs[i] = pos
            self.lens[i] = len(s)
            pos += len(s)
        self.sbuf = ''.join(seqs).encode()
        self.qbuf = ''.join(quals).encode()
        self._buffers(pos)

    @classmethod
    def from_arrays(cls, reads, quals, paired):
        """(n, L) uint8 read / quality arrays (mates interleaved when
        paired), without a per-read Python loop."""
        self = cls.__new__(cls)
        n, L = reads.shape
        self.n, self.paired = n, paired
        self.offs = (ctypes.c_int64 * max(n, 1)).from_buffer_copy(
            (np.arange(max(n, 1), dtype=np.int64) * L).tobytes())
        self.lens = (ctypes.c_int32 * max(n, 1)).from_buffer_copy(
            np.full(max(n, 1), L, dtype=np.int32).tobytes())
        self.sbuf = np.ascontiguousarray(reads).tobytes()
        self.qbuf = np.ascontiguousarray(quals).tobytes()
        self._buffers(n * L)
        return self

    def _buffers(self, total):
        self.seq_out = ctypes.create_string_buffer(max(total, 1))
        self.qual_out = ctypes.create_string_buffer(max(total, 1))
        self.rows = (oracle.OgRow * max(self.n, 1))()
        self.alns = (oracle.OgAln * max(self.n, 1))()
        self.alns2 = (oracle.OgAln * max(self.n, 1))()
        self.result = None


def _declare_fast(L):
    if getattr(L, '_fast_declared', False):
        return
    L.og_rows_from_alns.argtypes = [ctypes.POINTER(oracle.OgAln), ctypes.c_int64, ctypes.c_char_p,
                                    ctypes.c_char_p, ctypes.POINTER(ctypes.c_int64),
                                    ctypes.POINTER(ctypes.c_int32), ctypes.c_char_p,
                                    ctypes.c_char_p, ctypes.POINTER(oracle.OgRow), ctypes.c_int]
    L.og_pileup_mt.argtypes = list(L.og_pileup.argtypes) + [ctypes.c_int]
    L._fast_declared = True


def _map_fast(prep, ix, mode, nthreads, out):
    st = oracle.lib().og_map(ix.handle, ctypes.byref(oracle.params(mode)), prep.n, int(prep.paired),
                             prep.sbuf, prep.qbuf, prep.offs, prep.lens, out, nthreads)
    if st:
        raise RuntimeError('og_map status %d' % st)
    return np.frombuffer(out, dtype=_ALN_DTYPE, count=prep.n)


def map_arrays(refseqs, mode, reads, quals, paired, nthreads=0):
    """og_map of (n, L) read / quality arrays against refseqs: the records
    as a numpy array of _ALN_DTYPE (the device's ALN_DTYPE layout)."""
    prep = Prepared.from_arrays(reads, quals, paired)
    ix = oracle.Index(list(refseqs), oracle.seed_len(mode))
    return _map_fast(prep, ix, mode, nthreads, prep.alns).copy()


def _pileup_fast(prep, alns, recs, n_refs, ref_lens, nthreads, q=20):
    L = oracle.lib()
    L.og_rows_from_alns(alns, prep.n, prep.sbuf, prep.qbuf, prep.offs, prep.lens,
                        prep.seq_out, prep.qual_out, prep.rows, nthreads)
    sam_ref = recs['sam_ref']
    if prep.paired:
        both = (sam_ref[0::2] >= 0) & (sam_ref[1::2] >= 0)
        first = 2 * np.flatnonzero(both)
        units = np.stack([first, first + 1], axis=1).reshape(-1).astype(np.int64)
    else:
        one = np.flatnonzero(sam_ref >= 0)
        units = np.stack([one, np.full_like(one, -1)], axis=1).reshape(-1).astype(np.int64)
    n_units = len(units) // 2
    cap = max(ref_lens) + 2048
    dense = np.zeros(n_refs * cap * 6, dtype=np.int32)
    rc = np.zeros(n_refs, dtype=np.int64)
    fu = np.full(n_refs, -1, dtype=np.int64)
    mp = np.zeros(n_refs, dtype=np.int32)
    ev_cap = prep.n * 256 + 16
    ev = (oracle.OgEvent * ev_cap)()
    pool = ctypes.create_string_buffer(ev_cap * 4)
    ne, used = ctypes.c_int64(), ctypes.c_int64()
    p = lambda a, t: a.ctypes.data_as(ctypes.POINTER(t))  # noqa: E731
    st = L.og_pileup_mt(n_refs, cap, prep.rows, n_units,
                        p(units, ctypes.c_int64) if n_units else None, q,
                        p(dense, ctypes.c_int32), p(rc, ctypes.c_int64), p(fu, ctypes.c_int64),
                        p(mp, ctypes.c_int32), ev, ev_cap, ctypes.byref(ne), pool, len(pool),
                        ctypes.byref(used), nthreads)
    if st:
        raise RuntimeError('og_pileup_mt status %d' % st)
    return dense, rc, fu, mp, ev, ne.value, pool.raw, cap


def _position_sums(pile, r, length):
    """sum(counts[pos].values()) for pos 1..length of reference r of an
    og_pileup result (remap.py:236-237): the base counts, -1 where an N was
    seen, -2 where a deletion was, and every insertion token's count; the
    seed prefill adds 0."""
    dense, _rc, _fu, _mp, ev, ne, _pool, cap = pile
    d = np.asarray(dense).reshape(-1, cap, 6)[r, :length].astype(np.int64)
    s = d[:, 0] + d[:, 1] + d[:, 2] + d[:, 3] - (d[:, 4] != 0) - 2 * (d[:, 5] != 0)
    if ne:
        e = np.frombuffer(ev, dtype=np.int32, count=4 * ne).reshape(ne, 4)
        pos = e[(e[:, 0] == r) & (e[:, 1] >= 1) & (e[:, 1] <= length), 1]
        np.add.at(s, pos - 1, 1)
    return s


def distance_filter(names, all_seeds, pile, order, new_conseqs, filter_coverage, nthreads,
                    distance_report=None):
    """The consensus-distance filter of remap.sam_to_conseqs (remap.py:228-268,
    extract_relevant_seed :129-138) on the oracle's pileup: for every
    consensus (name order), its positions whose counts sum to at least
    filter_coverage; og_gotoh_align of each seed (name order) against them,
    global, gop 15 / gep 3, HYPHY_NUC (remap.py:33, :248); the seed's part
    under the consensus; og_levenshtein (C, so 30 kb strings take seconds).
    A consensus stays when its own seed is no farther than the nearest other;
    if none stays, the reference with the most merged pairs (ties: first
    counted) does.  The K x K alignments run on nthreads host threads
    (ctypes releases the GIL)."""
    from concurrent.futures import ThreadPoolExecutor
    from cpu_e2e import HYPHY_NUC
    if len(new_conseqs) < 2:
        return new_conseqs
    matrix, alphabet = HYPHY_NUC
    index = {names[r]: r for r in order}
    conseq_names = sorted(new_conseqs)
    relevant = {}
    for name in conseq_names:
        conseq = new_conseqs[name]
        keep = _position_sums(pile, index[name], len(conseq)) >= filter_coverage
        rel = ''.join(c for c, k in zip(conseq, keep) if k)
        if rel:
            relevant[name] = rel
    jobs = [(name, seed_name) for name in conseq_names if name in relevant for seed_name in conseq_names]

    def one(job):
        name, seed_name = job
        a_seed, a_conseq, _ = oracle.gotoh_align(oracle.clean_sequence(all_seeds[seed_name], alphabet),
                                                 oracle.clean_sequence(relevant[name], alphabet),
                                                 15, 3, True, alphabet, matrix)
        return oracle.levenshtein(oracle.extract_relevant_seed(a_conseq, a_seed), relevant[name])

    # longest alignments first, so the pool ends together
    by_size = sorted(range(len(jobs)), key=lambda j: -len(all_seeds[jobs[j][1]]) * len(relevant[jobs[j][0]]))
    dists = [None] * len(jobs)
    with ThreadPoolExecutor(max(1, nthreads)) as pool:
        for j, d in zip(by_size, pool.map(lambda j: one(jobs[j]), by_size)):
            dists[j] = d
    filtered = {}
    for name in conseq_names:
        if name not in relevant:
            continue
        seed_dist = other_dist = other_seed = None
        for (n2, seed_name), d in zip(jobs, dists):
            if n2 != name:
                continue
            if seed_name == name:
                seed_dist = d
            elif other_dist is None or d < other_dist:
                other_seed, other_dist = seed_name, d
        if seed_dist <= other_dist:
            filtered[name] = new_conseqs[name]
        if distance_report is not None:
            distance_report[name] = dict(seed_dist=seed_dist, other_dist=other_dist, other_seed=other_seed)
    if not filtered:
        rc = pile[1]
        counts = Counter()
        for r in order:
            counts[names[r]] = int(rc[r])
        best_ref = counts.most_common(1)[0][0]
        filtered[best_ref] = new_conseqs[best_ref]
    return filtered


def converged(old_names, new_names, new_counts, map_counts, raw_count, n_remaps):
    """remap.py:591-603: with the consensus names unchanged, stop when no
    reference gained mapped lines, or more than 95 % of raw_count mapped, or
    after MAX_REMAPS passes."""
    from cpu_e2e import MAX_REMAPS, MIN_MAPPING_EFFICIENCY
    if new_names != old_names:
        return False
    if all(n <= map_counts[name] for name, n in new_counts.items()):
        return True
    if sum(new_counts.values()) / float(raw_count) > MIN_MAPPING_EFFICIENCY:
        return True
    return n_remaps >= MAX_REMAPS


def timed_step(seed_set, all_seeds, seed_groups, prep, nthreads, count_threshold=10,
               max_iterations=1, min_iterations=None):
    """run_step on prepared reads: prelim e2e pass over every seed, seed
    selection, prelim consensus, then remap()'s loop (remap.py:544-606):
    --local pass against the consensus set, pileup, consensus, the
    consensus-distance filter (filter_coverage = count_threshold / 2,
    remap.py:576-581), stopping rules -- capped at max_iterations passes,
    and with the rules held off for min_iterations (bench configs only, as
    RemapPipeline.iterate).  raw_count = 2 x units (remap.py:457).
    Returns (conseqs, seconds); only this function's body is timed."""
    _declare_fast(oracle.lib())
    t0 = time.perf_counter()
    names = list(seed_set)
    ix = oracle.Index([seed_set[k] for k in names], 22)
    recs = _map_fast(prep, ix, oracle.E2E, nthreads, prep.alns)
    sam_ref = recs['sam_ref']
    mapped = (recs['flag'] & 4) == 0
    longest_m = _longest_m(recs)
    lines = np.bincount(sam_ref[sam_ref >= 0], minlength=len(names))
    filt = np.bincount(sam_ref[(sam_ref >= 0) & mapped & (longest_m > 50)], minlength=len(names))
    first = {}
    for r in np.flatnonzero(lines):
        first[names[r]] = int(np.argmax(sam_ref == r))
    refgroups = {}
    for name in sorted(first, key=first.get):
        thr = 1 if name == 'HIV1B-env-seed' else count_threshold
        _b, best = refgroups.get(seed_groups[name], (None, thr - 1))
        f = int(filt[names.index(name)])
        if f > best:
            refgroups[seed_groups[name]] = (name, f)
    seed_counts = {r: c for r, c in refgroups.values()}
    pile = _pileup_fast(prep, prep.alns, recs, len(names), [len(seed_set[k]) for k in names], nthreads)
    order = sorted((r for r in range(len(names)) if pile[2][r] >= 0), key=lambda r: first[names[r]])
    conseqs = {k: v for k, v in _conseqs(names, all_seeds, pile, order).items() if k in seed_counts}
    map_counts = {k: seed_counts[k] for k in conseqs}
    prelim_conseqs, cn, recs2 = dict(conseqs), [], None
    raw_count = 2.0 * (prep.n // 2 if prep.paired else prep.n)
    passes = []
    n_remaps = 0
    while conseqs:
        mapped_to = conseqs
        cn = list(conseqs)
        ix2 = oracle.Index([conseqs[k] for k in cn], 20)
        recs2 = _map_fast(prep, ix2, oracle.LOCAL, nthreads, prep.alns2)
        r2 = recs2['sam_ref']
        ok = (r2 >= 0) & ((recs2['flag'] & 4) == 0)
        per_ref = np.bincount(r2[ok], minlength=len(cn))
        firstm = {r: int(np.argmax(ok & (r2 == r))) for r in np.flatnonzero(per_ref)}
        new_counts = Counter()
        for r in sorted(firstm, key=firstm.get):
            new_counts[cn[r]] = int(per_ref[r])
        pile2 = _pileup_fast(prep, prep.alns2, recs2, len(cn), [len(conseqs[k]) for k in cn], nthreads)
        order2 = sorted((r for r in range(len(cn)) if pile2[2][r] >= 0), key=lambda r: pile2[2][r])
        new = _conseqs(cn, all_seeds, pile2, order2)
        conseqs = distance_filter(cn, all_seeds, pile2, order2, new, count_threshold / 2, nthreads)
        n_remaps += 1
        passes.append(dict(names=cn, new_counts=dict(new_counts), unfiltered=sorted(new),
                           kept=sorted(conseqs)))
        if max_iterations is not None and n_remaps >= max_iterations:
            break
        forced = min_iterations is not None and n_remaps < min_iterations
        if not forced and converged(set(mapped_to), set(conseqs), new_counts, map_counts, raw_count,
                                    n_remaps):
            break
        map_counts = dict(new_counts)
    secs = time.perf_counter() - t0
    prep.result = dict(prelim=recs, prelim_names=names, prelim_conseqs=prelim_conseqs,
                       remap=recs2, remap_names=cn, conseqs=conseqs, passes=passes)
    return conseqs, secs


_ALN_DTYPE = np.dtype([(name, np.int32) for name, _ in oracle.OgAln._fields_[:-1]] +
                      [('cigar', np.uint32, (oracle.MAXOPS,))])


def _longest_m(recs):
    ops = recs['cigar']
    n = recs['n_cigar'][:, None]
    is_m = ((ops & 15) == 0) & (np.arange(ops.shape[1])[None, :] < n)
    return np.where(is_m, ops >> 4, 0).max(axis=1)
