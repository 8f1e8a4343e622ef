"""
Device-resident prelim_map -> remap loop.

The reference runs bowtie2 on the FASTQ files once for prelim_map and once per
remap iteration, parsing SAM text in Python each time (prelim_map.py:114-151,
remap.py:474-606, :661-761).  Here the reads are ingested once into HBM and
every pass is a device call:

    prelim pass     mh_map(end-to-end) over every seed        (prelim_map.py:134)
    seed selection  per-rname line tallies (mh_map_counts)    (remap.py:482-528)
    prelim conseqs  mh_pileup + counts_to_conseqs (host)      (remap.py:531-541)
    remap loop      mh_map(--local) over the consensus set,   (remap.py:548-606)
                    mh_pileup, consensus-distance filter
                    (mh_gotoh_align), the three stopping rules

The control flow and every dict order mirror remap() so the consensus
sequences, counts and the final SAM records are the ones the reference would
compute from the same alignments.  With a `Shard`, each rank holds a
contiguous block of read pairs; per-reference tallies and the dense pileup
counters are all-reduced over RCCL between passes and every rank then takes
the same decisions.
"""
from collections import Counter

import numpy as np

from . import _native
from .consensus import Pileup, counts_to_conseqs, filter_conseqs
from .projects import ProjectConfig

CONSENSUS_Q_CUTOFF = 20       # remap.py:35
MIN_MAPPING_EFFICIENCY = 0.95  # remap.py:36
MAX_REMAPS = 3                # remap.py:37
READ_GAP_EXTEND = REF_GAP_EXTEND = 3   # prelim_map.py:27-30
MAXINS = 1200                 # -X 1200
E2E_SEEDLEN, LOCAL_SEEDLEN = 22, 20


def write_remap_counts(writer, counts, title, distance_report=None):
    """remap_counts.csv rows of one pass (remap.py:373-378): references in
    name order, each with its distance-filter columns when it has them."""
    extra = distance_report or {}
    for name in sorted(counts):
        row = dict(extra.get(name, {}), type='%s %s' % (title, name), count=counts[name])
        writer.writerow(row)


class Shard:
    """Multi-GPU view: this rank's first read index and the collectives used
    between passes (torch.distributed over RCCL; gloo works for tests)."""

    def __init__(self, rank, world, read_base, device=None):
        import torch
        import torch.distributed as dist
        self.torch, self.dist = torch, dist
        self.rank, self.world, self.read_base = rank, world, read_base
        self.device = device if device is not None else torch.device('cpu')

    def barrier(self):
        """Every rank has reached this point (e.g. opened its output files,
        so rank 0's writes cannot be truncated by a later open)."""
        self.sum_i64([0])

    def sum_i64(self, arr):
        t = self.torch.as_tensor(np.ascontiguousarray(arr, dtype=np.int64), device=self.device)
        self.dist.all_reduce(t, op=self.dist.ReduceOp.SUM)
        return t.cpu().numpy()

    def min_i64(self, arr):
        """min over ranks, -1 meaning 'none'."""
        a = np.where(np.asarray(arr) < 0, np.iinfo(np.int64).max, arr).astype(np.int64)
        t = self.torch.as_tensor(a, device=self.device)
        self.dist.all_reduce(t, op=self.dist.ReduceOp.MIN)
        out = t.cpu().numpy()
        return np.where(out == np.iinfo(np.int64).max, -1, out)

    def _gather(self, t):
        """all_gather of one equal-shaped tensor per rank, concatenated in rank
        order."""
        parts = [self.torch.empty_like(t) for _ in range(self.world)]
        self.dist.all_gather(parts, t)
        return self.torch.cat(parts)

    def _gather_sizes(self, values):
        t = self.torch.as_tensor(np.asarray(values, dtype=np.int64), device=self.device)
        return self._gather(t).cpu().numpy().reshape(self.world, len(values))

    def _text_device(self):
        # gloo moves point-to-point messages in host memory; RCCL needs them
        # on the device
        return self.torch.device('cpu') if self.dist.get_backend() == 'gloo' else self.device

    def all_gather_bytes(self, data):
        """Every rank's bytes (small texts such as a list of names), in
        rank order, on every rank."""
        torch = self.torch
        sizes = self._gather_sizes([len(data)])[:, 0]
        m = max(int(sizes.max()), 1)
        buf = np.zeros(m, dtype=np.uint8)
        buf[:len(data)] = np.frombuffer(bytes(data), dtype=np.uint8)
        dev = self._text_device()
        parts = [torch.empty(m, dtype=torch.uint8, device=dev) for _ in range(self.world)]
        self.dist.all_gather(parts, torch.as_tensor(buf, device=dev))
        return [parts[k].cpu().numpy()[:int(sizes[k])].tobytes() for k in range(self.world)]

    def gather_segments(self, segments):
        """Output text to rank 0: every rank passes the same number k of
        byte segments (e.g. its rows of each prelim.csv group, in the global
        group order); rank 0 receives [rank][segment] memoryviews, the other
        ranks None.  The lengths are all-gathered, then each rank's segments
        travel as one point-to-point message (device buffers under RCCL)."""
        torch = self.torch
        lens = np.array([len(x) for x in segments], dtype=np.int64)
        all_lens = self._gather_sizes(lens) if len(lens) else np.zeros((self.world, 0), np.int64)
        dev = self._text_device()

        def split(buf, ls):
            out, at = [], 0
            for n in ls.tolist():
                out.append(buf[at:at + n])
                at += n
            return out

        if self.rank != 0:
            total = int(lens.sum())
            if total:
                buf = np.empty(total, dtype=np.uint8)
                at = 0
                for x in segments:
                    buf[at:at + len(x)] = np.frombuffer(x, dtype=np.uint8)
                    at += len(x)
                self.dist.send(torch.from_numpy(buf).to(dev), dst=0)
            return None
        out = [[memoryview(x) for x in segments]]
        for r in range(1, self.world):
            total = int(all_lens[r].sum())
            if total:
                t = torch.empty(total, dtype=torch.uint8, device=dev)
                self.dist.recv(t, src=r)
                out.append(split(memoryview(t.cpu().numpy()), all_lens[r]))
            else:
                out.append([memoryview(b'')] * len(segments))
        return out

    def pileup(self, ctx, unit_base):
        """All-reduce the device counters in place and all-gather the
        insertion-token events.  Ranks first agree (MAX of a per-reference
        flag) on the references that hold data anywhere; only their rows
        travel: dense counts and read counts summed, N/deletion flags as bytes
        under MAX (an OR of 0/1), max_pos and the negated global first unit
        under MAX.  The events (4 int32 + token bytes each) are padded to the
        largest rank's size and all-gathered, then imported in rank order, so
        the token aggregation sees every rank's events.  No host objects are
        exchanged."""
        torch = self.torch
        dev = self.device
        if dev.type == 'cuda':
            _rc, fu, mp = ctx.pileup_scalars()
            has = torch.as_tensor(((fu >= 0) | (mp > 0)).astype(np.int32), device=dev)
            self.dist.all_reduce(has, op=self.dist.ReduceOp.MAX)
            sel = np.nonzero(has.cpu().numpy())[0].astype(np.int32)
            sum_b, max_b, flag_b = ctx.pileup_exchange_bytes(len(sel))
            s = torch.empty(sum_b // 4, dtype=torch.int32, device=dev)
            m = torch.empty(max_b // 4, dtype=torch.int32, device=dev)
            f = torch.empty(max(flag_b, 1), dtype=torch.uint8, device=dev)
            # the context's stream writes these buffers: torch's stream must be
            # done with their memory (allocator reuse) first
            torch.cuda.synchronize(dev)
            ctx.pileup_export(sel, unit_base, s.data_ptr(), m.data_ptr(), f.data_ptr())
            self.dist.all_reduce(s, op=self.dist.ReduceOp.SUM)
            self.dist.all_reduce(m, op=self.dist.ReduceOp.MAX)
            if flag_b:
                self.dist.all_reduce(f, op=self.dist.ReduceOp.MAX)
            torch.cuda.synchronize(dev)
            ctx.pileup_import(sel, s.data_ptr(), m.data_ptr(), f.data_ptr())
            sizes = self._gather_sizes(ctx.pileup_event_bytes())
            n_max, b_max = max(int(sizes[:, 0].max()), 1), max(int(sizes[:, 1].max()), 1)
            ev = torch.zeros(4 * n_max, dtype=torch.int32, device=dev)
            pool = torch.zeros(b_max, dtype=torch.uint8, device=dev)
            torch.cuda.synchronize(dev)   # the zero fills run on torch's stream
            ctx.pileup_events_export(ev.data_ptr(), pool.data_ptr())
            ev_all, pool_all = self._gather(ev), self._gather(pool)
            torch.cuda.synchronize(dev)
            ctx.pileup_events_import(sizes[:, 0], sizes[:, 1], ev_all.data_ptr(), 4 * n_max,
                                     pool_all.data_ptr(), b_max)
            return ctx.pileup_fetch(events=False)
        # CPU collective (tests): the same exchange over host copies
        fetched = reduce_fetched_host(self, ctx.pileup_fetch(), unit_base)
        fetched['events'] = self._gather_events(fetched['events'])
        fetched.pop('ev_raw', None)   # this rank's events only: Pileup packs the gathered ones
        return fetched

    def _gather_events(self, events):
        """(ref, pos, token, count) tuples of every rank, rank order, through
        fixed-size tensors: 4 int64 per event (ref, pos, count, token length)
        and the token bytes."""
        torch = self.torch
        meta = np.array([(r, p, n, len(t)) for r, p, t, n in events], dtype=np.int64).reshape(-1, 4)
        blob = np.frombuffer(''.join(t for _r, _p, t, _n in events).encode(), dtype=np.uint8)
        sizes = self._gather_sizes([len(meta), len(blob)])
        n_max, b_max = max(int(sizes[:, 0].max()), 1), max(int(sizes[:, 1].max()), 1)
        m = np.zeros((n_max, 4), dtype=np.int64)
        m[:len(meta)] = meta
        b = np.zeros(b_max, dtype=np.uint8)
        b[:len(blob)] = blob
        m_all = self._gather(torch.as_tensor(m, device=self.device)).cpu().numpy()
        b_all = self._gather(torch.as_tensor(b, device=self.device)).cpu().numpy()
        out = []
        for k in range(self.world):
            rows = m_all[k * n_max:k * n_max + int(sizes[k, 0])]
            text = b_all[k * b_max:k * b_max + int(sizes[k, 1])].tobytes().decode()
            at = 0
            for r, p, n, ln in rows.tolist():
                out.append((r, p, text[at:at + ln], n))
                at += ln
        return out


def reduce_fetched_host(shard, f, unit_base):
    """Host-side equivalent of the device export/all-reduce/import."""
    torch, dist = shard.torch, shard.dist
    out = dict(f)
    for key, op in (('dense', 'SUM'), ('read_counts', 'SUM'), ('max_pos', 'MAX')):
        t = torch.as_tensor(np.ascontiguousarray(f[key]).astype(np.int64))
        dist.all_reduce(t, op=getattr(dist.ReduceOp, op))
        out[key] = t.numpy().astype(f[key].dtype)
    for key in ('nflag', 'dflag'):
        t = torch.as_tensor(np.ascontiguousarray(f[key]).astype(np.int64))
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        out[key] = t.numpy().astype(np.uint8)
    fu = np.where(f['first_unit'] < 0, np.iinfo(np.int64).max, f['first_unit'] + unit_base)
    t = torch.as_tensor(fu.astype(np.int64))
    dist.all_reduce(t, op=dist.ReduceOp.MIN)
    fu = t.numpy()
    out['first_unit'] = np.where(fu == np.iinfo(np.int64).max, -1, fu)
    return out


class RemapPipeline:
    def __init__(self, ctx, config=None, count_threshold=10, rdgopen=10, rfgopen=10,
                 shard=None, callback=None):
        self.ctx = ctx
        self.config = config or ProjectConfig.loadDefault()
        self.seeds = self.config.all_region_sequences()      # remap.py:450-454
        self.seed_set = self.config.seed_sequences()         # prelim_map.py:102-106
        self.count_threshold = count_threshold
        self.rdgopen, self.rfgopen = rdgopen, rfgopen
        self.shard = shard
        self.callback = callback
        self.raw_count = None
        self.log = []
        self.first_mapped_to = None
        self.pass_refs = []

    # ---- plumbing --------------------------------------------------------
    def _params(self, mode):
        return _native.params(mode, rdg=(self.rdgopen, READ_GAP_EXTEND),
                              rfg=(self.rfgopen, REF_GAP_EXTEND), maxins=MAXINS)

    def _counts(self):
        c = self.ctx.map_counts()
        if self.shard is not None:
            sh = self.shard
            for key in ('lines', 'filtered', 'mapped'):
                c[key] = sh.sum_i64(c[key])
            for key in ('first_row', 'first_mapped'):
                c[key] = sh.min_i64(np.where(c[key] >= 0, c[key] + sh.read_base, -1))
            sf = c['star_first']
            c['star_first'] = int(sh.min_i64([sf + sh.read_base if sf >= 0 else -1])[0])
            c['unmapped'], c['star'] = (int(x) for x in sh.sum_i64([c['unmapped'], c['star']]))
        return c

    def _pileup(self, ref_lens, only=None):
        """Pileup of the last pass; `only` (reference indices): just these
        are counted (mh_pileup_only) and their counter rows fetched."""
        self.ctx.pileup(0, CONSENSUS_Q_CUTOFF, ref_lens, only=only)
        if self.shard is not None:
            unit_base = self.shard.read_base // 2 if self.ctx.reads_count()[1] else self.shard.read_base
            return self.shard.pileup(self.ctx, unit_base)
        return self.ctx.pileup_fetch(only=only, events=False)

    # ---- prelim_map ------------------------------------------------------
    def prelim(self):
        """End-to-end pass over every seed (prelim_map.py:96-140)."""
        names = list(self.seed_set)
        self.ctx.index_build(names, [self.seed_set[n] for n in names], E2E_SEEDLEN)
        self.ctx.map(self._params(_native.E2E))
        self.prelim_names = names
        self.prelim_stats = self._counts()
        return self.prelim_stats

    def prelim_groups(self):
        """(rname, count, filtered_count) per rname group of prelim.csv, in
        file order ('*' included) -- remap.py:485-515."""
        st = self.prelim_stats
        groups = [(int(st['first_row'][r]), self.prelim_names[r], int(st['lines'][r]),
                   int(st['filtered'][r])) for r in range(len(self.prelim_names))
                  if st['lines'][r] > 0]
        if st['star']:
            groups.append((int(st['star_first']), '*', int(st['star']), 0))
        groups.sort()
        return [(name, count, filt) for _, name, count, filt in groups]

    def select_seeds(self, groups):
        """Best rname per seed group above the count threshold
        (remap.py:517-528)."""
        refgroups = {}
        for refname, count, filtered in groups:
            if refname == '*':
                continue
            refgroup = self.config.getSeedGroup(refname)
            threshold = 1 if refname == 'HIV1B-env-seed' else self.count_threshold
            _best, best_count = refgroups.get(refgroup, (None, threshold - 1))
            if filtered > best_count:
                refgroups[refgroup] = (refname, filtered)
        return {best_ref: best_count for best_ref, best_count in refgroups.values()}

    def prelim_conseqs(self, seed_counts):
        """build_conseqs on the prelim alignments, then keep the seed-group
        winners (remap.py:531-541)."""
        names = self.prelim_names
        # only the seed-group winners' consensuses are kept: only their
        # counter rows are fetched and only theirs built, in refmap order
        # (the order of the kept ones is the same either way)
        winners = [r for r, n in enumerate(names) if n in seed_counts]
        fetched = self._pileup([len(self.seed_set[n]) for n in names], only=winners)
        pile = Pileup(fetched, names)
        rank = self.prelim_stats['first_row']
        order = [r for r in pile.refs_with_reads(rank=np.where(rank < 0, np.iinfo(np.int64).max, rank))
                 if names[r] in seed_counts]
        conseqs = counts_to_conseqs(pile, order, seeds=self.seeds)
        new_conseqs, map_counts = {}, {}
        for rname, conseq in conseqs.items():
            count = seed_counts.get(rname)
            if count is not None:
                map_counts[rname] = count
                new_conseqs[rname] = conseq
        return new_conseqs, map_counts

    # ---- remap loop ------------------------------------------------------
    def map_to_reference(self, refseqs):
        """One --local pass (remap.py:661-761): returns (new_counts,
        unmapped_count) with new_counts in first-mapped-line order."""
        names = list(refseqs)
        self.ctx.index_build(names, [refseqs[n] for n in names], LOCAL_SEEDLEN)
        self.ctx.map(self._params(_native.LOCAL))
        st = self._counts()
        new_counts = Counter()
        for r in sorted((r for r in range(len(names)) if st['mapped'][r] > 0),
                        key=lambda r: st['first_mapped'][r]):
            new_counts[names[r]] = int(st['mapped'][r])
        self.last_names = names
        self.last_refseqs = dict(refseqs)
        return new_counts, int(st['unmapped'])

    def build_conseqs_filtered(self, refseqs, distance_report=None):
        """build_conseqs(..., is_filtered=True, filter_coverage=threshold/2)
        on the last pass (remap.py:576-581)."""
        names = list(refseqs)
        fetched = self._pileup([len(refseqs[n]) for n in names])
        pile = Pileup(fetched, names)
        order = pile.refs_with_reads()
        new = counts_to_conseqs(pile, order, seeds=self.seeds)
        return filter_conseqs(self.ctx, pile, order, new, self.seeds, self.count_threshold / 2,
                              distance_report)

    def run(self, raw_count, max_iterations=None, remap_counts_writer=None, min_iterations=None):
        """prelim_map + remap on the resident reads: the device prelim pass,
        seed selection, then iterate()."""
        self.raw_count = raw_count
        self.prelim()
        groups = self.prelim_groups()
        if remap_counts_writer is not None:
            remap_counts_writer.writerows(dict(type='prelim %s' % name, count=count,
                                               filtered_count=filt)
                                          for name, count, filt in groups)
        conseqs, map_counts = self.prelim_conseqs(self.select_seeds(groups))
        return self.iterate(conseqs, map_counts, raw_count, max_iterations=max_iterations,
                            min_iterations=min_iterations, remap_counts_writer=remap_counts_writer)

    @staticmethod
    def converged(old_names, new_names, new_counts, map_counts, raw_count, n_remaps):
        """The stopping rules of remap.py:591-603.  They apply only while the
        set of consensus names is stable; then any one of them ends the loop:
        no reference mapped more lines than on the pass before, more than
        MIN_MAPPING_EFFICIENCY of raw_count mapped, or MAX_REMAPS passes."""
        if new_names != old_names:
            return False
        if all(n <= map_counts[name] for name, n in new_counts.items()):
            return True
        if sum(new_counts.values()) / float(raw_count) > MIN_MAPPING_EFFICIENCY:
            return True
        return n_remaps >= MAX_REMAPS

    def iterate(self, conseqs, map_counts, raw_count, max_iterations=None, min_iterations=None,
                remap_counts_writer=None, before_pass=None, after_pass=None):
        """remap()'s loop (remap.py:544-606) from the seed-group winners and
        their prelim counts: map with --local against the current consensus
        set, rebuild and filter the consensus, stop by converged().  Both the
        device pipeline (run) and the file-level drop-in (remap.remap) use
        this one loop.

        before_pass() / after_pass() hook the file outputs around each
        mapping pass (the unmapped FASTQs).  max_iterations caps the passes
        and min_iterations (BASELINE C3's "3 remap iterations") holds the
        stopping rules off; both are for benchmark configs only and are None
        for the reference's behaviour.
        Returns (consensus set after the last pass, its per-reference
        mapped-line counts, unmapped lines)."""
        self.raw_count = raw_count
        n_remaps = 0
        new_counts = Counter()
        unmapped_count = raw_count
        self.mapped_to = None
        self.first_mapped_to = dict(conseqs)   # the prelim consensus set the first pass maps to
        self.pass_refs = []                     # every pass's consensus set, in pass order
        while conseqs:
            if self.callback:
                self.callback(message='... remap iteration %d' % n_remaps, progress=0)
            if before_pass is not None:
                before_pass()
            self.mapped_to = mapped_to = conseqs
            self.pass_refs.append(dict(conseqs))
            new_counts, unmapped_count = self.map_to_reference(conseqs)
            if after_pass is not None:
                after_pass()
            distance_report = {}
            conseqs = self.build_conseqs_filtered(mapped_to, distance_report)
            n_remaps += 1
            self.log.append(dict(iteration=n_remaps, mapped=dict(new_counts),
                                 conseqs={k: len(v) for k, v in conseqs.items()}))
            if remap_counts_writer is not None:
                write_remap_counts(remap_counts_writer, new_counts, 'remap-{}'.format(n_remaps),
                                   distance_report)
            if max_iterations is not None and n_remaps >= max_iterations:
                break
            forced = min_iterations is not None and n_remaps < min_iterations
            if not forced and self.converged(set(mapped_to), set(conseqs), new_counts,
                                             map_counts, raw_count, n_remaps):
                break
            map_counts = dict(new_counts)
        self.conseqs = conseqs
        self.new_counts = new_counts
        self.unmapped_count = unmapped_count
        self.n_remaps = n_remaps
        return conseqs, new_counts, unmapped_count
