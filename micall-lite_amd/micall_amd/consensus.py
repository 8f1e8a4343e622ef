"""
Consensus from a device pileup: the host half of remap.sam_to_conseqs.

  counts_to_conseqs  micall/core/remap.py:309-333 (with the seed prefill of
                     :195-197: every seed position holds the seed base at
                     count 0)
  find_top_token     remap.py:892-902 (highest count, ties to the
                     lexicographically smallest token)
  filter_conseqs     remap.py:228-268 (consensus-distance filter: Gotoh
                     global alignment of every seed against the covered part
                     of each consensus, then edit distance)

The per-read work (merge_reads / update_counts) ran on the GPU
(mh_pileup); what arrives here is the dense A/C/G/T counters, the 'N' and
'-' flags and the few sparse insertion tokens, O(reference length).
"""
import re
from collections import Counter

import numpy as np

from . import _native

BASE_CODES = np.frombuffer(b'ACGT', dtype=np.uint8)
BASE_INDEX = np.full(256, 255, dtype=np.int64)   # 'A' 'C' 'G' 'T' -> 0..3, else 255
BASE_INDEX[BASE_CODES] = np.arange(4)
DASH = ord('-')

# micall/alignment/models/HYPHY_NUC.csv, the model of remap.py:33
HYPHY_NUC_ALPHABET = 'ACGT?'
HYPHY_NUC = [5, -4, -4, -4, 0,
             -4, 5, -4, -4, 0,
             -4, -4, 5, -4, 0,
             -4, -4, -4, 5, 0,
             0, 0, 0, 0, 0]
FILTER_GOP, FILTER_GEP = 15, 3   # remap.py:33 Aligner(gop=15, gep=3, is_global=True)


class Pileup:
    """Host view of one pileup (Context.pileup_fetch) over refs `refnames`."""

    def __init__(self, fetched, refnames):
        self.refnames = list(refnames)
        self.dense = fetched['dense']
        self.nflag = fetched['nflag']
        self.dflag = fetched['dflag']
        self.read_counts = fetched['read_counts']
        self.first_unit = fetched['first_unit']
        self.max_pos = fetched['max_pos']
        self.cap = fetched['cap']
        # insertion-token events as arrays (ref, pos, token offset / length in
        # a byte pool, merged pairs): the library's fetch hands them over this
        # way (ev_raw); a pileup built elsewhere gives (ref, pos, token,
        # count) tuples, packed here.  The per-reference lists and the
        # {ref: {pos: Counter}} view are built only when asked for.
        raw = fetched.get('ev_raw')
        if raw is None:
            evs = fetched.get('events') or []
            toks = [t for _r, _p, t, _n in evs]
            lens = np.array([len(t) for t in toks], dtype=np.int64)
            offs = np.zeros(len(toks), dtype=np.int64)
            if len(toks) > 1:
                offs[1:] = np.cumsum(lens)[:-1]
            raw = dict(ref=np.array([e[0] for e in evs], dtype=np.int64),
                       pos=np.array([e[1] for e in evs], dtype=np.int64), off=offs, len=lens,
                       count=np.array([e[3] for e in evs], dtype=np.int64),
                       pool=''.join(toks).encode('latin-1'))
        self._raw = raw
        self._ev_refs = set(np.unique(raw['ref']).tolist()) if len(raw['ref']) else set()
        self._ev_lists = None
        self._events = None

    def has_events(self, r):
        return r in self._ev_refs

    @property
    def _ev(self):
        """{ref: ([pos], [token], [count])} (the Python paths' view)."""
        if self._ev_lists is None:
            raw = self._raw
            pool = raw['pool']
            d = {}
            for r, pos, o, ln, k in zip(raw['ref'].tolist(), raw['pos'].tolist(), raw['off'].tolist(),
                                        raw['len'].tolist(), raw['count'].tolist()):
                g = d.get(r)
                if g is None:
                    g = d[r] = ([], [], [])
                g[0].append(pos)
                g[1].append(pool[o:o + ln].decode('latin-1'))
                g[2].append(k)
            self._ev_lists = d
        return self._ev_lists

    def ev_arrays(self, refs):
        """The events of references `refs` as arrays (ref, pos, offset,
        length, count) and the byte pool they index."""
        raw = self._raw
        if not len(raw['ref']):
            e = np.zeros(0, dtype=np.int64)
            return e, e, e, e, e, raw['pool']
        sel = np.isin(raw['ref'], np.asarray(list(refs), dtype=np.int64))
        return raw['ref'][sel], raw['pos'][sel], raw['off'][sel], raw['len'][sel], raw['count'][sel], raw['pool']

    @property
    def events(self):
        """{ref: {pos: Counter(token -> merged pairs)}}."""
        if self._events is None:
            self._events = {}
            for r, (ps, ts, cs) in self._ev.items():
                d = self._events[r] = {}
                for pos, tok, count in zip(ps, ts, cs):
                    d.setdefault(pos, Counter())[tok] += count
        return self._events

    def refs_with_reads(self, rank=None):
        """Reference indices that received a merged pair, in refmap order:
        by `rank` (e.g. first line of the rname group for the prelim SAM) or
        by the first merged unit (remap.py:192-194)."""
        present = [r for r in range(len(self.refnames)) if self.first_unit[r] >= 0]
        key = self.first_unit if rank is None else rank
        return sorted(present, key=lambda r: (key[r], r))

    def read_count_items(self, order):
        """read_counts Counter in insertion order (remap.py:186-191)."""
        c = Counter()
        for r in order:
            c[self.refnames[r]] = int(self.read_counts[r])
        return c

    def _slice(self, r, length):
        """dense, nflag, dflag for positions 1..length (zero past cap):
        views of the fetched rows when they reach that far."""
        if length <= self.cap:
            return self.dense[r, :length], self.nflag[r, :length] != 0, self.dflag[r, :length] != 0
        n = min(length, self.cap)
        d = np.zeros((length, 4), dtype=np.int64)
        nf = np.zeros(length, dtype=bool)
        df = np.zeros(length, dtype=bool)
        d[:n] = self.dense[r, :n]
        nf[:n] = self.nflag[r, :n] != 0
        df[:n] = self.dflag[r, :n] != 0
        return d, nf, df

    def counter_at(self, r, pos, seed, events=None):
        """The reference's pos_nucs[pos] Counter (for positions with events);
        `events`: that position's (token, count) pairs, if the caller has
        them (else they come from the events view)."""
        c = Counter()
        if seed and pos <= len(seed):
            c[seed[pos - 1]] = 0
        if pos <= self.cap:
            for k, tok in enumerate('ACGT'):
                v = int(self.dense[r, pos - 1, k])
                if v:
                    c[tok] += v
            if self.nflag[r, pos - 1]:
                c['N'] = -1
            if self.dflag[r, pos - 1]:
                c['-'] = -2
        if events is None:
            c.update(self.events.get(r, {}).get(pos, {}))
        else:
            for token, count in events:
                c[token] += count
        return c

    def native_arrays(self):
        """dense (n, cap, 4) int32 and the flags (n, cap) uint8, contiguous
        (converted once when a pileup arrives in another dtype)."""
        if getattr(self, '_native', None) is None:
            d, nf, df = self.dense, self.nflag, self.dflag
            if d.dtype != np.int32 or not d.flags.c_contiguous:
                d = np.ascontiguousarray(d, dtype=np.int32)
            if nf.dtype != np.uint8 or not nf.flags.c_contiguous:
                nf = np.ascontiguousarray(nf != 0, dtype=np.uint8)
            if df.dtype != np.uint8 or not df.flags.c_contiguous:
                df = np.ascontiguousarray(df != 0, dtype=np.uint8)
            self._native = (d, nf, df)
        return self._native

    def _rows(self, r):
        """The reference's fetched counter rows as the native call takes
        them: (cap, 4) int32 counts and uint8 flags, contiguous."""
        d, nf, df = self.dense[r], self.nflag[r], self.dflag[r]
        if d.dtype != np.int32 or not d.flags.c_contiguous:
            d = np.ascontiguousarray(d, dtype=np.int32)
        if nf.dtype != np.uint8 or not nf.flags.c_contiguous:
            nf = np.ascontiguousarray(nf != 0, dtype=np.uint8)
        if df.dtype != np.uint8 or not df.flags.c_contiguous:
            df = np.ascontiguousarray(df != 0, dtype=np.uint8)
        return d, nf, df

    def has_positive(self, r):
        if self.has_events(r):
            return True
        rd, rnf, rdf = self._rows(r)
        return _native.top_tokens(0, len(rd), rd, rnf, rdf, b'', np.zeros(1, dtype=np.uint8))

    def tokens(self, r, seed):
        """Top token per position 1..end-1 (remap.py:318-321), one byte each
        (0: no token), and {index: token} for the positions whose top token
        is longer than one character (a base with its insertion).  The
        base-like entries (counts, seed prefill, 'N', '-') are ranked by the
        library's host code (mh_top_tokens, one pass over the rows); the
        insertion tokens are merged in here."""
        end = max(int(self.max_pos[r]), len(seed) if seed else 0) + 1
        length = end - 1
        tok = np.zeros(max(length, 1), dtype=np.uint8)
        rd, rnf, rdf = self._rows(r)
        sb = seed.encode('latin-1') if seed else b''
        # (no count lies past max_pos: positive over 1..length is over the row)
        self.last_positive = _native.top_tokens(length, min(length, self.cap), rd, rnf, rdf, sb, tok)
        tok = tok[:length]
        longer = {}
        if self.has_events(r):
            d, nf, df = self._slice(r, length)
            # a few events: one Counter per position; many: vectorised (its
            # fixed cost, ~0.1 ms of numpy calls, pays from ~150 events)
            if len(self._ev[r][0]) < 160:
                self._event_tokens_loop(r, seed, length, d, nf, df, tok, longer)
            else:
                self._event_tokens(r, seed, length, d, nf, df, tok, longer)
        return tok, longer

    def _event_tokens_loop(self, r, seed, length, d, nf, df, tok, longer):
        """The positions holding insertion tokens, one Counter each
        (counter_at's, built from plain lists)."""
        ev = {}
        for pos, t, k in zip(*self._ev[r]):
            if pos <= length:
                e = ev.setdefault(pos, {})
                e[t] = e.get(t, 0) + k
        if not ev:
            return
        positions = list(ev)
        idx = np.asarray(positions, dtype=np.int64) - 1
        rows, nfs, dfs = d[idx].tolist(), nf[idx].tolist(), df[idx].tolist()
        nseed = len(seed) if seed else 0
        for pos, row, n_flag, d_flag in zip(positions, rows, nfs, dfs):
            c = {seed[pos - 1]: 0} if pos <= nseed else {}
            for k, v in enumerate(row):
                if v:
                    base = 'ACGT'[k]
                    c[base] = c.get(base, 0) + v
            if n_flag:
                c['N'] = -1
            if d_flag:
                c['-'] = -2
            for token, count in ev[pos].items():
                c[token] = c.get(token, 0) + count
            t = find_top_token(c)
            tok[pos - 1] = ord(t[0]) if t else 0
            if t and len(t) > 1:
                longer[pos - 1] = t

    def _event_tokens(self, r, seed, length, d, nf, df, tok, longer):
        """find_top_token (remap.py:892-902) at the positions holding
        insertion tokens, vectorised: the best event token per position
        (most pairs, then the smallest string) against the best base-like
        entry (a base with pairs or the seed's prefill, else 'N' -1, else
        '-' -2).  Positions with a one-character token (which adds to a base's
        count) or a seed character other than A/C/G/T take the per-position
        Counter instead."""
        ps, ts, cs = self._ev[r]
        pos = np.asarray(ps, dtype=np.int64)
        cnt = np.asarray(cs, dtype=np.int64)
        keep = pos <= length
        if not keep.all():
            sel = np.flatnonzero(keep)
            pos, cnt, ts = pos[sel], cnt[sel], [ts[k] for k in sel.tolist()]
        if len(pos) == 0:
            return
        toks = np.array(ts)
        nseed = len(seed) if seed else 0
        slow = set()
        # one entry per (pos, token), counts summed (the device's are
        # already distinct; a hand-built pileup may repeat one)
        # (the device hands them over in (pos, token) order: no sort then)
        if len(pos) > 1 and not ((pos[1:] > pos[:-1]) | ((pos[1:] == pos[:-1]) & (toks[1:] >= toks[:-1]))).all():
            o2 = np.lexsort((toks, pos))
            pos, toks, cnt = pos[o2], toks[o2], cnt[o2]
        new = np.r_[True, (pos[1:] != pos[:-1]) | (toks[1:] != toks[:-1])]
        if not new.all():
            starts = np.flatnonzero(new)
            pos, toks, cnt = pos[starts], toks[starts], np.add.reduceat(cnt, starts)
        # per position (a run of equal pos), the best token: the most pairs,
        # then the smallest string -- the first index reaching the run's max,
        # tokens being sorted within the run
        starts = np.flatnonzero(np.r_[True, pos[1:] != pos[:-1]])
        run = np.repeat(np.arange(len(starts)), np.diff(np.r_[starts, len(pos)]))
        gmax = np.maximum.reduceat(cnt, starts)
        at = np.where(cnt == gmax[run], np.arange(len(pos)), len(pos))
        best = np.minimum.reduceat(at, starts)
        upos = pos[starts]
        # token lengths from the code points (a str array pads with 0)
        tlen = (toks.view(np.uint32).reshape(len(toks), -1) != 0).sum(axis=1)
        short = tlen < 2
        if short.any():
            slow.update(pos[short].tolist())
        sb = np.full(len(upos), 255, dtype=np.int64)   # the seed's base at the position
        if nseed:
            ins = upos <= nseed
            sc = np.frombuffer(seed.encode('latin-1'), dtype=np.uint8)
            sb[ins] = BASE_INDEX[sc[upos[ins] - 1]]
            odd = ins & (sb == 255)
            if odd.any():
                slow.update(upos[odd].tolist())
        ecnt, etok = cnt[best], toks[best]
        idx = upos - 1
        rows = d[idx]                       # (k, 4) counts A C G T
        present = (rows > 0) | (sb[:, None] == np.arange(4)[None, :])
        vals = np.where(present, rows, np.iinfo(np.int64).min)
        bk = np.argmax(vals, axis=1)        # ties: the first of A < C < G < T
        has_base = present.any(axis=1)
        bcnt = np.where(has_base, vals[np.arange(len(upos)), bk], 0)
        nfl, dfl = nf[idx], df[idx]
        # no base-like entry: 'N' (-1) beats '-' (-2); neither: the event wins
        bcnt = np.where(has_base, bcnt, np.where(nfl, -1, np.where(dfl, -2, np.iinfo(np.int64).min)))
        btok = np.where(has_base, np.array(list('ACGT'))[bk], np.where(nfl, 'N', np.where(dfl, '-', '')))
        ev_wins = (ecnt > bcnt) | ((ecnt == bcnt) & (etok < btok))
        win = np.where(ev_wins, etok, btok)
        # first characters as code points ('' -> 0), the longer tokens by index
        tok[idx] = win.astype('<U1').view(np.uint32)
        multi = np.flatnonzero(np.where(ev_wins, tlen[best], 1) > 1)
        for k, t in zip(multi.tolist(), win[multi].tolist()):
            longer[int(idx[k])] = t
        for p in slow:
            at = np.flatnonzero(pos == p)
            c = self.counter_at(r, p, seed, events=zip(toks[at].tolist(), cnt[at].tolist()))
            t = find_top_token(c)
            tok[p - 1] = ord(t[0]) if t else 0
            longer.pop(p - 1, None)
            if t and len(t) > 1:
                longer[p - 1] = t

    def position_sums(self, r, seed, length):
        """sum(counts[pos].values()) for pos 1..length (remap.py:236-238)."""
        d, nf, df = self._slice(r, length)
        s = d[:, 0] + d[:, 1] + d[:, 2] + d[:, 3] - nf.astype(np.int64) - 2 * df.astype(np.int64)
        if self.has_events(r):
            _r, pos, _o, _l, cnt, _p = self.ev_arrays([r])
            keep = (pos >= 1) & (pos <= length)
            np.add.at(s, pos[keep] - 1, cnt[keep])
        return s


def find_top_token(base_counts):
    """remap.find_top_token (remap.py:892-902)."""
    top_count = top_token = None
    for token, count in base_counts.items():
        if top_count is None or count > top_count or (count == top_count and token < top_token):
            top_token, top_count = token, count
    return top_token


def _text(tok, longer, a, b):
    """Positions [a, b) of a stretch without '-' or missing tokens."""
    keys = [i for i in longer if a <= i < b]
    if not keys:
        return tok[a:b].tobytes().decode('latin-1')
    parts, at = [], a
    for i in sorted(keys):
        parts.append(tok[at:i].tobytes().decode('latin-1'))
        parts.append(longer[i])
        at = i + 1
    parts.append(tok[at:b].tobytes().decode('latin-1'))
    return ''.join(parts)


def _assemble(tok, longer):
    """The deletion-run rule of counts_to_conseqs (remap.py:322-332) over the
    token bytes: a missing token writes 'N' at once, a '-' adds to the open
    deletion, any other token first writes the open deletion when its length
    is not a multiple of 3.  So each maximal stretch of '-' and missing tokens
    becomes its 'N's followed by its '-'s (dropped when their count is a
    multiple of 3, or when the stretch ends the sequence)."""
    n = len(tok)
    gap = (tok == DASH) | (tok == 0)
    if not gap.any():
        return _text(tok, longer, 0, n)
    starts = np.flatnonzero(gap & ~np.r_[False, gap[:-1]])
    ends = np.flatnonzero(gap & ~np.r_[gap[1:], False]) + 1
    parts, at = [], 0
    for a, b in zip(starts.tolist(), ends.tolist()):
        parts.append(_text(tok, longer, at, a))
        dashes = int(np.count_nonzero(tok[a:b] == DASH))
        parts.append('N' * (b - a - dashes))
        if b < n and dashes % 3:
            parts.append('-' * dashes)
        at = b
    parts.append(_text(tok, longer, at, n))
    return ''.join(parts)


def counts_to_conseqs(pile, order, seeds=None):
    """{rname: consensus} in refmap order (remap.py:309-333): every
    reference in one call of the library's host code (mh_conseqs_build: the
    top token of each position's Counter, insertion tokens merged, then the
    deletion-run rule).  counts_to_conseqs_py is the same in Python (the
    tests hold the two equal)."""
    order = list(order)
    if not order:
        return {}
    dense, nflag, dflag = pile.native_arrays()
    lengths, seed_bytes = [], []
    for r in order:
        seed = seeds.get(pile.refnames[r]) if seeds else None
        lengths.append(max(int(pile.max_pos[r]), len(seed) if seed else 0))
        seed_bytes.append(seed.encode('latin-1') if seed else b'')
    built = _native.conseqs_build(order, lengths, seed_bytes, dense, nflag, dflag, *pile.ev_arrays(order))
    return {pile.refnames[r]: text.decode('latin-1') for r, (text, present) in zip(order, built) if present}


def counts_to_conseqs_py(pile, order, seeds=None):
    """counts_to_conseqs in Python (numpy per reference; the tests' second
    implementation)."""
    conseqs = {}
    for r in order:
        name = pile.refnames[r]
        seed = seeds.get(name) if seeds else None
        tok, longer = pile.tokens(r, seed)
        if not (pile.last_positive or pile.has_events(r)):
            continue
        conseqs[name] = _assemble(tok, longer)
    return conseqs


def extract_relevant_seed(aligned_conseq, aligned_seed):
    """remap.extract_relevant_seed (remap.py:129-138): the seed under the
    consensus from its first to its last non-gap column, gaps removed."""
    start = len(aligned_conseq) - len(aligned_conseq.lstrip('-'))
    end = len(aligned_conseq.rstrip('-'))
    if start >= end:
        # no non-gap column: the reference's match is None (AttributeError)
        match = re.match('-*([^-](.*[^-])?)', aligned_conseq)
        return aligned_seed[match.start(1):match.end(1)].replace('-', '')
    return aligned_seed[start:end].replace('-', '')


def clean_sequence(seq, alphabet=HYPHY_NUC_ALPHABET):
    """gotoh2.Aligner.clean_sequence (gotoh2.py:70-72)."""
    return re.sub('[^%s]' % (alphabet,), '?', seq.upper())


def filter_conseqs(ctx, pile, order, new_conseqs, seeds, filter_coverage, distance_report=None):
    """The consensus-distance filter of remap.sam_to_conseqs (:228-268).

    For every consensus (name order) its well-covered positions -- where the
    position's counts, sentinels included, sum to at least filter_coverage
    -- are aligned to every seed (global Gotoh, gop 15 / gep 3, HYPHY_NUC);
    the edit distance to the part of each seed they cover decides: a
    consensus stays when its own seed is no farther than the nearest other
    one.  If none stays, the one with the most merged pairs does.  All the
    K x K alignments and their edit distances are one device batch
    (mh_gotoh_distance_batch): the relevant seed is cut from each alignment
    and measured on the device, and only the distances come back."""
    if not seeds or len(new_conseqs) < 2:
        return new_conseqs
    index = {pile.refnames[r]: r for r in order}
    names = sorted(new_conseqs)
    relevant = {}
    for name in names:
        conseq = new_conseqs[name]
        keep = pile.position_sums(index[name], seeds.get(name), len(conseq)) >= filter_coverage
        covered = np.frombuffer(conseq.encode(), dtype=np.uint8)[keep[:len(conseq)]].tobytes().decode()
        if covered:
            relevant[name] = covered
    jobs = [(name, seed_name) for name in names if name in relevant for seed_name in names]
    # each sequence cleaned once (K seeds, K consensuses; not K x K times)
    clean_seed = {n: clean_sequence(seeds[n]) for n in names}
    clean_rel = {n: clean_sequence(relevant[n]) for n in relevant}
    # every distance in one batch: an exact length bound could skip 43 % of
    # the cells at C4-all size, but in two dependent batches each is as long
    # as its longest pair (profiles/diag/filter_timing.py, lev_pruned_ms)
    dists = ctx.gotoh_distance_many(
        [(clean_seed[seed_name], clean_rel[name], relevant[name]) for name, seed_name in jobs],
        FILTER_GOP, FILTER_GEP, True, HYPHY_NUC_ALPHABET, HYPHY_NUC)
    for result in dists:
        if isinstance(result, Exception):
            raise result
    per_name = {}
    for (name, seed_name), d in zip(jobs, dists):
        per_name.setdefault(name, []).append((seed_name, d))
    filtered = {}
    for name in names:
        if name not in relevant:
            continue
        seed_dist = other_dist = other_seed = None
        for seed_name, d in per_name[name]:
            if seed_name == name:
                seed_dist = d
            elif other_dist is None or d < other_dist:
                other_seed, other_dist = seed_name, d
        if seed_dist <= other_dist:
            filtered[name] = new_conseqs[name]
        if distance_report is not None:
            distance_report[name] = dict(seed_dist=seed_dist, other_dist=other_dist,
                                         other_seed=other_seed)
    if not filtered:
        best_ref = pile.read_count_items(order).most_common(1)[0][0]
        filtered[best_ref] = new_conseqs[best_ref]
    return filtered
