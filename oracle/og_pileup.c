/*
 * oracle/og_pileup.c -- TEST INFRASTRUCTURE ONLY.
 *
 * CPU restatement of the reference's consensus pileup, one merged read pair
 * at a time, used as the checker for micall-lite_amd/csrc/mh_pileup.hip:
 *   merge_reads      micall/core/remap.py:86-126
 *   apply_cigar      micall/core/sam2aln.py:84-153
 *   merge_pairs      micall/core/sam2aln.py:156-237
 *   merge_inserts    micall/core/sam2aln.py:240-273
 *   update_counts    micall/core/remap.py:271-306
 * Output is the reference's refmap in a dense form: per reference and
 * 1-based position, counts of the tokens A, C, G, T, a flag for 'N'
 * (count -1, remap.py:292-293) and a flag for '-' (count -2, :294-295);
 * every other token (base + insertion with len % 3 == 0, :297-299, or an
 * unusual base letter) is emitted as an event (ref, pos, token) to be
 * counted by the caller.  Pinned by tests/golden/pileup_golden.json, which
 * tests/golden/gen_golden.py generates by running the reference
 * sam_to_conseqs on the same SAM text.
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

enum { OP_M = 0, OP_I = 1, OP_D = 2, OP_S = 4 };

typedef struct {
    int32_t flag, ref, pos;     /* ref: index into the caller's @SQ list; pos 1-based */
    int32_t n_cigar;
    const uint32_t *cigar;      /* (len << 4) | op */
    int32_t len;
    const char *seq, *qual;
} og_row;

typedef struct { int32_t ref, pos, tok_off, tok_len; } og_event;

typedef struct { int key; char *seq, *qual; int len; } ins_t;

typedef struct {
    char *seq, *qual;   /* padded read in reference coordinates */
    int len;
    ins_t *ins;
    int n_ins;
} applied_t;

/* apply_cigar with clip_from=0, clip_to=None (the call in merge_reads) */
static int apply_cigar(const og_row *r, int pad, applied_t *out)
{
    int reflen = pad;
    for (int k = 0; k < r->n_cigar; ++k) {
        const int op = r->cigar[k] & 15, n = (int)(r->cigar[k] >> 4);
        if (op != OP_M && op != OP_I && op != OP_D && op != OP_S) return -3; /* :140-142 */
        if (op == OP_M || op == OP_D) reflen += n;
    }
    out->seq = malloc((size_t)reflen + 1);
    out->qual = malloc((size_t)reflen + 1);
    out->ins = malloc(sizeof(ins_t) * (size_t)(r->n_cigar + 1));
    out->n_ins = 0;
    memset(out->seq, '-', (size_t)pad);
    memset(out->qual, '!', (size_t)pad);
    int w = pad, left = 0;
    for (int k = 0; k < r->n_cigar; ++k) {
        const int op = r->cigar[k] & 15, n = (int)(r->cigar[k] >> 4);
        if (op == OP_M) {
            if (left + n > r->len) return -3;
            memcpy(out->seq + w, r->seq + left, (size_t)n);
            memcpy(out->qual + w, r->qual + left, (size_t)n);
            w += n; left += n;
        } else if (op == OP_D) {
            memset(out->seq + w, '-', (size_t)n);
            memset(out->qual + w, ' ', (size_t)n);
            w += n;
        } else if (op == OP_I) {
            if (left + n > r->len) return -3;
            ins_t *t = &out->ins[out->n_ins++];
            t->key = left + pad;       /* quirk: read offset + pad, :133-135 */
            t->len = n;
            t->seq = malloc((size_t)n + 1);
            t->qual = malloc((size_t)n + 1);
            memcpy(t->seq, r->seq + left, (size_t)n);
            memcpy(t->qual, r->qual + left, (size_t)n);
            left += n;
        } else {
            left += n;
        }
        if (left > r->len) return -3;
    }
    if (left < r->len) return -3;
    out->len = w;
    return 0;
}

static void free_applied(applied_t *a)
{
    for (int k = 0; k < a->n_ins; ++k) { free(a->ins[k].seq); free(a->ins[k].qual); }
    free(a->ins); free(a->seq); free(a->qual);
}

/* merge_pairs without insertions (ins1 = ins2 = None).  out needs
 * max(len1, len2) + 1 bytes; returns the merged length. */
static int merge_pairs(const char *s1, const char *q1, int l1, const char *s2, const char *q2,
                       int l2, int q_cutoff, int min_q_delta, char *out)
{
    if (l1 > l2) {
        const char *t = s1; s1 = s2; s2 = t;
        t = q1; q1 = q2; q2 = t;
        int x = l1; l1 = l2; l2 = x;
    }
    const char cut = (char)(q_cutoff + 33);
    int fwd = 0, rev = 0, n = 0;
    for (int i = 0; i < l2; ++i) {
        const char c2 = s2[i];
        if (c2 != '-') rev = 1;
        if (i < l1) {
            const char c1 = s1[i];
            if (!fwd) {
                if (c1 == '-' && c2 == '-') continue;
                fwd = 1;
                memcpy(out, s1, (size_t)i);   /* mseq = seq1[:i] */
                n = i;
            } else if (c1 == '-' && c2 == '-') {
                out[n++] = '-';
                continue;
            }
            const unsigned char a = (unsigned char)q1[i], b = (unsigned char)q2[i];
            if (c1 == c2) {
                out[n++] = (a > (unsigned char)cut || b > (unsigned char)cut) ? c1 : 'N';
            } else {
                const int dq = (int)b - (int)a;
                if ((dq < 0 ? -dq : dq) >= min_q_delta) {
                    const unsigned char m2 = b > (unsigned char)cut ? b : (unsigned char)cut;
                    const unsigned char m1 = a > (unsigned char)cut ? a : (unsigned char)cut;
                    if (a > m2) out[n++] = c1;
                    else if (b > m1) out[n++] = c2;
                    else out[n++] = 'N';
                } else {
                    out[n++] = 'N';
                }
            }
        } else {
            if (c2 == '-') out[n++] = rev ? '-' : 'n';
            else out[n++] = (unsigned char)q2[i] > (unsigned char)cut ? c2 : 'N';
        }
    }
    return n;
}

static int min_qual_above(const char *q, int n, char cut)
{
    unsigned char mn = 255;
    for (int k = 0; k < n; ++k) if ((unsigned char)q[k] < mn) mn = (unsigned char)q[k];
    return mn > (unsigned char)cut;   /* min('') raises in the reference; never empty here */
}

typedef struct { int key; char *seq; int len; } mins_t;

/* merge_inserts(ins1, ins2, q_cutoff), sam2aln.py:240-273 */
static int merge_inserts(const applied_t *a1, const applied_t *a2, int q_cutoff, mins_t *out)
{
    const char cut = (char)(q_cutoff + 33);
    int n = 0;
    if (a1) {
        for (int k = 0; k < a1->n_ins; ++k) {
            const ins_t *t = &a1->ins[k];
            if (!min_qual_above(t->qual, t->len, cut)) continue;
            out[n].key = t->key;
            out[n].seq = malloc((size_t)t->len + 1);
            memcpy(out[n].seq, t->seq, (size_t)t->len);
            out[n].len = t->len;
            ++n;
        }
    }
    if (a2) {
        for (int k = 0; k < a2->n_ins; ++k) {
            const ins_t *t = &a2->ins[k];
            if (!min_qual_above(t->qual, t->len, cut)) continue;
            const ins_t *o = NULL;
            if (a1) for (int z = 0; z < a1->n_ins; ++z) if (a1->ins[z].key == t->key) o = &a1->ins[z];
            const int cap = (o && o->len > t->len ? o->len : t->len) + 1;
            char *buf = malloc((size_t)cap);
            const int len = merge_pairs(o ? o->seq : "", o ? o->qual : "", o ? o->len : 0,
                                        t->seq, t->qual, t->len, q_cutoff, 5, buf);
            int at = -1;
            for (int z = 0; z < n; ++z) if (out[z].key == t->key) at = z;
            if (at < 0) at = n++;
            else free(out[at].seq);
            out[at].key = t->key;
            out[at].seq = buf;
            out[at].len = len;
        }
    }
    return n;
}

static int add_event(og_event *ev, int64_t ev_cap, int64_t *n_ev, char *pool, int64_t pool_cap,
                     int64_t *pool_used, int ref, int pos, char nuc, const char *ins, int ilen)
{
    if (*n_ev >= ev_cap || *pool_used + 1 + ilen > pool_cap) return -2;
    og_event *e = &ev[(*n_ev)++];
    e->ref = ref;
    e->pos = pos;
    e->tok_off = (int32_t)*pool_used;
    e->tok_len = 1 + ilen;
    pool[(*pool_used)++] = nuc;
    memcpy(pool + *pool_used, ins, (size_t)ilen);
    *pool_used += ilen;
    return 0;
}

/* Where one merged pair's counts go.  Serial: plain stores.  Threaded
 * (og_pileup_mt): the dense counters, read counts, first unit and max
 * position are updated atomically (every update commutes), and the events
 * go to a per-thread list that is appended in unit order afterwards. */
typedef struct {
    int n_refs;
    int32_t cap;
    int32_t *dense;
    int64_t *read_counts, *first_unit;
    int32_t *max_pos;
    og_event *ev;
    int64_t ev_cap, *n_ev;
    char *pool;
    int64_t pool_cap, *pool_used;
    int atomic;
} sink_t;

static void max_i32(int32_t *p, int32_t v, int atomic)
{
    if (!atomic) { if (v > *p) *p = v; return; }
    int32_t cur = __atomic_load_n(p, __ATOMIC_RELAXED);
    while (v > cur && !__atomic_compare_exchange_n(p, &cur, v, 1, __ATOMIC_RELAXED, __ATOMIC_RELAXED))
        ;
}

static void min_first(int64_t *p, int64_t v, int atomic)
{
    if (!atomic) { if (*p < 0) *p = v; return; }
    int64_t cur = __atomic_load_n(p, __ATOMIC_RELAXED);
    while ((cur < 0 || v < cur) &&
           !__atomic_compare_exchange_n(p, &cur, v, 1, __ATOMIC_RELAXED, __ATOMIC_RELAXED))
        ;
}

static void bump32(int32_t *p, int atomic)
{
    if (atomic) __atomic_fetch_add(p, 1, __ATOMIC_RELAXED); else *p += 1;
}

/* one unit (merge_reads + update_counts); returns a status */
static int pile_unit(const og_row *rows, const int64_t *unit_rows, int64_t u, int q_cutoff,
                     const sink_t *k)
{
    const og_row *r1 = unit_rows[2 * u] >= 0 ? &rows[unit_rows[2 * u]] : NULL;
    const og_row *r2 = unit_rows[2 * u + 1] >= 0 ? &rows[unit_rows[2 * u + 1]] : NULL;
    if (!r1) return 0;
    if (r2 && r1->ref != r2->ref) return 0;                 /* remap.py:96-98 */
    const og_row *mapped[2];
    int nm = 0;
    if (!(r1->flag & 4)) mapped[nm++] = r1;
    if (r2 && !(r2->flag & 4)) mapped[nm++] = r2;
    if (nm == 0) return 0;                                  /* :111-112 */
    const int ref = mapped[0]->ref;
    if (ref < 0 || ref >= k->n_refs) return -3;
    applied_t a1, a2;
    memset(&a2, 0, sizeof(a2));
    if (apply_cigar(mapped[0], mapped[0]->pos - 1, &a1)) return -3;
    if (nm == 2 && apply_cigar(mapped[1], mapped[1]->pos - 1, &a2)) { free_applied(&a1); return -3; }
    const int mlen_cap = (a1.len > a2.len ? a1.len : a2.len) + 1;
    char *mseq = malloc((size_t)mlen_cap);
    const int ml = merge_pairs(a1.seq, a1.qual, a1.len, nm == 2 ? a2.seq : "", nm == 2 ? a2.qual : "",
                               nm == 2 ? a2.len : 0, q_cutoff, 5, mseq);
    mins_t *mi = malloc(sizeof(mins_t) * (size_t)(a1.n_ins + a2.n_ins + 1));
    const int nmi = merge_inserts(&a1, nm == 2 ? &a2 : NULL, q_cutoff, mi);

    if (k->atomic) __atomic_fetch_add(&k->read_counts[ref], 1, __ATOMIC_RELAXED);
    else k->read_counts[ref] += 1;
    min_first(&k->first_unit[ref], u, k->atomic);
    int started = 0, status = 0;
    for (int i = 0; i < ml && status == 0; ++i) {
        const char c = mseq[i];
        const int pos = i + 1;
        if (!started) {
            if (c == '-') continue;
            started = 1;
        }
        if (c == 'n') continue;
        if (pos > k->cap) { status = -3; break; }
        max_i32(&k->max_pos[ref], pos, k->atomic);
        int32_t *cell = k->dense + ((size_t)ref * (size_t)k->cap + (size_t)(pos - 1)) * 6;
        if (c == 'N') { cell[4] = 1; continue; }     /* flags: every writer stores 1 */
        if (c == '-') { cell[5] = 1; continue; }
        const mins_t *ins = NULL;
        for (int z = 0; z < nmi; ++z) if (mi[z].key == pos) ins = &mi[z];
        if (ins && ins->len > 0 && ins->len % 3 == 0) {
            status = add_event(k->ev, k->ev_cap, k->n_ev, k->pool, k->pool_cap, k->pool_used, ref,
                               pos, c, ins->seq, ins->len);
        } else if (c == 'A') bump32(&cell[0], k->atomic);
        else if (c == 'C') bump32(&cell[1], k->atomic);
        else if (c == 'G') bump32(&cell[2], k->atomic);
        else if (c == 'T') bump32(&cell[3], k->atomic);
        else status = add_event(k->ev, k->ev_cap, k->n_ev, k->pool, k->pool_cap, k->pool_used, ref,
                                pos, c, "", 0);
    }
    for (int z = 0; z < nmi; ++z) free(mi[z].seq);
    free(mi);
    free(mseq);
    free_applied(&a1);
    if (nm == 2) free_applied(&a2);
    return status;
}

/*
 * units: n_units pairs of row indices (unit_rows[2u], unit_rows[2u+1]; -1 =
 * no mate), as matchmaker (remap.py:853-889) yields them.
 * dense: n_refs x cap x 6 int32 (A, C, G, T, N-flag, del-flag), pos 1..cap.
 * read_counts[ref] += 1 per merged pair (remap.py:191); first_unit[ref] =
 * first unit index that merged into ref (refmap insertion order);
 * max_pos[ref] = largest position whose counter was touched.
 */
int og_pileup(int n_refs, int32_t cap, const og_row *rows, int64_t n_units,
              const int64_t *unit_rows, int q_cutoff, int32_t *dense, int64_t *read_counts,
              int64_t *first_unit, int32_t *max_pos, og_event *ev, int64_t ev_cap,
              int64_t *n_ev, char *pool, int64_t pool_cap, int64_t *pool_used)
{
    *n_ev = 0;
    *pool_used = 0;
    const sink_t k = { n_refs, cap, dense, read_counts, first_unit, max_pos, ev, ev_cap, n_ev,
                       pool, pool_cap, pool_used, 0 };
    int status = 0;
    for (int64_t u = 0; u < n_units && status == 0; ++u) status = pile_unit(rows, unit_rows, u, q_cutoff, &k);
    return status;
}

/* og_pileup over nthreads threads (the CPU baseline of bench.py): the same
 * counters and the same event list, in the same order. */
int og_pileup_mt(int n_refs, int32_t cap, const og_row *rows, int64_t n_units,
                 const int64_t *unit_rows, int q_cutoff, int32_t *dense, int64_t *read_counts,
                 int64_t *first_unit, int32_t *max_pos, og_event *ev, int64_t ev_cap,
                 int64_t *n_ev, char *pool, int64_t pool_cap, int64_t *pool_used, int nthreads)
{
    if (nthreads < 1) nthreads = 1;
    *n_ev = 0;
    *pool_used = 0;
    int status = 0;
    og_event **tev = calloc((size_t)nthreads, sizeof(og_event *));
    char **tpool = calloc((size_t)nthreads, sizeof(char *));
    int64_t *tn = calloc((size_t)nthreads, sizeof(int64_t)), *tused = calloc((size_t)nthreads, sizeof(int64_t));
    const int64_t tev_cap = ev_cap / nthreads + 1024, tpool_cap = pool_cap / nthreads + 4096;
#pragma omp parallel num_threads(nthreads)
    {
        int t = 0;
#ifdef _OPENMP
        t = omp_get_thread_num();
#endif
        tev[t] = malloc(sizeof(og_event) * (size_t)tev_cap);
        tpool[t] = malloc((size_t)tpool_cap);
        const sink_t k = { n_refs, cap, dense, read_counts, first_unit, max_pos, tev[t], tev_cap,
                           &tn[t], tpool[t], tpool_cap, &tused[t], 1 };
        const int64_t per = (n_units + nthreads - 1) / nthreads;
        const int64_t lo = per * t, hi = lo + per < n_units ? lo + per : n_units;
        int st = 0;
        for (int64_t u = lo; u < hi && st == 0; ++u) st = pile_unit(rows, unit_rows, u, q_cutoff, &k);
        if (st) {
#pragma omp critical
            if (st < status) status = st;
        }
    }
    for (int t = 0; t < nthreads && status == 0; ++t) {     /* contiguous blocks: unit order */
        if (*n_ev + tn[t] > ev_cap || *pool_used + tused[t] > pool_cap) { status = -2; break; }
        for (int64_t e = 0; e < tn[t]; ++e) {
            ev[*n_ev + e] = tev[t][e];
            ev[*n_ev + e].tok_off += (int32_t)*pool_used;
        }
        memcpy(pool + *pool_used, tpool[t], (size_t)tused[t]);
        *n_ev += tn[t];
        *pool_used += tused[t];
    }
    for (int t = 0; t < nthreads; ++t) { free(tev[t]); free(tpool[t]); }
    free(tev); free(tpool); free(tn); free(tused);
    return status;
}
