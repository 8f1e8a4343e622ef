/*
 * oracle/og_mapper.c -- TEST INFRASTRUCTURE ONLY.
 *
 * CPU oracle of the read mapper that replaces the reference's bowtie2 2.2.8
 * shell-out (micall/core/prelim_map.py:114-140 end-to-end,
 * micall/core/remap.py:701-755 --local).  bowtie2 is an external binary that
 * is absent from /root/reference and from this image, so parity with it is
 * UNPINNED; this file is the executable specification the HIP mapper
 * (micall-lite_amd/csrc/mh_map.hip) must reproduce bit for bit, and it is
 * the mapper behind oracle/bowtie2_shim.py, which lets the stock reference
 * pipeline (bin/micall -> prelim_map -> remap -> sam2aln) produce the golden
 * CSVs under tests/golden/.
 *
 * The scoring and seeding follow bowtie2's documented defaults plus the
 * flags MiCall passes (--rdg 10,3 --rfg 10,3 -X 1200; --local for remap):
 *   match bonus 0 (end-to-end) / 2 (local); mismatch penalty
 *   2 + min(Q,40)/10 (--mp 6,2 quality-scaled); N penalty 1 (--np 1);
 *   gap of length k costs open + k*ext; no gap within 4 bases of either read
 *   end (--gbar 4); minimum score -0.6-0.6*L (e2e) or 20+8*ln(L) (local);
 *   at most 0.15*L ambiguous positions (--n-ceil); exact seeds of 22 (e2e) /
 *   20 (local) nt every 1+1.15*sqrt(L) / 1+0.75*sqrt(L) nt on both strands.
 * Deterministic choices where bowtie2 randomises (documented in DESIGN.md):
 *   hits are clustered by diagonal, the 4 best-supported clusters are
 *   extended by banded DP (the seeded diagonal +- og_band_half: bowtie2's
 *   gap limit for its DP rectangle, maxhalf 15), ties break towards the
 *   lower-ranked candidate / smaller coordinates, traceback prefers
 *   diagonal > insertion > deletion and gap-open over gap-extend.
 */
#include "og_mapper.h"

#include <limits.h>
#include <math.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

#define GBAR 4
#define NPEN 1

/* ------------------------------------------------------------------ */
/* per-length tables                                                  */
/* ------------------------------------------------------------------ */
int og_seed_interval(int mode, int len)
{
    const double f = mode == OG_LOCAL ? 0.75 : 1.15;
    int iv = (int)(1.0 + f * sqrt((double)len) + 0.5);
    return iv < 1 ? 1 : iv;
}

int og_min_score(int mode, int len)
{
    if (mode == OG_LOCAL) {
        double v = 20.0 + 8.0 * log((double)(len > 0 ? len : 1));
        long s = (long)v;
        return (int)(s < 0 ? 0 : s);
    }
    long s = (long)(-0.6 + -0.6 * (double)len);
    return (int)(s > 0 ? 0 : s);
}

int og_n_ceil(int len) { return (int)(0.0 + 0.15 * (double)len); }

/* Gaps of one kind an alignment can hold and still reach minsc from the
 * perfect score: the first costs open + ext, each further one ext (bowtie2
 * Scoring::maxReadGaps / maxRefGaps). */
static int max_gaps(int perfect, int minsc, int oe, int ex)
{
    int sc = perfect, num = 0;
    while (sc >= minsc) {
        sc -= num == 0 ? oe : ex;
        ++num;
    }
    return num - 1;
}

/* Half-width of the DP band around the seeded diagonal: the larger of the
 * two gap limits, capped at bowtie2's maxhalf (DynProgFramer::
 * frameSeedExtensionRect: maxgap = min(max(read gaps, ref gaps), maxhalf)). */
int og_band_half(const og_params *par, int len)
{
    const int perfect = par->mode == OG_LOCAL ? 2 * len : 0;
    const int minsc = og_min_score(par->mode, len);
    const int gd = max_gaps(perfect, minsc, par->rdg_open + par->rdg_ext, par->rdg_ext);
    const int gi = max_gaps(perfect, minsc, par->rfg_open + par->rfg_ext, par->rfg_ext);
    int h = gd > gi ? gd : gi;
    if (h > OG_MAXHALF) h = OG_MAXHALF;
    return h < 0 ? 0 : h;
}

static inline int mm_pen(int qchar)
{
    int q = qchar - 33;
    if (q < 0) q = 0;
    if (q > 40) q = 40;
    return 2 + q / 10;
}

static inline uint8_t base_code(uint8_t c)
{
    switch (c) {
    case 'A': case 'a': return 0;
    case 'C': case 'c': return 1;
    case 'G': case 'g': return 2;
    case 'T': case 't': return 3;
    default: return 4;
    }
}

/* ------------------------------------------------------------------ */
/* index: every N-free seed-length window of every reference, sorted   */
/* by (key, ref, pos).  Replaces bowtie2-build (prelim_map.py:106).    */
/* ------------------------------------------------------------------ */
typedef struct { uint64_t key; int32_t ref, pos; } ent_t;

struct og_index {
    int n_refs, seedlen;
    int32_t *lens;
    uint8_t **codes;
    int64_t n_ent;
    ent_t *ent;
};

static int cmp_ent(const void *a, const void *b)
{
    const ent_t *x = a, *y = b;
    if (x->key != y->key) return x->key < y->key ? -1 : 1;
    if (x->ref != y->ref) return x->ref < y->ref ? -1 : 1;
    return (x->pos > y->pos) - (x->pos < y->pos);
}

og_index *og_index_build(int n_refs, const char *const *seqs, int seedlen)
{
    og_index *ix = calloc(1, sizeof(*ix));
    ix->n_refs = n_refs;
    ix->seedlen = seedlen;
    ix->lens = malloc(sizeof(int32_t) * (size_t)(n_refs > 0 ? n_refs : 1));
    ix->codes = malloc(sizeof(uint8_t *) * (size_t)(n_refs > 0 ? n_refs : 1));
    int64_t total = 0;
    for (int r = 0; r < n_refs; ++r) {
        const int L = (int)strlen(seqs[r]);
        ix->lens[r] = L;
        ix->codes[r] = malloc((size_t)L + 1);
        for (int p = 0; p < L; ++p) ix->codes[r][p] = base_code((uint8_t)seqs[r][p]);
        total += L;
    }
    ix->ent = malloc(sizeof(ent_t) * (size_t)(total > 0 ? total : 1));
    int64_t n = 0;
    const uint64_t mask = seedlen >= 32 ? ~0ull : ((1ull << (2 * seedlen)) - 1);
    for (int r = 0; r < n_refs; ++r) {
        const uint8_t *c = ix->codes[r];
        const int L = ix->lens[r];
        uint64_t key = 0;
        int last_n = -1;
        for (int p = 0; p < L; ++p) {
            if (c[p] > 3) last_n = p;
            key = ((key << 2) | (c[p] & 3)) & mask;
            if (p >= seedlen - 1 && last_n <= p - seedlen) {
                ix->ent[n].key = key;
                ix->ent[n].ref = r;
                ix->ent[n].pos = p - seedlen + 1;
                ++n;
            }
        }
    }
    ix->n_ent = n;
    qsort(ix->ent, (size_t)n, sizeof(ent_t), cmp_ent);
    return ix;
}

void og_index_free(og_index *ix)
{
    if (!ix) return;
    for (int r = 0; r < ix->n_refs; ++r) free(ix->codes[r]);
    free(ix->codes);
    free(ix->lens);
    free(ix->ent);
    free(ix);
}

static void lookup(const og_index *ix, uint64_t key, int64_t *lo, int64_t *hi)
{
    int64_t a = 0, b = ix->n_ent;
    while (a < b) { int64_t mid = (a + b) / 2; if (ix->ent[mid].key < key) a = mid + 1; else b = mid; }
    *lo = a;
    b = ix->n_ent;
    while (a < b) { int64_t mid = (a + b) / 2; if (ix->ent[mid].key <= key) a = mid + 1; else b = mid; }
    *hi = a;
}

/* ------------------------------------------------------------------ */
/* candidates                                                          */
/* ------------------------------------------------------------------ */
typedef struct { int32_t strand, ref, diag; } hit_t;
typedef struct { int32_t strand, ref, center, support; } cand_t;

static int cmp_hit(const void *a, const void *b)
{
    const hit_t *x = a, *y = b;
    if (x->strand != y->strand) return x->strand - y->strand;
    if (x->ref != y->ref) return x->ref - y->ref;
    return (x->diag > y->diag) - (x->diag < y->diag);
}

static int cand_before(const cand_t *x, const cand_t *y)
{
    if (x->support != y->support) return x->support > y->support;
    if (x->strand != y->strand) return x->strand < y->strand;
    if (x->ref != y->ref) return x->ref < y->ref;
    return x->center < y->center;
}

/* Returns the number of candidates written to out (<= OG_MAXCAND). */
static int find_candidates(const og_index *ix, int mode, const uint8_t *const codes[2], int m,
                           cand_t *out, hit_t *hits, int *n_clusters)
{
    *n_clusters = 0;
    const int SL = ix->seedlen;
    if (m < SL) return 0;
    const int iv = og_seed_interval(mode, m);
    int ns = 1 + (m - SL) / iv;
    if (ns > OG_MAXSEEDS) ns = OG_MAXSEEDS;
    int nh = 0;
    for (int s = 0; s < 2 && nh < OG_MAXHITS_MATE; ++s) {
        for (int t = 0; t < ns && nh < OG_MAXHITS_MATE; ++t) {
            const int o = t * iv;
            uint64_t key = 0;
            int has_n = 0;
            for (int x = 0; x < SL; ++x) {
                const uint8_t c = codes[s][o + x];
                if (c > 3) { has_n = 1; break; }
                key = (key << 2) | c;
            }
            if (has_n) continue;
            int64_t lo, hi;
            lookup(ix, key, &lo, &hi);
            if (hi - lo > OG_MAXHITS_SEED) continue;
            for (int64_t e = lo; e < hi && nh < OG_MAXHITS_MATE; ++e) {
                hits[nh].strand = s;
                hits[nh].ref = ix->ent[e].ref;
                hits[nh].diag = ix->ent[e].pos - o;
                ++nh;
            }
        }
    }
    if (nh == 0) return 0;
    qsort(hits, (size_t)nh, sizeof(hit_t), cmp_hit);
    int nc = 0;
    cand_t best[OG_MAXCAND];
    int h0 = 0;
    while (h0 < nh) {
        int h1 = h0 + 1;
        while (h1 < nh && hits[h1].strand == hits[h0].strand && hits[h1].ref == hits[h0].ref &&
               hits[h1].diag - hits[h1 - 1].diag <= OG_CLUSTER_GAP)
            ++h1;
        /* center = most frequent diagonal, ties -> smallest */
        int center = hits[h0].diag, center_n = 0;
        for (int a = h0; a < h1;) {
            int b = a + 1;
            while (b < h1 && hits[b].diag == hits[a].diag) ++b;
            if (b - a > center_n) { center_n = b - a; center = hits[a].diag; }
            a = b;
        }
        cand_t c = { hits[h0].strand, hits[h0].ref, center, h1 - h0 };
        ++*n_clusters;
        /* insert into the top-K list (sorted by cand_before) */
        int at = nc;
        while (at > 0 && cand_before(&c, &best[at - 1])) --at;
        if (at < OG_MAXCAND) {
            int last = nc < OG_MAXCAND ? nc : OG_MAXCAND - 1;
            for (int z = last; z > at; --z) best[z] = best[z - 1];
            best[at] = c;
            if (nc < OG_MAXCAND) ++nc;
        }
        h0 = h1;
    }
    memcpy(out, best, sizeof(cand_t) * (size_t)nc);
    return nc;
}

/* ------------------------------------------------------------------ */
/* banded affine-gap DP + traceback                                    */
/* ------------------------------------------------------------------ */
typedef struct {
    int valid;
    int fail;                  /* why not valid: FAIL_* (diagnostics only) */
    int strand, ref, pos, end; /* [pos, end) reference span after trimming */
    int score;
    int xm, xo, xg, nm;
    int n_cigar;
    uint32_t cigar[OG_MAXOPS];
} caln_t;

static inline int imax(int a, int b) { return a > b ? a : b; }

enum { FAIL_NONE = 0, FAIL_SCORE = 1, FAIL_NCEIL = 2, FAIL_OTHER = 3 };

#ifdef OG_ROW_PROBE
void og_row_probe(int W, const int *H1, const int *H, int oeD, int exD);
#endif

static void dp_extend(const og_index *ix, const og_params *par, const uint8_t *rd,
                      const uint8_t *qv, int m, const cand_t *cd, uint8_t *bits,
                      uint8_t *ops, caln_t *out)
{
    const int local = par->mode == OG_LOCAL;
    const int ma = local ? 2 : 0;
    const int oeI = par->rfg_open + par->rfg_ext, exI = par->rfg_ext;
    const int oeD = par->rdg_open + par->rdg_ext, exD = par->rdg_ext;
    const uint8_t *ref = ix->codes[cd->ref];
    const int reflen = ix->lens[cd->ref];
    const int half = og_band_half(par, m), W = 2 * half + 1;   /* diagonals d0 .. d0 + W - 1 */
    const int d0 = cd->center - half;
    int Hp[OG_BAND], Ep[OG_BAND], H[OG_BAND], E[OG_BAND], F[OG_BAND], Hd[OG_BAND], H1[OG_BAND];
    uint8_t eb[OG_BAND];
    for (int k = 0; k < OG_BAND; ++k) { Hp[k] = 0; Ep[k] = OG_NEG; }
    int best = OG_NEG, bi = -1, bk = -1;
    out->valid = 0;
    out->fail = FAIL_SCORE;

    for (int i = 0; i < m; ++i) {
        const int gap_ok = i >= GBAR && i < m - GBAR;
        const int rb = rd[i], pen = mm_pen(qv[i]);
        for (int k = 0; k < W; ++k) {
            const int j = i + d0 + k;
            const int g = (j >= 0 && j < reflen) ? ref[j] : 4;
            const int s = (rb > 3 || g > 3) ? -NPEN : (rb == g ? ma : -pen);
            Hd[k] = Hp[k] + s;
            if (gap_ok && k + 1 < W) {
                const int ext = Ep[k + 1] - exI, opn = Hp[k + 1] - oeI;
                E[k] = imax(ext, opn);
                eb[k] = ext > opn;
            } else {
                E[k] = OG_NEG;
                eb[k] = 0;
            }
            H1[k] = imax(Hd[k], E[k]);
            if (local) H1[k] = imax(H1[k], 0);
        }
        for (int k = 0; k < W; ++k) {
            int fb = 0;
            if (gap_ok && k > 0) {
                const int ext = F[k - 1] - exD, opn = H[k - 1] - oeD;
                F[k] = imax(ext, opn);
                fb = ext > opn;
            } else {
                F[k] = OG_NEG;
            }
            H[k] = imax(H1[k], F[k]);
            int src;
            if (local && H[k] == 0) src = 0;
            else if (H[k] == Hd[k]) src = 1;
            else if (H[k] == E[k]) src = 2;
            else src = 3;
            bits[(size_t)i * OG_BAND + k] = (uint8_t)(src | (eb[k] << 2) | (fb << 3));
            if ((local || i == m - 1) && H[k] > best) { best = H[k]; bi = i; bk = k; }
        }
#ifdef OG_ROW_PROBE
        /* diagnostics build only (profiles/diag/lazy_f_probe.py) */
        if (gap_ok) og_row_probe(W, H1, H, oeD, exD);
#endif
        memcpy(Hp, H, sizeof(Hp));
        memcpy(Ep, E, sizeof(Ep));
    }
    if (bi < 0) return;
    if (local && best <= 0) return;
    if (best < og_min_score(par->mode, m)) return;
    out->fail = FAIL_OTHER;

    /* traceback: ops collected back to front */
    int i = bi, k = bk, state = 0, nops = 0;
    int first_j = 0;
    const int last_j = bi + d0 + bk;
    for (;;) {
        const uint8_t b = bits[(size_t)i * OG_BAND + k];
        if (state == 0) {
            const int src = b & 3;
            if (src == 0) break;
            if (src == 1) {
                ops[nops++] = OG_OP_M;
                first_j = i + d0 + k;
                if (--i < 0) break;
            } else {
                state = src == 2 ? 1 : 2;
            }
        } else if (state == 1) {
            ops[nops++] = OG_OP_I;
            state = (b >> 2) & 1 ? 1 : 0;
            --i; ++k;
            if (i < 0 || k >= W) return; /* unreachable by construction */
        } else {
            ops[nops++] = OG_OP_D;
            state = (b >> 3) & 1 ? 2 : 0;
            --k;
            if (k < 0) return; /* unreachable by construction */
        }
    }
    const int start_i = i + 1;
    /* reverse to forward order */
    for (int a = 0, z = nops - 1; a < z; ++a, --z) { uint8_t t = ops[a]; ops[a] = ops[z]; ops[z] = t; }

    /* ambiguous positions over the untrimmed alignment (--n-ceil) */
    {
        int nn = 0, ri = start_i, rj = first_j;
        for (int o = 0; o < nops; ++o) {
            if (ops[o] == OG_OP_M) {
                const int g = (rj >= 0 && rj < reflen) ? ref[rj] : 4;
                if (rd[ri] > 3 || g > 3) ++nn;
                ++ri; ++rj;
            } else if (ops[o] == OG_OP_I) ++ri;
            else ++rj;
        }
        if (nn > og_n_ceil(m)) { out->fail = FAIL_NCEIL; return; }
    }

    /* trim columns that hang off either reference end into soft clips */
    int lo = 0, hi = nops, clipL = start_i, clipR = m - 1 - bi, jL = first_j, jR = last_j;
    while (lo < hi && !(ops[lo] == OG_OP_M && jL >= 0)) {
        if (ops[lo] == OG_OP_M) { ++clipL; ++jL; }
        else if (ops[lo] == OG_OP_I) ++clipL;
        else ++jL;
        ++lo;
    }
    while (hi > lo && !(ops[hi - 1] == OG_OP_M && jR < reflen)) {
        if (ops[hi - 1] == OG_OP_M) { ++clipR; --jR; }
        else if (ops[hi - 1] == OG_OP_I) ++clipR;
        else --jR;
        --hi;
    }
    if (lo >= hi) return;

    /* stats + run-length CIGAR */
    int xm = 0, xo = 0, xg = 0, nc = 0;
    int ri = clipL, rj = jL;
    if (clipL) out->cigar[nc++] = ((uint32_t)clipL << 4) | OG_OP_S;
    for (int o = lo; o < hi;) {
        int p = o + 1;
        while (p < hi && ops[p] == ops[o]) ++p;
        const int len = p - o;
        if (nc >= OG_MAXOPS - 1) return;
        out->cigar[nc++] = ((uint32_t)len << 4) | ops[o];
        if (ops[o] == OG_OP_M) {
            for (int x = 0; x < len; ++x, ++ri, ++rj) {
                const int g = ref[rj];
                if (rd[ri] > 3 || g > 3 || rd[ri] != g) ++xm;
            }
        } else {
            ++xo;
            xg += len;
            if (ops[o] == OG_OP_I) ri += len; else rj += len;
        }
        o = p;
    }
    if (clipR) out->cigar[nc++] = ((uint32_t)clipR << 4) | OG_OP_S;
    out->n_cigar = nc;
    out->valid = 1;
    out->fail = FAIL_NONE;
    out->strand = cd->strand;
    out->ref = cd->ref;
    out->pos = jL;
    out->end = jR + 1;
    out->score = best;
    out->xm = xm; out->xo = xo; out->xg = xg; out->nm = xm + xg;
}

/* ------------------------------------------------------------------ */
/* MAPQ: bowtie2 "V2"-style table over (best, second best, min score). */
/* Unpinned (bowtie2 absent); integer thresholds, see DESIGN.md.       */
/* ------------------------------------------------------------------ */
int og_mapq(int mode, int len, int best, int has_sec, int sec)
{
    const int perfect = mode == OG_LOCAL ? 2 * len : 0;
    const int minsc = og_min_score(mode, len);
    int diff = perfect - minsc;
    if (diff < 1) diff = 1;
    const int over = best - minsc;
    /* over >= diff*f  <=>  10*over >= f10*diff */
#define GE(x, f10) (10 * (long)(x) >= (long)(f10) * diff)
    if (!has_sec) {
        if (GE(over, 8)) return mode == OG_LOCAL ? 44 : 42;
        if (GE(over, 7)) return 40;
        if (GE(over, 6)) return 24;
        if (GE(over, 5)) return 23;
        if (GE(over, 4)) return 8;
        if (GE(over, 3)) return 3;
        return 0;
    }
    int bd = best - sec;
    if (bd < 0) bd = -bd;
    const int top = over == diff;
    if (GE(bd, 10)) return top ? 39 : 33;
    if (GE(bd, 9)) return top ? 38 : 27;
    if (GE(bd, 8)) return top ? 37 : 26;
    if (GE(bd, 7)) return top ? 36 : 25;
    if (GE(bd, 6)) return top ? 35 : 21;
    if (GE(bd, 5)) return top ? 34 : GE(over, 8) ? 25 : GE(over, 7) ? 16 : 5;
    if (GE(bd, 4)) return top ? 33 : GE(over, 8) ? 21 : GE(over, 7) ? 14 : 4;
    if (GE(bd, 3)) return top ? 32 : GE(over, 8) ? 18 : GE(over, 7) ? 10 : 3;
    if (GE(bd, 2)) return top ? 31 : GE(over, 8) ? 16 : GE(over, 7) ? 9 : 2;
    if (GE(bd, 1)) return top ? 30 : GE(over, 8) ? 12 : GE(over, 7) ? 7 : 1;
    if (bd > 0) return GE(over, 6) ? 2 : 1;
    return GE(over, 6) ? 1 : 0;
#undef GE
}

/* ------------------------------------------------------------------ */
/* per mate: candidates -> DP -> best / second best                     */
/* ------------------------------------------------------------------ */
typedef struct {
    int n;            /* candidate alignments evaluated */
    caln_t a[OG_MAXCAND];
    int best;         /* index of best valid alignment, -1 if none */
    int yf;
    int n_clusters;   /* hit clusters before the top-OG_MAXCAND cut (diagnostics) */
    int rescued;      /* the alignment came from mate rescue */
} mate_t;

typedef struct {
    uint8_t *codes[2], *quals[2];
    hit_t *hits;
    uint8_t *bits, *ops;
} scratch_t;

/* 2-bit codes of a read on both strands (strand 1 = reverse complement,
 * qualities reversed with it); returns the number of ambiguous bases. */
static int load_codes(const uint8_t *seq, const uint8_t *qual, int m, scratch_t *sc)
{
    int nN = 0;
    for (int i = 0; i < m; ++i) {
        const uint8_t c = base_code(seq[i]);
        sc->codes[0][i] = c;
        sc->codes[1][m - 1 - i] = c > 3 ? 4 : (uint8_t)(3 - c);
        sc->quals[0][i] = qual[i];
        sc->quals[1][m - 1 - i] = qual[i];
        nN += c > 3;
    }
    return nN;
}

static void map_mate(const og_index *ix, const og_params *par, const uint8_t *seq,
                     const uint8_t *qual, int m, scratch_t *sc, mate_t *mt)
{
    mt->n = 0;
    mt->best = -1;
    mt->yf = OG_YF_NONE;
    mt->n_clusters = 0;
    mt->rescued = 0;
    if (m == 0) { mt->yf = OG_YF_LN; return; }
    if (load_codes(seq, qual, m, sc) > og_n_ceil(m)) { mt->yf = OG_YF_NS; return; }
    cand_t cands[OG_MAXCAND];
    const uint8_t *cc[2] = { sc->codes[0], sc->codes[1] };
    const int nc = find_candidates(ix, par->mode, cc, m, cands, sc->hits, &mt->n_clusters);
    for (int c = 0; c < nc; ++c) {
        const int s = cands[c].strand;
        dp_extend(ix, par, sc->codes[s], sc->quals[s], m, &cands[c], sc->bits, sc->ops, &mt->a[c]);
        mt->a[c].strand = s;
        if (mt->a[c].valid && (mt->best < 0 || mt->a[c].score > mt->a[mt->best].score)) mt->best = c;
    }
    mt->n = nc;
}

/* ------------------------------------------------------------------ */
/* Mate rescue.  When only one mate of a pair aligns, bowtie2 looks for */
/* the other one in the reference window the fragment-length limit     */
/* allows next to the aligned mate (the anchor) and aligns it there by  */
/* dynamic programming (Langmead & Salzberg 2012, paired-end search;    */
/* bowtie2 2.2.8 SwDriver::extendSeedsPaired, not in this image).  Here */
/* the window is the -X span on the anchor's side in fr orientation:    */
/*   anchor forward at [pos, end): the mate lies in [pos, pos + maxins) */
/*   anchor reverse at [pos, end): the mate lies in [end - maxins, end) */
/* (clipped to the reference), on the opposite strand.  Its diagonal is */
/* the one with the most base matches over the window (ties: leftmost), */
/* and the standard banded DP around it (dp_extend, same scoring, same  */
/* --score-min and --n-ceil) decides whether the mate aligns.            */
/* ------------------------------------------------------------------ */
static int rescue_diagonal(const og_index *ix, const caln_t *anchor, const uint8_t *codes, int m,
                           int maxins, int *diag)
{
    const int L = ix->lens[anchor->ref];
    long lo = anchor->strand == 0 ? anchor->pos : (long)anchor->end - maxins;
    long hi = anchor->strand == 0 ? (long)anchor->pos + maxins : anchor->end;
    if (lo < 0) lo = 0;
    if (hi > L) hi = L;
    if (m == 0 || hi - lo < m) return 0;
    const uint8_t *ref = ix->codes[anchor->ref];
    int best = -1;
    for (long d = lo; d + m <= hi; ++d) {
        int s = 0;
        for (int i = 0; i < m; ++i) s += codes[i] < 4 && codes[i] == ref[d + i];
        if (s > best) { best = s; *diag = (int)d; }
    }
    return 1;
}

static void rescue_pair(const og_index *ix, const og_params *par, const uint8_t *seq1,
                        const uint8_t *qual1, int len1, const uint8_t *seq2, const uint8_t *qual2,
                        int len2, scratch_t *sc, mate_t *m1, mate_t *m2)
{
    if ((m1->best >= 0) == (m2->best >= 0)) return;
    const mate_t *an = m1->best >= 0 ? m1 : m2;
    mate_t *tg = m1->best >= 0 ? m2 : m1;
    const uint8_t *seq = tg == m1 ? seq1 : seq2, *qual = tg == m1 ? qual1 : qual2;
    const int m = tg == m1 ? len1 : len2;
    if (tg->yf != OG_YF_NONE || m == 0) return;
    const caln_t *anchor = &an->a[an->best];
    load_codes(seq, qual, m, sc);
    const int s = 1 - anchor->strand;
    int diag = 0;
    if (!rescue_diagonal(ix, anchor, sc->codes[s], m, par->maxins, &diag)) return;
    const cand_t cd = { s, anchor->ref, diag, 0 };
    caln_t out;
    dp_extend(ix, par, sc->codes[s], sc->quals[s], m, &cd, sc->bits, sc->ops, &out);
    out.strand = s;
    if (!out.valid) return;
    tg->a[0] = out;
    tg->n = 1;
    tg->best = 0;
    tg->rescued = 1;
}

static int same_place(const caln_t *x, const caln_t *y)
{
    return x->strand == y->strand && x->ref == y->ref && x->pos == y->pos;
}

/* second best score among alignments distinct from the chosen one */
static int second_best(const mate_t *mt, int chosen, int *sec)
{
    int has = 0;
    for (int c = 0; c < mt->n; ++c) {
        if (c == chosen || !mt->a[c].valid || same_place(&mt->a[c], &mt->a[chosen])) continue;
        if (!has || mt->a[c].score > *sec) { *sec = mt->a[c].score; has = 1; }
    }
    return has;
}

static int concordant(const caln_t *x, const caln_t *y, int maxins)
{
    if (x->ref != y->ref || x->strand == y->strand) return 0;
    const caln_t *fw = x->strand == 0 ? x : y, *rv = x->strand == 0 ? y : x;
    const int lo = fw->pos < rv->pos ? fw->pos : rv->pos;
    const int hi = fw->end > rv->end ? fw->end : rv->end;
    if (hi - lo > maxins) return 0;
    if (rv->pos < fw->pos && rv->end < fw->end) return 0; /* dovetail / outie */
    return 1;
}

static void fill_aligned(og_aln *o, const caln_t *a, int mode, int m, const mate_t *mt, int chosen)
{
    o->ref = a->ref;
    o->pos = a->pos;
    o->rev = a->strand;
    o->score = a->score;
    int sec = 0;
    const int has = second_best(mt, chosen, &sec);
    o->secbest = has ? sec : INT32_MIN;
    o->mapq = og_mapq(mode, m, a->score, has, sec);
    o->xm = a->xm; o->xo = a->xo; o->xg = a->xg; o->nm = a->nm;
    o->n_cigar = a->n_cigar;
    memcpy(o->cigar, a->cigar, sizeof(uint32_t) * (size_t)a->n_cigar);
    o->sam_ref = a->ref;
    o->sam_pos = a->pos + 1;
}

static void clear_aln(og_aln *o)
{
    memset(o, 0, sizeof(*o));
    o->ref = -1;
    o->secbest = INT32_MIN;
    o->ys = INT32_MIN;
    o->rnext = -2;
    o->sam_ref = -1;
}

static void pair_up(const og_params *par, const mate_t *m1, const mate_t *m2, int len1, int len2,
                    og_aln *o1, og_aln *o2)
{
    clear_aln(o1);
    clear_aln(o2);
    o1->yf = m1->yf;
    o2->yf = m2->yf;
    int c1 = m1->best, c2 = m2->best, conc = 0;
    long best_sum = LONG_MIN;
    for (int x = 0; x < m1->n; ++x) {
        if (!m1->a[x].valid) continue;
        for (int y = 0; y < m2->n; ++y) {
            if (!m2->a[y].valid) continue;
            if (!concordant(&m1->a[x], &m2->a[y], par->maxins)) continue;
            const long s = (long)m1->a[x].score + m2->a[y].score;
            if (s > best_sum) { best_sum = s; c1 = x; c2 = y; conc = 1; }
        }
    }
    const int al1 = c1 >= 0, al2 = c2 >= 0;
    if (al1) fill_aligned(o1, &m1->a[c1], par->mode, len1, m1, c1);
    if (al2) fill_aligned(o2, &m2->a[c2], par->mode, len2, m2, c2);
    int f1 = 0x1 | 0x40, f2 = 0x1 | 0x80;
    if (conc) { f1 |= 0x2; f2 |= 0x2; }
    if (!al1) { f1 |= 0x4; f2 |= 0x8; }
    if (!al2) { f2 |= 0x4; f1 |= 0x8; }
    if (al1 && o1->rev) { f1 |= 0x10; f2 |= 0x20; }
    if (al2 && o2->rev) { f2 |= 0x10; f1 |= 0x20; }
    o1->flag = f1;
    o2->flag = f2;
    const int yt = conc ? OG_YT_CP : (al1 && al2) ? OG_YT_DP : OG_YT_UP;
    o1->yt = o2->yt = yt;
    if (al1 && al2) {
        o1->ys = o2->score;
        o2->ys = o1->score;
        if (o1->ref == o2->ref) {
            o1->rnext = o2->rnext = -1;
            const caln_t *a = &m1->a[c1], *b = &m2->a[c2];
            const int lo = a->pos < b->pos ? a->pos : b->pos;
            const int hi = a->end > b->end ? a->end : b->end;
            const int t = hi - lo;
            const int first_is_1 = a->pos <= b->pos;
            o1->tlen = first_is_1 ? t : -t;
            o2->tlen = first_is_1 ? -t : t;
        } else {
            o1->rnext = o2->ref;
            o2->rnext = o1->ref;
        }
        o1->pnext = o2->sam_pos;
        o2->pnext = o1->sam_pos;
    } else if (al1 || al2) {
        og_aln *A = al1 ? o1 : o2, *U = al1 ? o2 : o1;
        U->sam_ref = A->sam_ref;
        U->sam_pos = A->sam_pos;
        A->rnext = U->rnext = -1;
        A->pnext = A->sam_pos;
        U->pnext = A->sam_pos;
        U->ys = A->score;
    }
}

static void single_up(const og_params *par, const mate_t *mt, int len, og_aln *o)
{
    clear_aln(o);
    o->yf = mt->yf;
    o->yt = OG_YT_UU;
    if (mt->best >= 0) {
        fill_aligned(o, &mt->a[mt->best], par->mode, len, mt, mt->best);
        o->flag = o->rev ? 0x10 : 0;
    } else {
        o->flag = 0x4;
    }
}

/* per-read diagnostics (og_map_diag): why a mate did or did not align */
static void diagnose(const mate_t *mt, int32_t *d)
{
    int cause;
    if (mt->best >= 0) cause = mt->rescued ? OG_CAUSE_RESCUED : OG_CAUSE_ALIGNED;
    else if (mt->yf != OG_YF_NONE) cause = OG_CAUSE_FILTERED;
    else if (mt->n == 0) cause = OG_CAUSE_NO_CANDIDATE;
    else {
        cause = OG_CAUSE_OTHER;
        int any_score = 0, any_nceil = 0;
        for (int c = 0; c < mt->n; ++c) {
            any_score |= mt->a[c].fail == FAIL_SCORE;
            any_nceil |= mt->a[c].fail == FAIL_NCEIL;
        }
        if (any_nceil) cause = OG_CAUSE_NCEIL;
        if (any_score) cause = OG_CAUSE_SCORE_MIN;
    }
    d[0] = cause;
    d[1] = mt->n_clusters;
}

static int map_all(const og_index *ix, const og_params *par, int64_t n_reads, int paired,
                   const uint8_t *seq, const uint8_t *qual, const int64_t *offsets,
                   const int32_t *lens, og_aln *out, int nthreads, int32_t *diag)
{
    for (int64_t r = 0; r < n_reads; ++r)
        if (lens[r] < 0 || lens[r] > OG_MAXLEN) return -3;
    if (paired && (n_reads & 1)) return -3;
    const int64_t n_units = paired ? n_reads / 2 : n_reads;
#ifdef _OPENMP
    if (nthreads > 0) omp_set_num_threads(nthreads);
#pragma omp parallel
#endif
    {
        scratch_t sc;
        for (int s = 0; s < 2; ++s) {
            sc.codes[s] = malloc(OG_MAXLEN);
            sc.quals[s] = malloc(OG_MAXLEN);
        }
        sc.hits = malloc(sizeof(hit_t) * OG_MAXHITS_MATE);
        sc.bits = malloc((size_t)OG_MAXLEN * OG_BAND);
        sc.ops = malloc(2 * OG_MAXLEN + 2 * OG_BAND);
        mate_t *ma = malloc(sizeof(mate_t)), *mb = malloc(sizeof(mate_t));
#ifdef _OPENMP
#pragma omp for schedule(dynamic, 64)
#endif
        for (int64_t u = 0; u < n_units; ++u) {
            if (paired) {
                const int64_t r1 = 2 * u, r2 = 2 * u + 1;
                map_mate(ix, par, seq + offsets[r1], qual + offsets[r1], lens[r1], &sc, ma);
                map_mate(ix, par, seq + offsets[r2], qual + offsets[r2], lens[r2], &sc, mb);
                rescue_pair(ix, par, seq + offsets[r1], qual + offsets[r1], lens[r1],
                            seq + offsets[r2], qual + offsets[r2], lens[r2], &sc, ma, mb);
                pair_up(par, ma, mb, lens[r1], lens[r2], &out[r1], &out[r2]);
                if (diag) { diagnose(ma, diag + 2 * r1); diagnose(mb, diag + 2 * r2); }
            } else {
                map_mate(ix, par, seq + offsets[u], qual + offsets[u], lens[u], &sc, ma);
                single_up(par, ma, lens[u], &out[u]);
                if (diag) diagnose(ma, diag + 2 * u);
            }
        }
        for (int s = 0; s < 2; ++s) { free(sc.codes[s]); free(sc.quals[s]); }
        free(sc.hits); free(sc.bits); free(sc.ops); free(ma); free(mb);
    }
    (void)nthreads;
    return 0;
}

int og_map(const og_index *ix, const og_params *par, int64_t n_reads, int paired,
           const uint8_t *seq, const uint8_t *qual, const int64_t *offsets,
           const int32_t *lens, og_aln *out, int nthreads)
{
    return map_all(ix, par, n_reads, paired, seq, qual, offsets, lens, out, nthreads, NULL);
}

int og_map_diag(const og_index *ix, const og_params *par, int64_t n_reads, int paired,
                const uint8_t *seq, const uint8_t *qual, const int64_t *offsets,
                const int32_t *lens, og_aln *out, int nthreads, int32_t *diag)
{
    return map_all(ix, par, n_reads, paired, seq, qual, offsets, lens, out, nthreads, diag);
}

/* ------------------------------------------------------------------ */
/* SAM-orientation rows of the mapped reads for og_pileup (what temp.sam */
/* holds after a pass): sequence printed as upper-case ACGT / N, reverse  */
/* complemented with the qualities reversed when the read aligned to the  */
/* reverse strand.  The row layout is og_pileup.c's og_row.  Used by the  */
/* CPU baseline (oracle/cpu_pipeline.py) to keep Python out of its timed  */
/* region.                                                                */
/* ------------------------------------------------------------------ */
typedef struct {
    int32_t flag, ref, pos, n_cigar;
    const uint32_t *cigar;
    int32_t len;
    const char *seq, *qual;
} og_row_view;

int og_rows_from_alns(const og_aln *alns, int64_t n, const uint8_t *seq, const uint8_t *qual,
                      const int64_t *offsets, const int32_t *lens, char *seq_out,
                      char *qual_out, og_row_view *rows, int nthreads)
{
#ifdef _OPENMP
#pragma omp parallel for schedule(static) num_threads(nthreads > 0 ? nthreads : 1)
#endif
    for (int64_t i = 0; i < n; ++i) {
        const og_aln *a = &alns[i];
        const int m = lens[i];
        const uint8_t *s = seq + offsets[i], *q = qual + offsets[i];
        char *so = seq_out + offsets[i], *qo = qual_out + offsets[i];
        const int rev = a->ref >= 0 && a->rev;
        for (int k = 0; k < m; ++k) {
            const int src = rev ? m - 1 - k : k;
            const uint8_t c = base_code(s[src]);
            so[k] = c > 3 ? 'N' : "ACGT"[rev ? 3 - c : c];
            qo[k] = (char)q[src];
        }
        og_row_view *r = &rows[i];
        r->flag = a->flag;
        r->ref = a->sam_ref;
        r->pos = a->sam_pos;
        r->n_cigar = a->ref >= 0 && !(a->flag & 4) ? a->n_cigar : 0;
        r->cigar = a->cigar;
        r->len = m;
        r->seq = so;
        r->qual = qo;
    }
    return 0;
}
