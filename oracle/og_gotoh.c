/*
 * oracle/og_gotoh.c -- TEST INFRASTRUCTURE ONLY.
 *
 * CPU restatement of the reference's affine-gap Gotoh aligner
 * (micall/alignment/src/_gotoh2.c), written from the algorithm, used only by
 * tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg as the
 * checker for the HIP kernel in micall-lite_amd/csrc/mh_gotoh.hip.  Nothing in
 * the product links or loads this file.
 *
 * Pinned against: the reference extension compiled from its own source by
 * oracle/Makefile into oracle/_ref/ (tests/golden/gotoh_golden.json is
 * generated from it by tests/golden/gen_golden.py), and the reference KATs in
 * micall/alignment/tests/test.py:174-286.
 *
 * Algorithm (reference file:line in _gotoh2.c):
 *   - cost-minimising matrices R (best), P (vertical: consume seq1 only),
 *     Q (horizontal: consume seq2 only), initialize :93-132,
 *     cost_assignment :137-201;
 *   - seven tie bits per cell (a=R from P, b=R from Q, c=R from diagonal,
 *     d/e = P extend/open, f/g = Q extend/open) :150-198;
 *   - Altschul-Erickson edge assignment, steps 8-11, reverse sweep :205-313;
 *   - traceback preferring a > b > c, ends-free ("local") start = first
 *     strict minimum over the last column then the last row :316-438;
 *   - score = -min cost :437.
 * Non-alphabet characters are rejected (status -3) instead of indexing the
 * score matrix out of bounds as the reference would (_gotoh2.c:87, :185).
 */
#include <limits.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#define OG_INF INT_MAX

enum { BIT_A = 1, BIT_B = 2, BIT_C = 4, BIT_D = 8, BIT_E = 16, BIT_F = 32, BIT_G = 64 };

static int imin(int x, int y) { return x <= y ? x : y; }
/* An infinite predecessor never satisfies the reference's (overflowing)
 * extend test, _gotoh2.c:157,167: checked explicitly below. */

int og_gotoh_align(const char *s1, const char *s2, int gop, int gep, int is_global,
                   const char *alphabet, const int *matrix,
                   char *out1, char *out2, int cap, int *score)
{
    const int m = (int)strlen(s1), n = (int)strlen(s2);
    const int L = (int)strlen(alphabet);
    if (m == 0 || n == 0 || L == 0 || cap < m + n + 1) return -3;

    int code[256];
    for (int k = 0; k < 256; ++k) code[k] = -1;
    for (int k = 0; k < L; ++k) code[(unsigned char)alphabet[k]] = k;

    /* The costs are kept two rows at a time (rows i-1 and i of R and P, row
     * i of Q) plus R's last column: the traceback reads R only there and on
     * the last row.  The bit matrix is the one full (m+2)x(n+2) array, one
     * byte per cell, so a 30 kb x 30 kb alignment (C4-all's SARS-CoV-2
     * consensus against its seed) needs 0.9 GB instead of 12. */
    const size_t W = (size_t)n + 1, BW = (size_t)n + 2;
    int *a = malloc(sizeof(int) * (size_t)m), *b = malloc(sizeof(int) * (size_t)n);
    int *R0 = malloc(sizeof(int) * W), *R1 = malloc(sizeof(int) * W),
        *P0 = malloc(sizeof(int) * W), *P1 = malloc(sizeof(int) * W),
        *Q = malloc(sizeof(int) * W), *Rcol = malloc(sizeof(int) * ((size_t)m + 1));
    uint8_t *bt = calloc((size_t)(m + 2) * BW, 1);
    char *r1 = malloc((size_t)m + n + 1), *r2 = malloc((size_t)m + n + 1);
    int status = 0;
    if (!a || !b || !R0 || !R1 || !P0 || !P1 || !Q || !Rcol || !bt || !r1 || !r2) { status = -2; goto done; }

    for (int i = 0; i < m; ++i) if ((a[i] = code[(unsigned char)s1[i]]) < 0) { status = -3; goto done; }
    for (int j = 0; j < n; ++j) if ((b[j] = code[(unsigned char)s2[j]]) < 0) { status = -3; goto done; }

#define BX(i, j) ((size_t)(i) * BW + (size_t)(j))
    const int u = gep, v = gop;

    /* ---- cost assignment (row-major, same visiting order as :142-143);
     * Rp/Pp: row i-1, Rc/Pc: row i ---- */
    int *Rp = R0, *Rc = R1, *Pp = P0, *Pc = P1;
    for (int i = 0; i <= m; ++i) {
        for (int j = 0; j <= n; ++j) {
            int p, q, r;
            /* P: vertical gap, from the cell above */
            if (i == 0) {
                p = OG_INF;
            } else {
                const int pu = Pp[j], ru = Rp[j];
                p = u + imin(pu, ru + v);
                if (pu != OG_INF && p == pu + u) bt[BX(i - 1, j)] |= BIT_D;
                if (p == ru + v + u) bt[BX(i - 1, j)] |= BIT_E;
            }
            /* Q: horizontal gap, from the cell to the left */
            if (j == 0) {
                q = OG_INF;
            } else {
                const int ql = Q[j - 1], rl = Rc[j - 1];
                q = u + imin(ql, rl + v);
                if (ql != OG_INF && q == ql + u) bt[BX(i, j - 1)] |= BIT_F;
                if (q == rl + v + u) bt[BX(i, j - 1)] |= BIT_G;
            }
            int dg = 0;
            if (i == 0 && j == 0) {
                r = 0;
            } else if (i == 0 || j == 0) {
                r = is_global ? imin(p, q) : 0; /* borders: v+u*k global, 0 ends-free */
            } else {
                dg = Rp[j - 1] - matrix[a[i - 1] * L + b[j - 1]];
                r = imin(imin(dg, p), q);
            }
            Pc[j] = p; Q[j] = q; Rc[j] = r;
            if (r == p) bt[BX(i, j)] |= BIT_A;
            if (r == q) bt[BX(i, j)] |= BIT_B;
            if (i > 0 && j > 0 && r == dg) bt[BX(i, j)] |= BIT_C;
        }
        Rcol[i] = Rc[n];
        int *t = Rp; Rp = Rc; Rc = t;
        t = Pp; Pp = Pc; Pc = t;
    }
    const int *Rlast = Rp;   /* row m after the final swap */

    /* ---- boundary bits of the (m+2)x(n+2) bit matrix (:117-131) ---- */
    if (!is_global) {
        for (int j = 0; j <= n + 1; ++j) bt[BX(m + 1, j)] = BIT_C;
        for (int i = 0; i <= m + 1; ++i) bt[BX(i, n + 1)] = BIT_C;
    }
    bt[BX(m + 1, n + 1)] = BIT_C;

    /* ---- edge assignment, Altschul-Erickson steps 8-11 (:205-313) ---- */
    for (int i = m; i >= 0; --i) {
        for (int j = n; j >= 0; --j) {
            uint8_t *h = &bt[BX(i, j)];
            uint8_t *dn = &bt[BX(i + 1, j)], *rt = &bt[BX(i, j + 1)];
            const uint8_t dgb = bt[BX(i + 1, j + 1)];
            const int no_a_below = !(*dn & BIT_A), no_e = !(*h & BIT_E);
            const int no_b_right = !(*rt & BIT_B), no_g = !(*h & BIT_G);
            const int no_c_diag = !(dgb & BIT_C);
            if ((no_a_below || no_e) && (no_b_right || no_g) && no_c_diag)
                *h &= (uint8_t)~(BIT_A | BIT_B | BIT_C);          /* step 8 */
            if (no_a_below && no_b_right && no_c_diag) continue;   /* step 9 */
            if ((*dn & BIT_A) && (*h & BIT_D)) {                    /* step 10 */
                if (*h & BIT_E) *dn &= (uint8_t)~BIT_D; else *dn |= BIT_D;
                if (*h & BIT_A) *h &= (uint8_t)~BIT_E; else *h |= BIT_E;
                *h |= BIT_A;
            } else {
                *dn &= (uint8_t)~BIT_D;
                *h &= (uint8_t)~BIT_E;
            }
            if ((*rt & BIT_B) && (*h & BIT_F)) {                    /* step 11 */
                if (*h & BIT_G) *rt &= (uint8_t)~BIT_F; else *rt |= BIT_F;
                if (*h & BIT_B) *h &= (uint8_t)~BIT_G; else *h |= BIT_G;
                *h |= BIT_B;
            } else {
                *rt &= (uint8_t)~BIT_F;
                *h &= (uint8_t)~BIT_G;
            }
        }
    }

    /* ---- traceback (:316-438) ---- */
    {
        int ii = m, jj = n, best = Rlast[n];
        if (!is_global) {
            for (int i = 0; i <= m; ++i) if (Rcol[i] < best) { best = Rcol[i]; ii = i; jj = n; }
            for (int j = 0; j <= n; ++j) if (Rlast[j] < best) { best = Rlast[j]; ii = m; jj = j; }
        }
        int len = 0; /* built back to front in r1/r2 */
        if (ii < m) for (int k = m - 1; k >= ii; --k) { r1[len] = s1[k]; r2[len] = '-'; ++len; }
        if (jj < n) for (int k = n - 1; k >= jj; --k) { r1[len] = '-'; r2[len] = s2[k]; ++len; }
        while (ii > 0 && jj > 0) {
            const uint8_t x = bt[BX(ii, jj)];
            if (x & BIT_A)      { r1[len] = s1[ii - 1]; r2[len] = '-'; --ii; }
            else if (x & BIT_B) { r1[len] = '-'; r2[len] = s2[jj - 1]; --jj; }
            else if (x & BIT_C) { r1[len] = s1[ii - 1]; r2[len] = s2[jj - 1]; --ii; --jj; }
            else { status = -1; goto done; }
            ++len;
        }
        while (ii > 0) { r1[len] = s1[ii - 1]; r2[len] = '-'; --ii; ++len; }
        while (jj > 0) { r1[len] = '-'; r2[len] = s2[jj - 1]; --jj; ++len; }
        for (int k = 0; k < len; ++k) { out1[k] = r1[len - 1 - k]; out2[k] = r2[len - 1 - k]; }
        out1[len] = out2[len] = '\0';
        *score = -best;
    }
#undef BX
done:
    free(a); free(b); free(R0); free(R1); free(P0); free(P1); free(Q); free(Rcol); free(bt);
    free(r1); free(r2);
    return status;
}

/* Unit-cost edit distance (stand-in for python-Levenshtein's
 * Levenshtein.distance used at remap.py:250; that module is not installed). */
int og_levenshtein(const char *x, const char *y)
{
    const int m = (int)strlen(x), n = (int)strlen(y);
    int *row = malloc(sizeof(int) * (size_t)(n + 1));
    if (!row) return -2;
    for (int j = 0; j <= n; ++j) row[j] = j;
    for (int i = 1; i <= m; ++i) {
        int diag = row[0];
        row[0] = i;
        for (int j = 1; j <= n; ++j) {
            const int up = row[j];
            int best = diag + (x[i - 1] != y[j - 1]);
            if (up + 1 < best) best = up + 1;
            if (row[j - 1] + 1 < best) best = row[j - 1] + 1;
            row[j] = best;
            diag = up;
        }
    }
    const int d = row[n];
    free(row);
    return d;
}
