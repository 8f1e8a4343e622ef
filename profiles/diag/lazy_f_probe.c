/* lazy_f_probe.c -- diagnostics only: linked with the oracle mapper built
 * with -DOG_ROW_PROBE (profiles/diag/lazy_f_probe.py), it counts, over every
 * gapped DP row of dp_extend, what a lazy deletion move in k_dp could skip.
 *
 * k_dp's deletion move (mh_map.hip dp_row_gap) is the prefix max P of the
 * shifted row x(k) = H1(k) + exD k (scan_max: four DPP row shifts and one
 * row_bcast), then F(k) = P(k - 1) - (oeD - exD), H = max(H1, F), and the
 * traceback bit fb'(k) = x(k) < P(k).  Counted per row:
 *   mono      x non-decreasing: P == x, every fb' bit 0, F never wins --
 *             the rows a one-step test (x(k-1) <= x(k) on every lane) could
 *             skip exactly;
 *   fwin      some lane has F > H1 (the deletion move changes H);
 *   gate1     no lane's gap-of-one F wins (H1(k-1) - oeD <= H1(k)): the
 *             one-step "F cannot win" test;
 *   gate1_bad gate1 holds but a longer gap still wins (the one-step test is
 *             not exact);
 *   fb_live   some lane has fb' = 1 (x(k) < P(k)): the bits a skipped row
 *             would have to reproduce wherever the traceback can read them. */
#include <stdint.h>

static uint64_t n_rows, n_mono, n_fwin, n_gate1, n_gate1_bad, n_fb_live, n_lanes, n_lanes_fwin;

static void add(uint64_t *c, uint64_t v) { __atomic_fetch_add(c, v, __ATOMIC_RELAXED); }

void og_row_probe(int W, const int *H1, const int *H, int oeD, int exD)
{
    int mono = 1, fwin = 0, gate1 = 1, fb_live = 0, lanes_fwin = 0;
    int64_t P = (int64_t)H1[0];
    for (int k = 1; k < W; ++k) {
        const int64_t x = (int64_t)H1[k] + (int64_t)exD * k;
        const int64_t xp = (int64_t)H1[k - 1] + (int64_t)exD * (k - 1);
        if (x < xp) mono = 0;
        if (H1[k - 1] - oeD > H1[k]) gate1 = 0;
        if (x < P) fb_live = 1;
        if (x > P) P = x;
        if (H[k] > H1[k]) { fwin = 1; ++lanes_fwin; }
    }
    add(&n_rows, 1);
    add(&n_lanes, (uint64_t)(W - 1));
    add(&n_lanes_fwin, (uint64_t)lanes_fwin);
    if (mono) add(&n_mono, 1);
    if (fwin) add(&n_fwin, 1);
    if (gate1) add(&n_gate1, 1);
    if (gate1 && fwin) add(&n_gate1_bad, 1);
    if (fb_live) add(&n_fb_live, 1);
}

void og_row_probe_get(uint64_t *out8)
{
    out8[0] = n_rows;
    out8[1] = n_mono;
    out8[2] = n_fwin;
    out8[3] = n_gate1;
    out8[4] = n_gate1_bad;
    out8[5] = n_fb_live;
    out8[6] = n_lanes;
    out8[7] = n_lanes_fwin;
}

void og_row_probe_reset(void)
{
    n_rows = n_mono = n_fwin = n_gate1 = n_gate1_bad = n_fb_live = n_lanes = n_lanes_fwin = 0;
}
