// mh_gotoh.hip -- the _gotoh2 aligner (micall/alignment/src/_gotoh2.c) on
// gfx950, used by the consensus-distance filter (remap.py:244-263: global,
// gop 15, gep 3, HYPHY_NUC) and aln2counts' coordinate mapping (local,
// EmpHIV25).  A batch of alignments is one launch, one workgroup of 1024
// threads per alignment (blockIdx.x = alignment), each with its own scratch:
//   phase 1  cost assignment (_gotoh2.c:137-201) by anti-diagonals; R/P/Q
//            live in three rolling diagonal buffers in LDS (with both
//            sequences' codes and the score matrix; in global memory when a
//            sequence is too long for LDS); each cell's tie bits go to three
//            byte planes so no two cells of a diagonal write the same byte:
//            abc(i,j) by (i,j), de(i,j) by (i+1,j), fg(i,j) by (i,j+1)
//   phase 2  Altschul-Erickson edge assignment (:205-313) by anti-diagonals
//            in reverse; its writes to d(i+1,j) and f(i,j+1) are never read
//            again (each cell reads its own d/f before its upper/left
//            neighbour runs) and are dropped
//   phase 3  traceback (:316-438) by one thread.
// The planes are stored anti-diagonal-major over the (m+2) x (n+2) grid
// (doff[s] = first byte of diagonal s, cells by row i): the cells a
// diagonal step touches are consecutive bytes, so every plane access of a
// step is coalesced (row-major planes put each thread on its own cache line).
// Bit-for-bit specification: oracle/og_gotoh.c.
#include <limits.h>

#include <mutex>
#include <vector>

#include "mh_internal.h"

namespace mh {

constexpr int G_INF = INT_MAX;
enum { GA = 1, GB = 2, GC = 4, GD = 8, GE_ = 16, GF = 32, GG = 64 };
constexpr int GOTOH_THREADS = 1024;
constexpr size_t GOTOH_LDS_MAX = 160 * 1024 - 256;   // (the traceback's static LDS)
constexpr int GOTOH_PF = 4;   // LDS variant: cells per thread per diagonal (m < GOTOH_PF * 1024)

// LDS variant layout: R/P/Q rolling diagonals 9 (m+2) ints, the L x L
// matrix, seq1 codes, seq2 codes; phase 2 reuses the R/P/Q space for the
// final abc of 3 diagonals
__host__ __device__ inline size_t gotoh_al16(size_t x) { return (x + 15) & ~(size_t)15; }
__host__ __device__ inline size_t gotoh_codes_end(int m, int n, int L)
{
    return sizeof(int) * (9 * (size_t)(m + 2) + (size_t)L * L) + gotoh_al16(m) + gotoh_al16(n);
}
constexpr int TB = 128;                                // traceback window (diagonals x rows)
constexpr size_t TB_LDS = (size_t)TB * TB + 2 * TB;   // window + both sequences' characters

struct GotohArgs {
    const int8_t *a;      // seq1 codes, m
    const int8_t *b;      // seq2 codes, n
    int m, n, L;
    const int *mat;       // L x L
    int u, v, is_global;
    int *diagR, *diagP, *diagQ;   // 3 x (m + 2) each (global variant)
    int *lastcol, *lastrow;       // R(i, n), R(m, j)
    uint8_t *abc, *de, *fg;       // (m+2) x (n+2), anti-diagonal-major
    const char *s1, *s2;
    char *out1, *out2;            // m + n + 1
    int *result;                  // [0] status, [1] score, [2] length
};

__device__ __forceinline__ int gmin(int x, int y) { return x <= y ? x : y; }

// A workgroup barrier that orders LDS only.  __syncthreads() is also a
// workgroup release fence for global memory, so every wave would wait for
// its plane stores (and prefetch loads) to land at each anti-diagonal step;
// the steps of the LDS variant never read back a global value written by
// another step, so they only need the LDS ordering.
__device__ __forceinline__ void lds_barrier()
{
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
}

template <bool LDS>
__device__ __forceinline__ void step_barrier()
{
    if (LDS) lds_barrier();
    else __syncthreads();   // rolling diagonals in global memory
}

// First plane byte of anti-diagonal s of the (M+1) x (N+1) grid (M = m+1,
// N = n+1): the sum of len(t) = min(t, M) - max(0, t - N) + 1 over t < s.
__host__ __device__ __forceinline__ int64_t doff_of(int64_t s, int64_t M, int64_t N)
{
    const int64_t s1 = s <= M + 1 ? s * (s - 1) / 2 : M * (M + 1) / 2 + (s - 1 - M) * M;
    const int64_t s2 = s <= N + 1 ? 0 : (s - 1 - N) * (s - N) / 2;
    return s + s1 - s2;
}

// plane base of diagonal s, indexed by row i: diagonal s starts at row
// max(0, s - (n+1))
__device__ __forceinline__ int64_t dbase(int s, int m, int n)
{
    const int lo = s - (n + 1) > 0 ? s - (n + 1) : 0;
    return doff_of(s, m + 1, n + 1) - lo;
}

__device__ __forceinline__ size_t pidx(const GotohArgs &A, int i, int j)
{
    return (size_t)(dbase(i + j, A.m, A.n) + i);
}

template <bool LDS>
__global__ __launch_bounds__(GOTOH_THREADS) void k_gotoh(const GotohArgs *batch)
{
    extern __shared__ __attribute__((aligned(16))) unsigned char gsm[];
    const GotohArgs A = batch[blockIdx.x];
    const int m = A.m, n = A.n, L = A.L;
    const int u = A.u, v = A.v;
    int *dR = A.diagR, *dP = A.diagP, *dQ = A.diagQ;
    const int8_t *ca = A.a, *cb = A.b;
    const int *mat = A.mat;
    if (LDS) {   // rolling diagonals, codes and matrix in LDS
        int *w = (int *)gsm;
        dR = w;
        dP = w + 3 * (m + 2);
        dQ = w + 6 * (m + 2);
        int *lm = w + 9 * (m + 2);
        int8_t *la = (int8_t *)(lm + L * L), *lb = la + gotoh_al16(m);
        for (int x = threadIdx.x; x < L * L; x += blockDim.x) lm[x] = A.mat[x];
        for (int x = threadIdx.x; x < m; x += blockDim.x) la[x] = A.a[x];
        for (int x = threadIdx.x; x < n; x += blockDim.x) lb[x] = A.b[x];
        mat = lm; ca = la; cb = lb;
        __syncthreads();
    }
    // ---- phase 1: cost assignment by anti-diagonals ----
    for (int s = 0; s <= m + n; ++s) {
        const int ilo = s - n > 0 ? s - n : 0, ihi = s < m ? s : m;
        int *Rc = dR + (s % 3) * (m + 2), *Pc = dP + (s % 3) * (m + 2), *Qc = dQ + (s % 3) * (m + 2);
        const int *R1 = dR + ((s + 2) % 3) * (m + 2), *P1 = dP + ((s + 2) % 3) * (m + 2),
                  *Q1 = dQ + ((s + 2) % 3) * (m + 2);
        const int *R2 = dR + ((s + 1) % 3) * (m + 2);
        // plane bases of diagonals s and s - 1 (wave-uniform arithmetic)
        uint8_t *abc0 = A.abc + dbase(s, m, n);
        uint8_t *de1 = A.de + dbase(s - 1, m, n);
        uint8_t *fg1 = A.fg + dbase(s - 1, m, n);
        for (int i = ilo + (int)threadIdx.x; i <= ihi; i += blockDim.x) {
            const int j = s - i;
            int p, q, r, dg = 0;
            if (i == 0) {
                p = G_INF;
            } else {
                const int pu = P1[i - 1], ru = R1[i - 1];   // (i-1, j) on diagonal s-1
                p = u + gmin(pu, ru + v);
                uint8_t de = 0;
                if (pu != G_INF && p == pu + u) de |= GD;
                if (p == ru + v + u) de |= GE_;
                de1[i - 1] = de;                            // de(i-1, j)
            }
            if (j == 0) {
                q = G_INF;
            } else {
                const int ql = Q1[i], rl = R1[i];           // (i, j-1) on diagonal s-1
                q = u + gmin(ql, rl + v);
                uint8_t fg = 0;
                if (ql != G_INF && q == ql + u) fg |= GF;
                if (q == rl + v + u) fg |= GG;
                fg1[i] = fg;                                // fg(i, j-1)
            }
            if (i == 0 && j == 0) {
                r = 0;
            } else if (i == 0 || j == 0) {
                r = A.is_global ? gmin(p, q) : 0;
            } else {
                dg = R2[i - 1] - mat[ca[i - 1] * L + cb[j - 1]];
                r = gmin(gmin(dg, p), q);
            }
            Rc[i] = r; Pc[i] = p; Qc[i] = q;
            uint8_t abc = 0;
            if (r == p) abc |= GA;
            if (r == q) abc |= GB;
            if (i > 0 && j > 0 && r == dg) abc |= GC;
            abc0[i] = abc;
            if (j == n) A.lastcol[i] = r;
            if (i == m) A.lastrow[j] = r;
        }
        step_barrier<LDS>();
    }
    // boundary c bits (_gotoh2.c:117-131)
    if (!A.is_global) {
        for (int j = threadIdx.x; j <= n + 1; j += blockDim.x) A.abc[pidx(A, m + 1, j)] = GC;
        for (int i = threadIdx.x; i <= m + 1; i += blockDim.x) A.abc[pidx(A, i, n + 1)] = GC;
    }
    if (threadIdx.x == 0) A.abc[pidx(A, m + 1, n + 1)] = GC;
    __syncthreads();
    // ---- phase 2: edge assignment, anti-diagonals in reverse ----
    // A cell reads its own phase-1 bytes and the final abc of (i+1, j),
    // (i, j+1) (diagonal s+1) and (i+1, j+1) (s+2).  The LDS variant keeps
    // those final values of the last two diagonals in LDS and loads the next
    // diagonal's phase-1 bytes while this one is computed, so a step waits on
    // no global load.  Boundary cells (i = m+1 or j = n+1) hold GC in local
    // mode, 0 in global mode, GC at (m+1, n+1).
    const uint8_t bnd = A.is_global ? 0 : GC;
    auto edge = [&](uint8_t x, uint8_t dep, uint8_t fgp, uint8_t dn, uint8_t rt, uint8_t dgn) -> uint8_t {
        uint8_t e = dep & GE_, d = dep & GD;
        uint8_t g = fgp & GG, f = fgp & GF;
        const bool no_a_below = !(dn & GA), no_e = !e, no_b_right = !(rt & GB), no_g = !g;
        const bool no_c_diag = !(dgn & GC);
        if ((no_a_below || no_e) && (no_b_right || no_g) && no_c_diag) x &= (uint8_t)~(GA | GB | GC);
        if (!(no_a_below && no_b_right && no_c_diag)) {
            if ((dn & GA) && d) x |= GA;
            if ((rt & GB) && f) x |= GB;
        }
        return x;
    };
    if (LDS) {
        uint8_t *fin = (uint8_t *)gsm;   // 3 x (m + 2): final abc by row (phase 1's R/P/Q space)
        uint8_t px[GOTOH_PF], pd[GOTOH_PF], pf[GOTOH_PF];
        auto fetch = [&](int sd) {
            const int ilo = sd - n > 0 ? sd - n : 0, ihi = sd < m ? sd : m;
            const int64_t b0 = dbase(sd, m, n);
#pragma unroll
            for (int k = 0; k < GOTOH_PF; ++k) {
                const int i = ilo + (int)threadIdx.x + k * GOTOH_THREADS;
                if (i <= ihi) {
                    px[k] = A.abc[b0 + i];
                    pd[k] = A.de[b0 + i];
                    pf[k] = A.fg[b0 + i];
                }
            }
        };
        fetch(m + n);
        for (int s = m + n; s >= 0; --s) {
            const int ilo = s - n > 0 ? s - n : 0, ihi = s < m ? s : m;
            const int64_t b0 = dbase(s, m, n);
            uint8_t cx[GOTOH_PF], cd[GOTOH_PF], cf[GOTOH_PF];
#pragma unroll
            for (int k = 0; k < GOTOH_PF; ++k) { cx[k] = px[k]; cd[k] = pd[k]; cf[k] = pf[k]; }
            if (s > 0) fetch(s - 1);
            uint8_t *f0 = fin + (s % 3) * (m + 2);
            const uint8_t *f1 = fin + ((s + 1) % 3) * (m + 2), *f2 = fin + ((s + 2) % 3) * (m + 2);
#pragma unroll
            for (int k = 0; k < GOTOH_PF; ++k) {
                const int i = ilo + (int)threadIdx.x + k * GOTOH_THREADS;
                if (i > ihi) break;
                const int j = s - i;
                const bool lastr = i == m, lastc = j == n;
                const uint8_t dn = lastr ? (lastc ? GC : bnd) : f1[i + 1];
                const uint8_t rt = lastc ? (lastr ? GC : bnd) : f1[i];
                const uint8_t dgn = (lastr || lastc) ? ((lastr && lastc) ? GC : bnd) : f2[i + 1];
                const uint8_t x = edge(cx[k], cd[k], cf[k], dn, rt, dgn);
                A.abc[b0 + i] = x;
                f0[i] = x;
            }
            lds_barrier();
        }
        __syncthreads();   // the traceback reads the planes
    } else {
        for (int s = m + n; s >= 0; --s) {
            const int ilo = s - n > 0 ? s - n : 0, ihi = s < m ? s : m;
            const int64_t b0 = dbase(s, m, n), b1 = dbase(s + 1, m, n), b2 = dbase(s + 2, m, n);
            for (int i = ilo + (int)threadIdx.x; i <= ihi; i += blockDim.x) {
                const int64_t h = b0 + i;
                // (i+1, j) and (i, j+1) on diagonal s+1, (i+1, j+1) on s+2
                A.abc[h] = edge(A.abc[h], A.de[h], A.fg[h], A.abc[b1 + i + 1], A.abc[b1 + i],
                                A.abc[b2 + i + 1]);
            }
            __syncthreads();
        }
    }
    // ---- phase 3: traceback ----
    // The walk is serial, so it never waits on global memory: the block
    // stages a TB x TB window of abc (diagonals s0 .. s0-TB+1, rows
    // ii .. ii-TB+1 of the current cell (ii, jj), which holds every cell the
    // path can reach before it leaves the window) and the TB characters of
    // each sequence before ii / jj into LDS; thread 0 walks the window and
    // writes the output characters; repeat.  The gap runs at both ends are
    // written by the whole block.
    uint8_t *win = (uint8_t *)gsm + (LDS ? gotoh_codes_end(m, n, L) : 0);
    char *wc1 = (char *)win + TB * TB, *wc2 = wc1 + TB;
    __shared__ unsigned long long tb_key;
    __shared__ int tb_ii, tb_jj, tb_len, tb_status;
    if (threadIdx.x == 0) tb_key = ~0ull;
    __syncthreads();
    if (!A.is_global) {
        // the first strict minimum in the reference's scan order: R(m, n),
        // then R(i, n) for i = 0..m, then R(m, j) for j = 0..n
        unsigned long long k = ~0ull;
        for (int x = threadIdx.x; x < m + n + 3; x += blockDim.x) {
            const int val = x == 0 ? A.lastrow[n] : (x <= m + 1 ? A.lastcol[x - 1] : A.lastrow[x - m - 2]);
            const unsigned long long kk = ((unsigned long long)((uint32_t)val ^ 0x80000000u) << 32) | (uint32_t)x;
            k = kk < k ? kk : k;
        }
        atomicMin(&tb_key, k);
        __syncthreads();
    }
    int ii = m, jj = n, best = A.lastrow[n];
    if (!A.is_global) {
        const int x = (int)(tb_key & 0xffffffffu);
        best = (int)((uint32_t)(tb_key >> 32) ^ 0x80000000u);
        if (x >= 1 && x <= m + 1) { ii = x - 1; jj = n; }
        else if (x > m + 1) { ii = m; jj = x - m - 2; }
    }
    char *r1 = A.out1, *r2 = A.out2;   // built back to front, reversed by the host
    // end gaps: seq1 past ii, then seq2 past jj
    for (int x = threadIdx.x; x < m - ii; x += blockDim.x) { r1[x] = A.s1[m - 1 - x]; r2[x] = '-'; }
    for (int x = threadIdx.x; x < n - jj; x += blockDim.x) {
        r1[m - ii + x] = '-';
        r2[m - ii + x] = A.s2[n - 1 - x];
    }
    if (threadIdx.x == 0) { tb_ii = ii; tb_jj = jj; tb_len = (m - ii) + (n - jj); tb_status = 0; }
    __syncthreads();
    for (;;) {
        const int i0 = tb_ii, j0 = tb_jj;
        if (i0 <= 0 || j0 <= 0 || tb_status) break;
        const int s0 = i0 + j0;
        for (int x = threadIdx.x; x < TB * TB; x += blockDim.x) {
            const int t = x / TB, r = x % TB;
            const int sd = s0 - t, i = i0 - r, j = sd - i;
            uint8_t v = 0;
            if (i >= 1 && j >= 1 && j <= n) v = A.abc[dbase(sd, m, n) + i];   // (r <= t on the path)
            win[x] = v;
        }
        for (int x = threadIdx.x; x < TB; x += blockDim.x) {
            wc1[x] = i0 - 1 - x >= 0 ? A.s1[i0 - 1 - x] : 0;
            wc2[x] = j0 - 1 - x >= 0 ? A.s2[j0 - 1 - x] : 0;
        }
        __syncthreads();
        if (threadIdx.x == 0) {
            int i = i0, j = j0, len = tb_len, status = 0;
            while (i > 0 && j > 0) {
                const int t = s0 - (i + j), r = i0 - i, c = j0 - j;
                if (t >= TB || r >= TB || c >= TB) break;
                const uint8_t x = win[t * TB + r];
                if (x & GA) { r1[len] = wc1[r]; r2[len] = '-'; --i; }
                else if (x & GB) { r1[len] = '-'; r2[len] = wc2[c]; --j; }
                else if (x & GC) { r1[len] = wc1[r]; r2[len] = wc2[c]; --i; --j; }
                else { status = -1; break; }
                ++len;
            }
            tb_ii = i; tb_jj = j; tb_len = len; tb_status = status;
        }
        __syncthreads();
    }
    // start gaps: what is left of seq1, then of seq2
    const int fi = tb_ii, fj = tb_jj, flen = tb_len, status = tb_status;
    if (status == 0) {
        for (int x = threadIdx.x; x < fi; x += blockDim.x) { r1[flen + x] = A.s1[fi - 1 - x]; r2[flen + x] = '-'; }
        for (int x = threadIdx.x; x < fj; x += blockDim.x) {
            r1[flen + fi + x] = '-';
            r2[flen + fi + x] = A.s2[fj - 1 - x];
        }
    }
    if (threadIdx.x == 0) {
        A.result[0] = status;
        A.result[1] = -best;
        A.result[2] = status == 0 ? flen + fi + fj : flen;
    }
}

static size_t align16(size_t x) { return (x + 15) & ~(size_t)15; }

// Per alignment: an "io" block (codes, strings, output strings, result: what
// crosses PCIe) and a "work" block (diagonal buffers, last row / column and
// the three tie planes, zeroed on the device).
static size_t gotoh_io_bytes(int m, int n)
{
    return align16(m + 8) + align16(n + 8) + align16(m + 1) + align16(n + 1) +
           2 * align16(m + n + 1) + 64;
}

// LDS of the LDS variant: rolling R/P/Q diagonals, the score matrix, codes
static size_t gotoh_lds_bytes(int m, int n, int L)
{
    return gotoh_codes_end(m, n, L) + TB_LDS;
}

static size_t gotoh_work_bytes(int m, int n)
{
    return 3 * align16(sizeof(int) * 3 * (m + 2)) + align16(sizeof(int) * (m + 2)) +
           align16(sizeof(int) * (n + 2)) + 3 * align16((size_t)(m + 2) * (n + 2));
}

// Retained scratch above this is released after the call (one very long
// alignment must not pin device memory for the rest of the session).
constexpr size_t GOTOH_KEEP_BYTES = (size_t)1 << 30;

int run_gotoh_batch(Ctx &c, int count, const char *const *s1, const char *const *s2, int gop,
                    int gep, int is_global, const char *alphabet, const int *matrix,
                    char *const *out1, char *const *out2, const int *cap, int *score, int *status)
{
    const int L = (int)strlen(alphabet);
    if (count < 0 || L == 0) { set_error("mh_gotoh_align: bad arguments"); return -3; }
    if (count == 0) return 0;
    int code[256];
    for (int k = 0; k < 256; ++k) code[k] = -1;
    for (int k = 0; k < L; ++k) code[(unsigned char)alphabet[k]] = k;
    std::vector<int> ms(count), ns(count);
    size_t lds = 0;
    std::vector<size_t> io(count + 1, 0), work(count + 1, 0);
    for (int t = 0; t < count; ++t) {
        if (!s1[t] || !s2[t] || !out1[t] || !out2[t]) { set_error("mh_gotoh_align: null argument"); return -3; }
        ms[t] = (int)strlen(s1[t]);
        ns[t] = (int)strlen(s2[t]);
        if (ms[t] == 0 || ns[t] == 0 || cap[t] < ms[t] + ns[t] + 1) {
            set_error("mh_gotoh_align: bad arguments (alignment %d)", t);
            return -3;
        }
        for (int i = 0; i < ms[t]; ++i)
            if (code[(unsigned char)s1[t][i]] < 0) { set_error("mh_gotoh_align: '%c' not in alphabet", s1[t][i]); return -3; }
        for (int j = 0; j < ns[t]; ++j)
            if (code[(unsigned char)s2[t][j]] < 0) { set_error("mh_gotoh_align: '%c' not in alphabet", s2[t][j]); return -3; }
        io[t + 1] = io[t] + gotoh_io_bytes(ms[t], ns[t]);
        lds = std::max(lds, ms[t] < GOTOH_PF * GOTOH_THREADS ? gotoh_lds_bytes(ms[t], ns[t], L)
                                                             : GOTOH_LDS_MAX + 1);
        work[t + 1] = work[t] + gotoh_work_bytes(ms[t], ns[t]);
    }
    const size_t sz_mat = align16(sizeof(int) * L * L), sz_args = align16(sizeof(GotohArgs) * count);
    // device buffer: [io blocks][matrix][argument blocks][work blocks]
    const size_t off_mat = io[count], off_args = off_mat + sz_mat, off_work = off_args + sz_args;
    const size_t total = off_work + work[count] + 256;
    std::lock_guard<std::mutex> guard(c.gotoh_mutex);   // the scratch is per context
    if (c.gotoh_cap < total) {
        hipFree(c.gotoh_buf);
        c.gotoh_buf = nullptr;
        c.gotoh_cap = 0;
        MH_HIP(hipMalloc(&c.gotoh_buf, total));
        c.gotoh_cap = total;
    }
    char *d = c.gotoh_buf;
    std::vector<char> img(io[count], 0);   // host image of the io blocks
    std::vector<GotohArgs> args(count);
    for (int t = 0; t < count; ++t) {
        const int m = ms[t], n = ns[t];
        size_t o = io[t], w = off_work + work[t];
        auto take_io = [&](size_t sz) { const size_t at = o; o += align16(sz); return at; };
        auto take_w = [&](size_t sz) { char *at = d + w; w += align16(sz); return at; };
        GotohArgs &A = args[t];
        const size_t oa = take_io(m + 8), ob = take_io(n + 8), o1 = take_io(m + 1),
                     o2 = take_io(n + 1), oo1 = take_io(m + n + 1), oo2 = take_io(m + n + 1),
                     ores = take_io(64);
        A.diagR = (int *)take_w(sizeof(int) * 3 * (m + 2));
        A.diagP = (int *)take_w(sizeof(int) * 3 * (m + 2));
        A.diagQ = (int *)take_w(sizeof(int) * 3 * (m + 2));
        A.lastcol = (int *)take_w(sizeof(int) * (m + 2));
        A.lastrow = (int *)take_w(sizeof(int) * (n + 2));
        const size_t cells = (size_t)(m + 2) * (n + 2);
        A.abc = (uint8_t *)take_w(cells);
        A.de = (uint8_t *)take_w(cells);
        A.fg = (uint8_t *)take_w(cells);
        for (int i = 0; i < m; ++i) img[oa + i] = (char)code[(unsigned char)s1[t][i]];
        for (int j = 0; j < n; ++j) img[ob + j] = (char)code[(unsigned char)s2[t][j]];
        memcpy(&img[o1], s1[t], m);
        memcpy(&img[o2], s2[t], n);
        A.a = (const int8_t *)(d + oa);
        A.b = (const int8_t *)(d + ob);
        A.s1 = d + o1;
        A.s2 = d + o2;
        A.out1 = d + oo1;
        A.out2 = d + oo2;
        A.result = (int *)(d + ores);
        A.m = m; A.n = n; A.L = L; A.mat = (const int *)(d + off_mat);
        A.u = gep; A.v = gop; A.is_global = is_global ? 1 : 0;
    }
    hipStream_t st = c.stream;
    MH_HIP(hipMemsetAsync(d + off_work, 0, work[count], st));
    MH_HIP(hipMemcpyAsync(d, img.data(), io[count], hipMemcpyHostToDevice, st));
    MH_HIP(hipMemcpyAsync(d + off_mat, matrix, sizeof(int) * L * L, hipMemcpyHostToDevice, st));
    MH_HIP(hipMemcpyAsync(d + off_args, args.data(), sizeof(GotohArgs) * count,
                          hipMemcpyHostToDevice, st));
    const int pg = prof_begin(c, "k_gotoh");
    if (lds <= GOTOH_LDS_MAX) {
        MH_HIP(hipFuncSetAttribute((const void *)k_gotoh<true>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                   (int)lds));
        hipLaunchKernelGGL(k_gotoh<true>, dim3((unsigned)count), dim3(GOTOH_THREADS), lds, st,
                           (const GotohArgs *)(d + off_args));
    } else {
        hipLaunchKernelGGL(k_gotoh<false>, dim3((unsigned)count), dim3(GOTOH_THREADS), TB_LDS, st,
                           (const GotohArgs *)(d + off_args));
    }
    prof_end(c, pg);
    hipError_t e = hipGetLastError();
    if (e == hipSuccess) e = hipMemcpyAsync(img.data(), d, io[count], hipMemcpyDeviceToHost, st);
    if (e == hipSuccess) e = hipStreamSynchronize(st);
    if (e != hipSuccess) return hip_fail(e, "k_gotoh");
    for (int t = 0; t < count; ++t) {
        const GotohArgs &A = args[t];
        int res[3];
        memcpy(res, &img[(const char *)A.result - d], sizeof(res));
        status[t] = res[0] ? -1 : 0;
        score[t] = res[1];
        const int len = res[0] ? 0 : res[2];
        const char *t1 = &img[A.out1 - d], *t2 = &img[A.out2 - d];
        for (int k = 0; k < len; ++k) { out1[t][k] = t1[len - 1 - k]; out2[t][k] = t2[len - 1 - k]; }
        out1[t][len] = out2[t][len] = '\0';
    }
    if (c.gotoh_cap > GOTOH_KEEP_BYTES) {
        hipFree(c.gotoh_buf);
        c.gotoh_buf = nullptr;
        c.gotoh_cap = 0;
    }
    return 0;
}

int run_gotoh(Ctx &c, const char *s1, const char *s2, int gop, int gep, int is_global,
              const char *alphabet, const int *matrix, char *out1, char *out2, int cap, int *score)
{
    int status = 0;
    if (int st = run_gotoh_batch(c, 1, &s1, &s2, gop, gep, is_global, alphabet, matrix, &out1,
                                 &out2, &cap, score, &status))
        return st;
    if (status) { set_error("Traceback failed, try local alignment"); return -1; }
    return 0;
}

}  // namespace mh
