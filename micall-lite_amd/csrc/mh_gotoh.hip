// mh_gotoh.hip -- the _gotoh2 aligner (micall/alignment/src/_gotoh2.c) on
// gfx950, used by the consensus-distance filter (remap.py:244-263: global,
// gop 15, gep 3, HYPHY_NUC).  One workgroup of 1024 threads per alignment:
//   phase 1  cost assignment (_gotoh2.c:137-201) by anti-diagonals; R/P/Q
//            live in three rolling diagonal buffers; each cell's tie bits go
//            to three byte planes so no two cells of a diagonal write the
//            same byte: abc(i,j) by (i,j), de(i,j) by (i+1,j), fg(i,j) by (i,j+1)
//   phase 2  Altschul-Erickson edge assignment (:205-313) by anti-diagonals
//            in reverse; its writes to d(i+1,j) and f(i,j+1) are never read
//            again (each cell reads its own d/f before its upper/left
//            neighbour runs) and are dropped
//   phase 3  traceback (:316-438) by one thread.
// Bit-for-bit specification: oracle/og_gotoh.c.
#include <limits.h>

#include <vector>

#include "mh_internal.h"

namespace mh {

constexpr int G_INF = INT_MAX;
enum { GA = 1, GB = 2, GC = 4, GD = 8, GE_ = 16, GF = 32, GG = 64 };

struct GotohArgs {
    const int8_t *a;      // seq1 codes, m
    const int8_t *b;      // seq2 codes, n
    int m, n, L;
    const int *mat;       // L x L
    int u, v, is_global;
    int *diagR, *diagP, *diagQ;   // 3 x (m + 2) each
    int *lastcol, *lastrow;       // R(i, n), R(m, j)
    uint8_t *abc, *de, *fg;       // (m+2) x (n+2)
    const char *s1, *s2;
    char *out1, *out2;            // m + n + 1
    int *result;                  // [0] status, [1] score, [2] length
};

__device__ __forceinline__ int gmin(int x, int y) { return x <= y ? x : y; }

__global__ __launch_bounds__(1024) void k_gotoh(GotohArgs A)
{
    const int m = A.m, n = A.n;
    const int W = n + 2;
    const int u = A.u, v = A.v;
    // ---- phase 1: cost assignment by anti-diagonals ----
    for (int s = 0; s <= m + n; ++s) {
        const int ilo = s - n > 0 ? s - n : 0, ihi = s < m ? s : m;
        int *Rc = A.diagR + (s % 3) * (m + 2), *Pc = A.diagP + (s % 3) * (m + 2),
            *Qc = A.diagQ + (s % 3) * (m + 2);
        const int *R1 = A.diagR + ((s + 2) % 3) * (m + 2), *P1 = A.diagP + ((s + 2) % 3) * (m + 2),
                  *Q1 = A.diagQ + ((s + 2) % 3) * (m + 2);
        const int *R2 = A.diagR + ((s + 1) % 3) * (m + 2);
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
                A.de[(size_t)(i - 1) * W + j] = de;
            }
            if (j == 0) {
                q = G_INF;
            } else {
                const int ql = Q1[i], rl = R1[i];           // (i, j-1) on diagonal s-1
                q = u + gmin(ql, rl + v);
                uint8_t fg = 0;
                if (ql != G_INF && q == ql + u) fg |= GF;
                if (q == rl + v + u) fg |= GG;
                A.fg[(size_t)i * W + j - 1] = fg;
            }
            if (i == 0 && j == 0) {
                r = 0;
            } else if (i == 0 || j == 0) {
                r = A.is_global ? gmin(p, q) : 0;
            } else {
                dg = R2[i - 1] - A.mat[A.a[i - 1] * A.L + A.b[j - 1]];
                r = gmin(gmin(dg, p), q);
            }
            Rc[i] = r; Pc[i] = p; Qc[i] = q;
            uint8_t abc = 0;
            if (r == p) abc |= GA;
            if (r == q) abc |= GB;
            if (i > 0 && j > 0 && r == dg) abc |= GC;
            A.abc[(size_t)i * W + j] = abc;
            if (j == n) A.lastcol[i] = r;
            if (i == m) A.lastrow[j] = r;
        }
        __syncthreads();
    }
    // boundary c bits (_gotoh2.c:117-131)
    if (!A.is_global) {
        for (int j = threadIdx.x; j <= n + 1; j += blockDim.x) A.abc[(size_t)(m + 1) * W + j] = GC;
        for (int i = threadIdx.x; i <= m + 1; i += blockDim.x) A.abc[(size_t)i * W + n + 1] = GC;
    }
    if (threadIdx.x == 0) A.abc[(size_t)(m + 1) * W + n + 1] = GC;
    __syncthreads();
    // ---- phase 2: edge assignment, anti-diagonals in reverse ----
    for (int s = m + n; s >= 0; --s) {
        const int ilo = s - n > 0 ? s - n : 0, ihi = s < m ? s : m;
        for (int i = ilo + (int)threadIdx.x; i <= ihi; i += blockDim.x) {
            const int j = s - i;
            const size_t h = (size_t)i * W + j;
            uint8_t x = A.abc[h];
            uint8_t e = A.de[h] & GE_, d = A.de[h] & GD;
            uint8_t g = A.fg[h] & GG, f = A.fg[h] & GF;
            const uint8_t dn = A.abc[h + W], rt = A.abc[h + 1], dgn = A.abc[h + W + 1];
            const bool no_a_below = !(dn & GA), no_e = !e, no_b_right = !(rt & GB), no_g = !g;
            const bool no_c_diag = !(dgn & GC);
            if ((no_a_below || no_e) && (no_b_right || no_g) && no_c_diag) x &= (uint8_t)~(GA | GB | GC);
            if (!(no_a_below && no_b_right && no_c_diag)) {
                if ((dn & GA) && d) {
                    e = (x & GA) ? 0 : GE_;
                    x |= GA;
                } else {
                    e = 0;
                }
                if ((rt & GB) && f) {
                    g = (x & GB) ? 0 : GG;
                    x |= GB;
                } else {
                    g = 0;
                }
            }
            A.abc[h] = x;
            (void)e; (void)g;
        }
        __syncthreads();
    }
    // ---- phase 3: traceback (one thread) ----
    if (threadIdx.x == 0) {
        int ii = m, jj = n, best = A.lastrow[n];
        if (!A.is_global) {
            for (int i = 0; i <= m; ++i) if (A.lastcol[i] < best) { best = A.lastcol[i]; ii = i; jj = n; }
            for (int j = 0; j <= n; ++j) if (A.lastrow[j] < best) { best = A.lastrow[j]; ii = m; jj = j; }
        }
        int len = 0;
        char *r1 = A.out1, *r2 = A.out2;   // built back to front, reversed by the host
        if (ii < m) for (int k = m - 1; k >= ii; --k) { r1[len] = A.s1[k]; r2[len] = '-'; ++len; }
        if (jj < n) for (int k = n - 1; k >= jj; --k) { r1[len] = '-'; r2[len] = A.s2[k]; ++len; }
        int status = 0;
        while (ii > 0 && jj > 0) {
            const uint8_t x = A.abc[(size_t)ii * W + jj];
            if (x & GA) { r1[len] = A.s1[ii - 1]; r2[len] = '-'; --ii; }
            else if (x & GB) { r1[len] = '-'; r2[len] = A.s2[jj - 1]; --jj; }
            else if (x & GC) { r1[len] = A.s1[ii - 1]; r2[len] = A.s2[jj - 1]; --ii; --jj; }
            else { status = -1; break; }
            ++len;
        }
        if (status == 0) {
            while (ii > 0) { r1[len] = A.s1[ii - 1]; r2[len] = '-'; --ii; ++len; }
            while (jj > 0) { r1[len] = '-'; r2[len] = A.s2[jj - 1]; --jj; ++len; }
        }
        A.result[0] = status;
        A.result[1] = -best;
        A.result[2] = len;
    }
}

int run_gotoh(Ctx &c, const char *s1, const char *s2, int gop, int gep, int is_global,
              const char *alphabet, const int *matrix, char *out1, char *out2, int cap, int *score)
{
    const int m = (int)strlen(s1), n = (int)strlen(s2), L = (int)strlen(alphabet);
    if (m == 0 || n == 0 || L == 0 || cap < m + n + 1) { set_error("mh_gotoh_align: bad arguments"); return -3; }
    int code[256];
    for (int k = 0; k < 256; ++k) code[k] = -1;
    for (int k = 0; k < L; ++k) code[(unsigned char)alphabet[k]] = k;
    std::vector<int8_t> ha(m), hb(n);
    for (int i = 0; i < m; ++i) if ((ha[i] = (int8_t)code[(unsigned char)s1[i]]) < 0) { set_error("mh_gotoh_align: '%c' not in alphabet", s1[i]); return -3; }
    for (int j = 0; j < n; ++j) if ((hb[j] = (int8_t)code[(unsigned char)s2[j]]) < 0) { set_error("mh_gotoh_align: '%c' not in alphabet", s2[j]); return -3; }
    const size_t cells = (size_t)(m + 2) * (n + 2);
    // one allocation for everything
    const size_t sz_codes = (size_t)m + n + 16, sz_mat = sizeof(int) * L * L,
                 sz_diag = sizeof(int) * 3 * (m + 2) * 3, sz_last = sizeof(int) * (m + n + 4),
                 sz_bits = 3 * cells, sz_str = (size_t)2 * (m + n + 2) * 2, sz_res = 64;
    const size_t total = sz_codes + sz_mat + sz_diag + sz_last + sz_bits + sz_str + sz_res + 256;
    if (c.gotoh_cap < total) {
        hipFree(c.gotoh_buf);
        c.gotoh_buf = nullptr;
        c.gotoh_cap = 0;
        MH_HIP(hipMalloc(&c.gotoh_buf, total));
        c.gotoh_cap = total;
    }
    char *d = c.gotoh_buf;
    size_t o = 0;
    auto take = [&](size_t sz) { char *p = d + o; o += (sz + 15) & ~(size_t)15; return p; };
    GotohArgs A{};
    int8_t *da = (int8_t *)take(m + 8), *db = (int8_t *)take(n + 8);
    int *dm = (int *)take(sz_mat);
    A.diagR = (int *)take(sizeof(int) * 3 * (m + 2));
    A.diagP = (int *)take(sizeof(int) * 3 * (m + 2));
    A.diagQ = (int *)take(sizeof(int) * 3 * (m + 2));
    A.lastcol = (int *)take(sizeof(int) * (m + 2));
    A.lastrow = (int *)take(sizeof(int) * (n + 2));
    A.abc = (uint8_t *)take(cells);
    A.de = (uint8_t *)take(cells);
    A.fg = (uint8_t *)take(cells);
    char *ds1 = take(m + 1), *ds2 = take(n + 1);
    A.out1 = take(m + n + 1);
    A.out2 = take(m + n + 1);
    A.result = (int *)take(sz_res);
    hipStream_t st = c.stream;
    MH_HIP(hipMemsetAsync(A.abc, 0, 3 * ((cells + 15) & ~(size_t)15), st));
    MH_HIP(hipMemcpyAsync(da, ha.data(), m, hipMemcpyHostToDevice, st));
    MH_HIP(hipMemcpyAsync(db, hb.data(), n, hipMemcpyHostToDevice, st));
    MH_HIP(hipMemcpyAsync(dm, matrix, sz_mat, hipMemcpyHostToDevice, st));
    MH_HIP(hipMemcpyAsync(ds1, s1, m, hipMemcpyHostToDevice, st));
    MH_HIP(hipMemcpyAsync(ds2, s2, n, hipMemcpyHostToDevice, st));
    A.a = da; A.b = db; A.m = m; A.n = n; A.L = L; A.mat = dm;
    A.u = gep; A.v = gop; A.is_global = is_global ? 1 : 0;
    A.s1 = ds1; A.s2 = ds2;
    hipLaunchKernelGGL(k_gotoh, dim3(1), dim3(1024), 0, st, A);
    hipError_t e = hipGetLastError();
    int res[3] = {0, 0, 0};
    std::vector<char> t1(m + n + 1), t2(m + n + 1);
    if (e == hipSuccess) e = hipMemcpyAsync(res, A.result, sizeof(res), hipMemcpyDeviceToHost, st);
    if (e == hipSuccess) e = hipStreamSynchronize(st);
    if (e == hipSuccess && res[0] == 0) {
        e = hipMemcpy(t1.data(), A.out1, res[2], hipMemcpyDeviceToHost);
        if (e == hipSuccess) e = hipMemcpy(t2.data(), A.out2, res[2], hipMemcpyDeviceToHost);
    }
    if (e != hipSuccess) return hip_fail(e, "k_gotoh");
    if (res[0] != 0) { set_error("Traceback failed, try local alignment"); return -1; }
    const int len = res[2];
    for (int k = 0; k < len; ++k) { out1[k] = t1[len - 1 - k]; out2[k] = t2[len - 1 - k]; }
    out1[len] = out2[len] = '\0';
    *score = res[1];
    return 0;
}

}  // namespace mh
