// mh_gotoh.hip -- the _gotoh2 aligner (micall/alignment/src/_gotoh2.c) on
// gfx950, used by the consensus-distance filter (remap.py:244-263: global,
// gop 15, gep 3, HYPHY_NUC) and aln2counts' coordinate mapping (local,
// EmpHIV25).  A batch of alignments is one launch, one workgroup of 1024
// threads per alignment (blockIdx.x = alignment), each with its own scratch:
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

#include <mutex>
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

__global__ __launch_bounds__(1024) void k_gotoh(const GotohArgs *batch)
{
    const GotohArgs A = batch[blockIdx.x];
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

static size_t align16(size_t x) { return (x + 15) & ~(size_t)15; }

// Per alignment: an "io" block (codes, strings, output strings, result: what
// crosses PCIe) and a "work" block (diagonal buffers, last row / column and
// the three tie planes, zeroed on the device).
static size_t gotoh_io_bytes(int m, int n)
{
    return align16(m + 8) + align16(n + 8) + align16(m + 1) + align16(n + 1) +
           2 * align16(m + n + 1) + 64;
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
    hipLaunchKernelGGL(k_gotoh, dim3((unsigned)count), dim3(1024), 0, st,
                       (const GotohArgs *)(d + off_args));
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
