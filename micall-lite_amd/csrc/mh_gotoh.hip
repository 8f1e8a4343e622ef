// mh_gotoh.hip -- the _gotoh2 aligner (micall/alignment/src/_gotoh2.c) on
// gfx950, used by the consensus-distance filter (remap.py:244-263: global,
// gop 15, gep 3, HYPHY_NUC) and aln2counts' coordinate mapping (local,
// EmpHIV25).  A batch of alignments is three launches.
//
// The DP grid (rows 0..m of seq1, columns 0..n of seq2) is cut into strips
// of 64 rows, one wave (one workgroup) each, spread over the whole GPU.  In
// a strip lane l owns row 64k + l and steps along the columns skewed by its
// lane (at step t it is at column t - l), so the cell above a lane's cell is
// the lane before it one step earlier and the cell up-left two steps
// earlier: both arrive by one DPP lane shift, and a step needs no barrier.
// Every step's 64 cells lie on one anti-diagonal.  A strip's first lane
// takes the row above it from the strip before, which is running a few
// dozen columns ahead: the last row of every strip goes to global memory
// and is published in blocks of 32 columns (a per-strip progress counter,
// release / acquire at device scope); the reader loads a block ahead.
// Strips are taken by ticket (one atomic counter), in the order their
// dependencies run, so a strip only ever waits for one already running.
//   k_gotoh_fwd  cost assignment (_gotoh2.c:137-201): R/P/Q in registers,
//                each cell's tie bits to three byte planes: abc(i,j) by
//                (i,j), de(i,j) by (i+1,j), fg(i,j) by (i,j+1)
//   k_gotoh_bwd  Altschul-Erickson edge assignment (:205-313), lane l at
//                column n + 63 - l - t, strips bottom-up; a cell's final
//                bits reach the lane above one step later and the strip
//                above through its first row; its writes to d(i+1,j) and
//                f(i,j+1) are never read again (each cell reads its own d/f
//                before its upper/left neighbour runs) and are dropped
//   k_gotoh_tb   traceback (:316-438) by one thread over LDS windows.
// The planes are stored anti-diagonal-major over the (m+2) x (n+2) grid
// (doff[s] = first byte of diagonal s, cells by row i), so a step's plane
// bytes are consecutive; they are written and read through buffer
// resources: the diagonal base is a scalar offset, a lane's row its vector
// offset, and a lane with no cell this step points past the buffer (the
// hardware drops the store / returns 0) instead of branching.
// Bit-for-bit specification: oracle/og_gotoh.c.
#include <limits.h>

#include <mutex>
#include <vector>

#include "mh_internal.h"

namespace mh {

constexpr int G_INF = INT_MAX;
enum { GA = 1, GB = 2, GC = 4, GD = 8, GE_ = 16, GF = 32, GG = 64 };
constexpr int GOTOH_THREADS = 1024;        // k_gotoh_tb
constexpr int GBLK = 32;                   // boundary columns published / awaited at a time
constexpr int GBC_MAX = 32 * 1024;         // seq2 codes kept in LDS up to this length
constexpr uint32_t GOOB = 0x80000000u;     // a buffer offset past every plane (planes < 2 GiB)
constexpr int TB = 128;                                // traceback window (diagonals x rows)
constexpr size_t TB_LDS = (size_t)TB * TB + 2 * TB;   // window + both sequences' characters

__host__ __device__ inline size_t gotoh_al16(size_t x) { return (x + 15) & ~(size_t)15; }

struct GotohArgs {
    const int8_t *a;      // seq1 codes, m
    const int8_t *b;      // seq2 codes, n
    int m, n, L;
    const int *mat;       // L x L
    int u, v, is_global;
    int *lastcol, *lastrow;       // R(i, n), R(m, j)
    uint8_t *bits;                // (m+2) x (n+2) tie bits a..g of every cell, anti-diagonal-major
    uint8_t *rowde;               // d / e bits of every strip's last row (strips x (n+1))
    unsigned long long *brow1;    // k_gotoh_fwd: R, P of every strip's last row (strips x (n+1))
    int *brow2;                   // k_gotoh_bwd: final abc of every strip's first row, by n - j
    int *flags;                   // [0] a wait timed out
    const char *s1, *s2;
    char *out1, *out2;            // m + n + 1
    int *result;                  // [0] status, [1] score, [2] length
};

// the strips of a batch, in ticket order (alignment-major)
struct GotohStrips {
    const GotohArgs *args;
    const int *first;             // per alignment: its first ticket; [count] = total
    int count;
    int *ticket;                  // [0] fwd, [1] bwd
};

__device__ __forceinline__ int gmin(int x, int y) { return x <= y ? x : y; }

// First plane byte of anti-diagonal s of the (M+1) x (N+1) grid (M = m+1,
// N = n+1): the sum of len(t) = min(t, M) - max(0, t - N) + 1 over t < s.
__host__ __device__ __forceinline__ int64_t doff_of(int64_t s, int64_t M, int64_t N)
{
    const int64_t s1 = s <= M + 1 ? s * (s - 1) / 2 : M * (M + 1) / 2 + (s - 1 - M) * M;
    const int64_t s2 = s <= N + 1 ? 0 : (s - 1 - N) * (s - N) / 2;
    return s + s1 - s2;
}

// cells of anti-diagonal s of the plane grid
__host__ __device__ __forceinline__ int64_t dlen(int64_t s, int64_t M, int64_t N)
{
    return (s < M ? s : M) - (s - N > 0 ? s - N : 0) + 1;
}

// plane base of diagonal s, indexed by row i: diagonal s starts at row
// max(0, s - (n+1))
__device__ __forceinline__ int64_t dbase(int s, int m, int n)
{
    const int lo = s - (n + 1) > 0 ? s - (n + 1) : 0;
    return doff_of(s, m + 1, n + 1) - lo;
}

// lane l <- lane l - 1 (lane 0 keeps old) / lane l <- lane l + 1 (lane 63 keeps old)
__device__ __forceinline__ int from_prev_lane(int old, int v)
{
    return __builtin_amdgcn_update_dpp(old, v, 0x138, 0xF, 0xF, false);
}
__device__ __forceinline__ int from_next_lane(int old, int v)
{
    return __builtin_amdgcn_update_dpp(old, v, 0x130, 0xF, 0xF, false);
}

// a wave-uniform value the compiler cannot prove uniform (loaded through a
// pointer), moved to scalar registers
template <class T>
__device__ __forceinline__ T uni(T v)
{
    static_assert(sizeof(T) == 8 || sizeof(T) == 4, "uni: 4 or 8 bytes");
    if constexpr (sizeof(T) == 8) {
        uint64_t x;
        __builtin_memcpy(&x, &v, 8);
        const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)x);
        const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(x >> 32));
        x = (uint64_t)hi << 32 | lo;
        __builtin_memcpy(&v, &x, 8);
    } else {
        uint32_t x;
        __builtin_memcpy(&x, &v, 4);
        x = __builtin_amdgcn_readfirstlane(x);
        __builtin_memcpy(&v, &x, 4);
    }
    return v;
}

// a buffer resource over bytes [p, p + bytes): the base and size are
// wave-uniform, so the descriptor lives in scalar registers
__device__ __forceinline__ __amdgpu_buffer_rsrc_t brsrc(const void *p, uint32_t bytes)
{
    return __builtin_amdgcn_make_buffer_rsrc((void *)uni(p), (short)0, (int)uni(bytes), 0x00020000);
}

constexpr int GWAIT_MAX = 1 << 23;   // polls before a wait is declared broken (~0.25 s)

// boundary cells: device-coherent loads / stores (another strip, on any XCD,
// reads them while this launch runs)
template <class T>
__device__ __forceinline__ T dev_load(const T *p)
{
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
template <class T>
__device__ __forceinline__ void dev_store(T *p, T v)
{
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// the strip of ticket u: (alignment, index in ticket order)
__device__ __forceinline__ void strip_of(const GotohStrips &S, int u, int &t, int &q)
{
    int lo = 0, hi = S.count;   // first[lo] <= u < first[hi]
    while (hi - lo > 1) {
        const int mid = (lo + hi) >> 1;
        if (S.first[mid] <= u) lo = mid; else hi = mid;
    }
    t = lo;
    q = u - S.first[lo];
}

// A boundary cell of the forward pass as one 64-bit word written by one
// store: R (26 bits, signed), P (26 bits, signed; all ones = infinity) and
// the producing strip's tag (12 bits, never 0), so the reader polls the
// cells themselves and the writer needs no store-completion wait.  The
// host bounds |R|, |P| < 2^24.
constexpr uint32_t RP_INF = 0x1FFFFFFu;
__device__ __forceinline__ uint32_t strip_tag(int k) { return (uint32_t)(k % 4095) + 1; }
__device__ __forceinline__ unsigned long long rp_pack(int r, int p, uint32_t tag)
{
    const uint64_t pf = p == G_INF ? RP_INF : ((uint32_t)p & 0x3FFFFFFu);
    return ((uint64_t)(uint32_t)r & 0x3FFFFFFu) | pf << 26 | (uint64_t)tag << 52;
}
__device__ __forceinline__ int rp_r(unsigned long long w) { return ((int)((uint32_t)w << 6)) >> 6; }
__device__ __forceinline__ int rp_p(unsigned long long w)
{
    const uint32_t f = (uint32_t)(w >> 26) & 0x3FFFFFFu;
    return f == RP_INF ? G_INF : ((int)(f << 6)) >> 6;
}
__device__ __forceinline__ uint32_t rp_tag(unsigned long long w) { return (uint32_t)(w >> 52); }

// Poll a block of boundary cells (lanes 0..31 hold one each) until every
// cell the block has carries the producing strip's tag.  A wait that
// outlasts any legitimate one (~0.25 s) sets flags[0] and gives up, so a
// broken protocol ends the launch with an error instead of hanging.
template <class T, class Tag>
__device__ __forceinline__ T poll_block(const T *p, int lane, bool has, Tag tagged, int *flags)
{
    T v{};
    for (int it = 0;; ++it) {
        if (has) v = dev_load(p + lane);
        if (__builtin_amdgcn_ballot_w64(has && !tagged(v)) == 0) return v;
        if (it >= GWAIT_MAX ||
            __builtin_amdgcn_readfirstlane(__hip_atomic_load(flags, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT))) {
            __hip_atomic_store(flags, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            return v;
        }
        __builtin_amdgcn_s_sleep(2);
    }
}

// Cost assignment of one strip.  Every cell's seven tie bits go to ONE plane
// byte, stored one step late: at step t lane l holds abc of (i, j - 1) from
// the step before, computes fg of (i, j - 1) itself (from cell (i, j)) and
// gets de of (i, j - 1) from the lane below (cell (i + 1, j - 1)) by a lane
// shift.  The strip's last row gets its de bits from the next strip's first
// lane, which stores them in a side row (rowde).
template <bool BCL>   // seq2's codes in LDS (else read from global memory every step)
__global__ __launch_bounds__(64) void k_gotoh_fwd(GotohStrips S)
{
    extern __shared__ __attribute__((aligned(16))) unsigned char gsm[];
    const int lane = threadIdx.x;
    int u = 0;
    if (lane == 0) u = atomicAdd(&S.ticket[0], 1);
    u = __builtin_amdgcn_readfirstlane(__shfl(u, 0));
    int ta, k;
    strip_of(S, u, ta, k);
    const GotohArgs &A = S.args[ta];
    const int m = uni(A.m), n = uni(A.n), L = uni(A.L), uu = uni(A.u), v = uni(A.v);
    const bool glob = uni(A.is_global);
    int *mat = (int *)gsm;
    int8_t *bcl = (int8_t *)(gsm + gotoh_al16(sizeof(int) * L * L));
    for (int x = lane; x < L * L; x += 64) mat[x] = A.mat[x];
    if (BCL)
        for (int x = lane; x < n; x += 64) bcl[x] = A.b[x];
    __syncthreads();
    const int ns = (m + 1 + 63) / 64;
    const int W1 = n + 1;
    const int64_t cells = (int64_t)(m + 2) * (n + 2);
    const __amdgpu_buffer_rsrc_t rbits = brsrc(A.bits, (uint32_t)cells);
    const __amdgpu_buffer_rsrc_t rcol = brsrc(A.lastcol, 4u * (m + 1)), rrow = brsrc(A.lastrow, 4u * (n + 1));
    const int i = 64 * k + lane;
    const bool rowok = i <= m;
    const int arow = (i >= 1 && rowok) ? A.a[i - 1] * L : 0;
    const bool produce = k + 1 < ns, consume = k > 0;
    const unsigned long long *above = A.brow1 + (size_t)(k - 1) * W1;   // row 64k - 1
    unsigned long long *below = A.brow1 + (size_t)k * W1;
    // de bits of row 64k - 1 (the strip above's last row), by column
    const __amdgpu_buffer_rsrc_t rside = brsrc(A.rowde + (size_t)(k - 1) * W1, consume ? (uint32_t)W1 : 0u);
    const int *flags = A.flags;
    int Rme = 0, Pme = G_INF, Qme = G_INF;   // this lane's cell of the last step: (i, j - 1)
    int Rdg = 0;                              // R(i - 1, j - 1): the row above one step ago
    int bcode = 0;                            // seq2 code of column j - 1
    int abcp = 0;                             // abc of (i, j - 1), stored this step
    unsigned long long blk = 0;                  // lanes 0..31: the row above, this block's columns
    // plane bases of diagonals s = 64 k + t and s - 1, kept running:
    // D(s + 1) = D(s) + len(s)
    int64_t Ds = doff_of(64 * k, m + 1, n + 1);
    int64_t Dprev = Ds - (k > 0 ? dlen(64 * k - 1, m + 1, n + 1) : 0);
    for (int t = 0; t <= n + 64; ++t) {
        const int j = t - lane;
        const int tq = t & (GBLK - 1);
        if (consume && tq == 0 && t <= n) {
            // this block of the row above: poll its cells until they carry
            // the strip above's tag, and use them at once (the wait then
            // covers the load only here, not at every step's read)
            const uint32_t want = strip_tag(k - 1);
            blk = poll_block(above + t, lane, lane < GBLK && t + lane < W1,
                             [&](unsigned long long w) { return rp_tag(w) == want; }, (int *)flags);
            asm volatile("; touch %0" : "+v"(blk));
        }
        int Rup = from_prev_lane(0, Rme), Pup = from_prev_lane(G_INF, Pme);
        const int bnew = (t >= 1 && t <= n) ? (BCL ? (int)bcl[t - 1] : (int)A.b[t - 1]) : 0;
        bcode = from_prev_lane(bnew, bcode);
        if (consume && t <= n) {
            const int r0 = rp_r(((unsigned long long)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(blk >> 32), tq) << 32) |
                                (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)blk, tq));
            const int p0 = rp_p(((unsigned long long)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(blk >> 32), tq) << 32) |
                                (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)blk, tq));
            Rup = lane == 0 ? r0 : Rup;
            Pup = lane == 0 ? p0 : Pup;
        }
        const bool act = rowok && j >= 0 && j <= n;
        const bool top = i == 0, left = j == 0;
        const int pm = gmin(Pup, Rup + v);
        const int p = top ? G_INF : uu + pm;
        const int qm = gmin(Qme, Rme + v);
        const int q = left ? G_INF : uu + qm;
        // de of (i - 1, j) and fg of (i, j - 1)
        const int de = (act && !top) ? ((Pup != G_INF && pm == Pup) ? GD : 0) | (pm == Rup + v ? GE_ : 0) : 0;
        const int fg = (act && !left) ? ((Qme != G_INF && qm == Qme) ? GF : 0) | (qm == Rme + v ? GG : 0) : 0;
        const int dg = Rdg - mat[arow + bcode];
        const int border = glob ? gmin(p, q) : 0;
        const int r = (top && left) ? 0 : ((top || left) ? border : gmin(gmin(dg, p), q));
        const int abc = (r == p ? GA : 0) | (r == q ? GB : 0) | ((!top && !left && r == dg) ? GC : 0);
        // the byte of (i, j - 1): its abc (last step), fg (this lane now) and
        // de (the lane below now; the strip's last row: rowde)
        const int deb = from_next_lane(0, de);
        const int s = 64 * k + t;
        const uint32_t b1 = (uint32_t)(Dprev - (s - 1 - (n + 1) > 0 ? s - 1 - (n + 1) : 0));
        Dprev = Ds;
        Ds += dlen(s, m + 1, n + 1);
        const bool pend = rowok && j >= 1 && j <= n + 1;
        __builtin_amdgcn_raw_buffer_store_b8((uint8_t)(abcp | fg | (lane == 63 ? 0 : deb)), rbits,
                                             pend ? (uint32_t)i : GOOB, b1, 0);
        // the first lane's de belongs to the strip above's last row
        if (consume)
            __builtin_amdgcn_raw_buffer_store_b8((uint8_t)de, rside, (lane == 0 && act) ? (uint32_t)j : GOOB, 0, 0);
        if (t >= n)   // some lane is at column n
            __builtin_amdgcn_raw_buffer_store_b32(r, rcol, (act && j == n) ? 4u * (uint32_t)i : GOOB, 0, 0);
        if (!produce)   // the last strip holds row m
            __builtin_amdgcn_raw_buffer_store_b32(r, rrow, (act && i == m) ? 4u * (uint32_t)j : GOOB, 0, 0);
        abcp = act ? abc : 0;
        Rdg = Rup;
        Rme = act ? r : 0;
        Pme = act ? p : G_INF;
        Qme = act ? q : G_INF;
        // the strip's last row (lane 63, column t - 63) to the strip below
        const int jp = t - 63;
        if (produce && jp >= 0 && jp <= n && lane == 63) dev_store(below + jp, rp_pack(r, p, strip_tag(k)));
    }
}

// Edge assignment of one strip (bottom-up, right to left).  Each block of
// GBLK steps first loads the block's plane bytes (loaded during the block
// before), then computes, then stores the block's final bytes: loads and
// stores never interleave inside a block, so no step waits on a store.
__global__ __launch_bounds__(64) void k_gotoh_bwd(GotohStrips S)
{
    const int lane = threadIdx.x;
    int u = 0;
    if (lane == 0) u = atomicAdd(&S.ticket[1], 1);
    u = __builtin_amdgcn_readfirstlane(__shfl(u, 0));
    int ta, q0;
    strip_of(S, u, ta, q0);
    const GotohArgs &A = S.args[ta];
    const int m = uni(A.m), n = uni(A.n);
    const int ns = (m + 1 + 63) / 64;
    const int k = ns - 1 - q0;                 // strips bottom-up
    const int W1 = n + 1;
    const int64_t cells = (int64_t)(m + 2) * (n + 2);
    const __amdgpu_buffer_rsrc_t rbits = brsrc(A.bits, (uint32_t)cells);
    const uint8_t bnd = A.is_global ? 0 : GC;
    const int i = 64 * k + lane;
    const bool rowok = i <= m, lastr = i == m;
    const bool produce = k > 0, consume = k + 1 < ns;
    const int *under = A.brow2 + (size_t)(k + 1) * W1;   // row 64k + 64, by tau = n - j
    int *mytop = A.brow2 + (size_t)k * W1;
    // de bits of this strip's last row (stored by the strip below), by column
    const __amdgpu_buffer_rsrc_t rside = brsrc(A.rowde + (size_t)k * W1, consume ? (uint32_t)W1 : 0u);
    const int *flags = A.flags;
    int mine = 0;        // final abc of (i, j + 1): this lane, one step ago
    int dnp = 0;         // final abc of (i + 1, j + 1): the lane below, two steps ago
    // plane base of the step's diagonal s = 64 k + n + 63 - t, running down:
    // D(s - 1) = D(s) - len(s - 1)
    const int s0 = 64 * k + n + 63;
    int64_t Dld = doff_of(s0, m + 1, n + 1), Dst = Dld;
    int cx[GBLK], nx[GBLK], ox[GBLK];
    // the plane bytes of steps t0 .. t0 + GBLK - 1
    auto load_block = [&](int t0b, int *dst) {
#pragma unroll
        for (int q = 0; q < GBLK; ++q) {
            const int tt = t0b + q, jj = n + 63 - lane - tt, sd = s0 - tt;
            const uint32_t base = (uint32_t)(Dld - (sd - (n + 1) > 0 ? sd - (n + 1) : 0));
            const bool ok = rowok && jj >= 0 && jj <= n && tt <= n + 63;
            dst[q] = __builtin_amdgcn_raw_buffer_load_b8(rbits, ok ? (uint32_t)i : GOOB, base, 0);
            Dld -= dlen(sd - 1, m + 1, n + 1);
        }
    };
    load_block(0, cx);
    for (int t0 = 0; t0 <= n + 63; t0 += GBLK) {
        // the strip below's first row for this block (lane 63's cells below)
        // (tagged with the strip below's tag), and lanes 0..31: the de side
        // bits of lane 63's cells (column n - t)
        int blk = 0, side = 0;
        if (consume && t0 <= n) {
            const int want = (k + 1) % 0xFFFFFF + 1;
            blk = poll_block(under + t0, lane, lane < GBLK && t0 + lane < W1,
                             [&](int w) { return (w >> 8) == want; }, (int *)flags);
            side = __builtin_amdgcn_raw_buffer_load_b8(rside, (lane < GBLK && t0 + lane <= n) ?
                                                       (uint32_t)(n - t0 - lane) : GOOB, 0, 0);
        }
        asm volatile("; touch %0 %1" : "+v"(blk), "+v"(side));
#pragma unroll
        for (int q = 0; q < GBLK; ++q) asm volatile("; touch %0" : "+v"(cx[q]));
        load_block(t0 + GBLK, nx);
#pragma unroll
        for (int q = 0; q < GBLK; ++q) {
            const int t = t0 + q;
            const int j = n + 63 - lane - t;
            int dnb = from_next_lane(0, mine);                   // final abc of (i + 1, j)
            const int d63 = __builtin_amdgcn_readlane(blk, q) & 0xFF;
            dnb = (lane == 63 && consume && t <= n) ? d63 : dnb;
            const bool act = rowok && j >= 0 && j <= n;
            const bool lastc = j == n;
            const int c = cx[q] | (lane == 63 ? __builtin_amdgcn_readlane(side, q) : 0);
            const int dn = lastr ? (lastc ? GC : bnd) : dnb;
            const int rt = lastc ? (lastr ? GC : bnd) : mine;
            const int dgn = (lastr || lastc) ? ((lastr && lastc) ? GC : bnd) : dnp;
            // Altschul-Erickson steps 8-11 of the cell
            int x = c;
            const bool no_a_below = !(dn & GA), no_e = !(c & GE_), no_b_right = !(rt & GB), no_g = !(c & GG);
            const bool no_c_diag = !(dgn & GC);
            if ((no_a_below || no_e) && (no_b_right || no_g) && no_c_diag) x &= ~(GA | GB | GC);
            if (!(no_a_below && no_b_right && no_c_diag)) {
                if ((dn & GA) && (c & GD)) x |= GA;
                if ((rt & GB) && (c & GF)) x |= GB;
            }
            ox[q] = act ? x : 0;
            dnp = dnb;
            mine = act ? x : 0;
        }
        // the block's final bytes; the strip's first row (lane 0) to the strip above
#pragma unroll
        for (int q = 0; q < GBLK; ++q) {
            const int t = t0 + q, j = n + 63 - lane - t, sd = s0 - t;
            const uint32_t b0 = (uint32_t)(Dst - (sd - (n + 1) > 0 ? sd - (n + 1) : 0));
            Dst -= dlen(sd - 1, m + 1, n + 1);
            const bool act = rowok && j >= 0 && j <= n && t <= n + 63;
            __builtin_amdgcn_raw_buffer_store_b8((uint8_t)ox[q], rbits, act ? (uint32_t)i : GOOB, b0, 0);
            const int tp = t - 63;
            if (produce && tp >= 0 && tp <= n && lane == 0) dev_store(mytop + tp, (k % 0xFFFFFF + 1) << 8 | ox[q]);
        }
#pragma unroll
        for (int q = 0; q < GBLK; ++q) cx[q] = nx[q];
    }
}

// One workgroup per alignment: the best start cell and the traceback.
__global__ __launch_bounds__(GOTOH_THREADS) void k_gotoh_tb(const GotohArgs *batch)
{
    extern __shared__ __attribute__((aligned(16))) unsigned char gsm[];
    const GotohArgs A = batch[blockIdx.x];
    const int m = A.m, n = A.n;
    const int gabort = A.flags[0];
    // ---- phase 3: traceback ----
    // The walk is serial, so it never waits on global memory: the block
    // stages a TB x TB window of abc (diagonals s0 .. s0-TB+1, rows
    // ii .. ii-TB+1 of the current cell (ii, jj), which holds every cell the
    // path can reach before it leaves the window) and the TB characters of
    // each sequence before ii / jj into LDS; thread 0 walks the window and
    // writes the output characters; repeat.  The gap runs at both ends are
    // written by the whole block.
    uint8_t *win = gsm;
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
            uint8_t vv = 0;
            if (i >= 1 && j >= 1 && j <= n) vv = A.bits[dbase(sd, m, n) + i];   // (r <= t on the path)
            win[x] = vv;
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
        A.result[0] = gabort ? -4 : status;
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

static size_t gotoh_work_bytes(int m, int n)
{
    const size_t strips = (size_t)(m + 1 + 63) / 64;
    return align16(sizeof(int) * (m + 2)) + align16(sizeof(int) * (n + 2)) +
           align16((size_t)(m + 2) * (n + 2)) + align16(8 * strips * (n + 1)) +
           align16(sizeof(int) * strips * (n + 1)) + align16(strips * (n + 1)) + 16;
}

// Retained scratch above this is released after the call (one very long
// alignment must not pin device memory for the rest of the session).
constexpr size_t GOTOH_KEEP_BYTES = (size_t)1 << 30;

int run_gotoh_batch(Ctx &c, int count, const char *const *s1, const char *const *s2, int gop,
                    int gep, int is_global, const char *alphabet, const int *matrix,
                    char *const *out1, char *const *out2, const int *cap, int *score, int *status)
{
    const int L = (int)strlen(alphabet);
    if (count < 0 || L == 0 || L > 64) { set_error("mh_gotoh_align: bad arguments"); return -3; }
    if (count == 0) return 0;
    int code[256];
    for (int k = 0; k < 256; ++k) code[k] = -1;
    for (int k = 0; k < L; ++k) code[(unsigned char)alphabet[k]] = k;
    int64_t mat_max = 0;
    for (int x = 0; x < L * L; ++x) mat_max = std::max<int64_t>(mat_max, std::abs((int64_t)matrix[x]));
    if (gop < 0 || gep < 0 || gop > (1 << 16) || gep > (1 << 16)) { set_error("mh_gotoh_align: bad gap penalties"); return -3; }
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
        // boundary cells carry R and P in 26 bits (k_gotoh_fwd rp_pack)
        if ((int64_t)(ms[t] + ns[t] + 2) * (mat_max + gop + gep + 1) >= ((int64_t)1 << 24)) {
            set_error("mh_gotoh_align: alignment %d too long for the score range", t);
            return -3;
        }
        if ((uint64_t)(ms[t] + 2) * (uint64_t)(ns[t] + 2) >= (uint64_t)GOOB) {
            set_error("mh_gotoh_align: alignment %d too large (%d x %d)", t, ms[t], ns[t]);
            return -3;
        }
        work[t + 1] = work[t] + gotoh_work_bytes(ms[t], ns[t]);
    }
    // strips in ticket order: every alignment's, alignment by alignment
    std::vector<int> first(count + 1, 0);
    for (int t = 0; t < count; ++t) first[t + 1] = first[t] + (ms[t] + 1 + 63) / 64;
    const size_t sz_mat = align16(sizeof(int) * L * L), sz_args = align16(sizeof(GotohArgs) * count);
    const size_t sz_first = align16(sizeof(int) * (count + 1)) + 16;   // + the two ticket counters
    // device buffer: [io blocks][matrix][arguments][strip table, tickets][work blocks]
    const size_t off_mat = io[count], off_args = off_mat + sz_mat, off_first = off_args + sz_args,
                 off_work = off_first + sz_first;
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
        A.lastcol = (int *)take_w(sizeof(int) * (m + 2));
        A.lastrow = (int *)take_w(sizeof(int) * (n + 2));
        const size_t cells = (size_t)(m + 2) * (n + 2);
        A.bits = (uint8_t *)take_w(cells);
        const size_t strips = (size_t)(m + 1 + 63) / 64;
        A.brow1 = (unsigned long long *)take_w(8 * strips * (n + 1));
        A.brow2 = (int *)take_w(sizeof(int) * strips * (n + 1));
        A.rowde = (uint8_t *)take_w(strips * (n + 1));
        A.flags = (int *)take_w(16);
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
    MH_HIP(hipMemsetAsync(d + off_first, 0, sz_first, st));
    MH_HIP(hipMemcpyAsync(d, img.data(), io[count], hipMemcpyHostToDevice, st));
    MH_HIP(hipMemcpyAsync(d + off_mat, matrix, sizeof(int) * L * L, hipMemcpyHostToDevice, st));
    MH_HIP(hipMemcpyAsync(d + off_args, args.data(), sizeof(GotohArgs) * count,
                          hipMemcpyHostToDevice, st));
    MH_HIP(hipMemcpyAsync(d + off_first, first.data(), sizeof(int) * (count + 1), hipMemcpyHostToDevice, st));
    GotohStrips S;
    S.args = (const GotohArgs *)(d + off_args);
    S.first = (const int *)(d + off_first);
    S.count = count;
    S.ticket = (int *)(d + off_first + sz_first - 16);
    const int strips = first[count];
    const int pf = prof_begin(c, "k_gotoh_fwd");
    int nmax = 0;
    for (int t = 0; t < count; ++t) nmax = std::max(nmax, ns[t]);
    const size_t lds_fwd = gotoh_al16(sizeof(int) * L * L) + (nmax <= GBC_MAX ? gotoh_al16(nmax) : 0);
    if (nmax <= GBC_MAX) {
        MH_HIP(hipFuncSetAttribute((const void *)k_gotoh_fwd<true>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                   (int)lds_fwd));
        hipLaunchKernelGGL(k_gotoh_fwd<true>, dim3((unsigned)strips), dim3(64), lds_fwd, st, S);
    } else {
        hipLaunchKernelGGL(k_gotoh_fwd<false>, dim3((unsigned)strips), dim3(64), lds_fwd, st, S);
    }
    prof_end(c, pf);
    const int pb = prof_begin(c, "k_gotoh_bwd");
    hipLaunchKernelGGL(k_gotoh_bwd, dim3((unsigned)strips), dim3(64), 0, st, S);
    prof_end(c, pb);
    const int pg = prof_begin(c, "k_gotoh");
    hipLaunchKernelGGL(k_gotoh_tb, dim3((unsigned)count), dim3(GOTOH_THREADS), TB_LDS, st,
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
        if (res[0] == -4) { set_error("k_gotoh: a strip's wait for its neighbour timed out (alignment %d)", t); return -4; }
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
