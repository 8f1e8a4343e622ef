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
//   k_gotoh_tb   traceback (:316-438) over LDS windows, one wave walking
//                runs of one move (a ballot per run).
//   k_lev_prep / k_lev  (the consensus-distance filter only, remap.py:249-251)
//                the relevant seed cut from the traceback's output and its
//                edit distance to the relevant consensus, bit-parallel, in
//                strips of 64 pattern blocks (see the section below).
// The planes are stored anti-diagonal-major over the (m+2) x (n+2) grid
// (doff[s] = first byte of diagonal s, cells by row i), so a step's plane
// bytes are consecutive; they are written and read through buffer
// resources: the diagonal base is a scalar offset, a lane's row its vector
// offset, and a lane with no cell this step points past the buffer (the
// hardware drops the store / returns 0) instead of branching.
// Bit-for-bit specification: oracle/og_gotoh.c.
#include <limits.h>

#include <atomic>
#include <functional>
#include <memory>
#include <thread>
#include <system_error>
#include <algorithm>
#include <mutex>
#include <type_traits>
#include <unordered_map>
#include <utility>
#include <vector>

#include "mh_internal.h"

namespace mh {

constexpr int G_INF = INT_MAX;
constexpr int G_HUGE = 1 << 29;
enum { GA = 1, GB = 2, GC = 4, GD = 8, GE_ = 16, GF = 32, GG = 64 };
constexpr int GOTOH_THREADS = 1024;        // k_gotoh_tb
constexpr int GBLK = 32;                   // boundary columns published / awaited at a time
constexpr int BBLK = 16;                   // the same in k_gotoh_bwd (5 register arrays of it)
constexpr uint32_t GOOB = 0x80000000u;     // a buffer offset past every plane (planes < 2 GiB)
// traceback window: TBD anti-diagonals x TBR rows (a window twice as deep
// in diagonals, for the mostly diagonal paths, measured no faster: the walk
// is bound by its serial LDS reads, not by the window loads)
constexpr int TBD = 128, TBR = 128;
constexpr size_t TB_LDS = (size_t)TBD * TBR + TBR + TBD;   // window + both sequences' characters

__host__ __device__ inline size_t gotoh_al16(size_t x) { return (x + 15) & ~(size_t)15; }

typedef unsigned int g4u __attribute__((ext_vector_type(4)));

struct GotohArgs {
    const int8_t *a;      // seq1 codes, m
    const int8_t *b;      // seq2 codes, n
    int m, n, L;
    const int *mat;       // L x L
    const int8_t *prof;   // L x prof_width(n): the score profile
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

// the strips of a batch in ticket order: tick[u] = (alignment, the strip's
// index in the pass's dependency order), longest remaining critical path
// first (see mh_gotoh_align_batch)
struct GotohStrips {
    const GotohArgs *args;
    const int2 *tick;
    int strips;
    int *ticket;                  // [0] fwd, [1] bwd
    // diagnostics (MH_GOTOH_STAMPS=path, else null): per ticket and block,
    // the shader clock before and after the block's wait, fwd then bwd
    unsigned long long *stamps;
    int stamp_blocks;
    // a wait longer than this many ticks of the 100 MHz s_memrealtime clock
    // is declared broken (the host retries the batch once)
    unsigned long long wait_ticks;
};

// a diagnostic clock stamp (lane 0 stores it)
__device__ __forceinline__ void stamp(const GotohStrips &S, int pass, int u, int blk, int which)
{
    if (S.stamps == nullptr || blk >= S.stamp_blocks) return;
    const unsigned long long now = clock64();
    if (threadIdx.x == 0)
        S.stamps[(((size_t)pass * S.strips + u) * S.stamp_blocks + blk) * 2 + which] = now;
}

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

// default wait limit: 20 s of the 100 MHz real-time clock, far past any
// legitimate wait (a strip waits for the strip above it, which holds a
// lower ticket and is resident or done), also on a GPU shared by several
// processes or running at a throttled clock
constexpr unsigned long long GWAIT_TICKS = 20ull * 100000000ull;

// boundary cells: device-coherent loads / stores (another strip, on any XCD,
// reads them while this launch runs)
// through global (not flat) instructions: a flat access also counts in
// lgkmcnt, so every later LDS wait would wait for the store's round trip
template <class T>
__device__ __forceinline__ T dev_load(const T *p)
{
    return __hip_atomic_load((const __attribute__((address_space(1))) T *)p, __ATOMIC_RELAXED,
                             __HIP_MEMORY_SCOPE_AGENT);
}
template <class T>
__device__ __forceinline__ void dev_store(T *p, T v)
{
    __hip_atomic_store((__attribute__((address_space(1))) T *)p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// the strip of ticket u: (alignment, index in the pass's dependency order)
__device__ __forceinline__ void strip_of(const GotohStrips &S, int u, int &t, int &q)
{
    const int2 x = S.tick[u];
    t = __builtin_amdgcn_readfirstlane(x.x);
    q = __builtin_amdgcn_readfirstlane(x.y);
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
// outlasts S.wait_ticks of real time sets flags[0] and gives up, so a broken
// protocol ends the launch with an error instead of hanging.
template <class T, class Tag>
__device__ __forceinline__ T poll_block(const T *p, int lane, bool has, Tag tagged, int *flags,
                                        unsigned long long wait_ticks)
{
    T v{};
    unsigned long long t0 = 0;
    for (int it = 0;; ++it) {
        if (has) v = dev_load(p + lane);
        if (__builtin_amdgcn_ballot_w64(has && !tagged(v)) == 0) return v;
        // the clock is read every 64 polls (every poll under a short test limit)
        if ((it & 63) == 0 || wait_ticks < 4096) {
            const unsigned long long now = __builtin_amdgcn_s_memrealtime();
            if (it == 0) t0 = now;
            if (now - t0 > wait_ticks || __builtin_amdgcn_readfirstlane(dev_load(flags))) {
                dev_store(flags, 1);
                return v;
            }
        }
        __builtin_amdgcn_s_sleep(2);
    }
}

// The score profile: row c holds the score of seq1 code c against every
// column of seq2 (mat[c][b[j - 1]] at c * PW + PROF_PAD + j; zero outside
// 1..n), so a lane at column j reads its score at a fixed per-lane base + t.
constexpr int PROF_PAD = 128;                       // >= 64 columns before 1 and 96 after n
// Profiles up to this stay in LDS.  A larger one costs residency (one
// 64-lane strip per workgroup: a 48 KiB profile leaves 3 strips per CU), and
// the profile streamed from global memory one block ahead is then faster:
// C4-all's pairs without SARS-CoV-2 (HCV seeds, 48 KiB profiles) 25 -> 12 ms
// of k_gotoh_fwd, HIV-only pairs (<= 15 KiB) equal either way
// (profiles/r06/diag/profile_lds.txt).
constexpr size_t GPROF_LDS_MAX = 16 * 1024;
__host__ __device__ inline int prof_width(int n) { return (int)gotoh_al16((size_t)n + 2 * PROF_PAD); }

// unrolled calls f(integral_constant<int, Q>) for Q = 0 .. N - 1
template <class F, int... Q>
__device__ __forceinline__ void unroll_seq(F &&f, std::integer_sequence<int, Q...>)
{
    (f(std::integral_constant<int, Q>{}), ...);
}
template <int N, class F>
__device__ __forceinline__ void unroll(F &&f)
{
    unroll_seq(f, std::make_integer_sequence<int, N>{});
}

// lane l <- lane l + 1; lane 63 <- x: after GBLK steps lanes 64 - GBLK ..
// 63 hold lane 63's values of the block's steps in order
__device__ __forceinline__ int shift_in63(int x, int reg)
{
    return __builtin_amdgcn_update_dpp(x, reg, 0x130, 0xF, 0xF, false);
}

// Cost assignment of one strip.  Every cell's seven tie bits go to ONE plane
// byte, stored one step late: at step t lane l holds abc of (i, j - 1) from
// the step before, computes fg of (i, j - 1) itself (from cell (i, j)) and
// gets de of (i, j - 1) from the lane below (cell (i + 1, j - 1)) by a lane
// shift.  The strip's last row gets its de bits from the next strip's first
// lane, which stores them in a side row (rowde).
//
// The steps run in blocks of GBLK.  At a block's start the row above's
// cells for its columns go to LDS (every lane reads step q's cell there, a
// broadcast), and the plane bases of its steps to lanes 0..31 (read back by
// lane index); lane 63's cells of the block's steps are shifted into lanes
// 32..63 as they come and published to the strip below by one store at the
// block's end.  Lanes off the grid (a column below 0 or above n, a row above
// m) compute garbage instead of testing their column: off-grid values only
// ever flow to off-grid cells (a lane's inputs are its own previous column
// and the lane above's same column) and the stores test their cell.  So a
// block away from the columns 0, 1 and n (the bulk of the grid) needs no
// per-lane test at all (EDGE false), and only the first strip (row 0) and
// the last (row m) carry their own few (TL).
template <bool PL>   // the score profile in LDS (else read from global memory)
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
    const int PW = prof_width(n);
    int2 *brd = (int2 *)gsm;                        // the row above at the block's columns
    int8_t *lprof = (int8_t *)(gsm + sizeof(int2) * GBLK);
    if (PL) {
        const uint4 *src = (const uint4 *)uni(A.prof);
        for (int x = lane; x < L * PW / 16; x += 64) ((uint4 *)lprof)[x] = src[x];
        __syncthreads();
    }
    const int8_t *prof = PL ? lprof : (const int8_t *)(const __attribute__((address_space(1))) int8_t *)uni(A.prof);
    const int ns = (m + 1 + 63) / 64;
    const int W1 = n + 1;
    const int64_t cells = (int64_t)(m + 2) * (n + 2);
    const __amdgpu_buffer_rsrc_t rbits = brsrc(A.bits, (uint32_t)cells);
    const __amdgpu_buffer_rsrc_t rcol = brsrc(A.lastcol, 4u * (m + 1)), rrow = brsrc(A.lastrow, 4u * (n + 1));
    const int i = 64 * k + lane;
    const bool rowok = i <= m;
    const int code = (i >= 1 && rowok) ? A.a[i - 1] : 0;
    const int prow = code * PW + PROF_PAD - lane;   // + t: the score of column t - lane
    const bool produce = k + 1 < ns, consume = k > 0;
    const bool tl = k == 0 || !produce;             // the first or the last strip
    const unsigned long long *above = A.brow1 + (size_t)(k - 1) * W1;   // row 64k - 1
    unsigned long long *below = A.brow1 + (size_t)k * W1;
    // de bits of row 64k - 1 (the strip above's last row), by n - column
    const __amdgpu_buffer_rsrc_t rside = brsrc(A.rowde + (size_t)(k - 1) * W1, consume ? (uint32_t)W1 : 0u);
    const uint32_t plane_off = rowok ? (uint32_t)i : GOOB;
    const uint32_t col_off = rowok ? 4u * (uint32_t)i : GOOB;
    const int de_keep = i < m ? 0x7F : 0;           // row m takes no de bits from below
    const bool top = i == 0;
    const bool left_p = glob && !top;               // column 0 holds P (global) or 0
    const int *flags = A.flags;
    const uint32_t tag = strip_tag(k);
    // this lane's cell of the last step, (i, j - 1), and R(i - 1, j - 1), the
    // row above one step ago.  Before column 0 they start huge: the values
    // off the grid to the left then stay far above every real one, so that
    // a global alignment's column 0 (R = P, Q infinite, no c tie) needs no
    // test of its own (G_HUGE + 64 steps of drift stays below G_INF)
    int Rme = G_HUGE, Pme = G_HUGE, Qme = G_HUGE;
    int Rdg = G_HUGE;
    int abcp = 0;                             // abc of (i, j - 1), stored this step
    int pR = 0, pP = 0;                       // lanes 32..63: lane 63's R, P at the block's steps
    // !PL: a block's 32 profile bytes of this lane come from 9 aligned dwords
    // loaded one block ahead through a buffer resource and realigned once per
    // block (a byte load per step was a FLAT load, and its wait, vmcnt(0),
    // also waited for every plane store before it)
    const __amdgpu_buffer_rsrc_t rprof = brsrc(PL ? nullptr : (const void *)uni(A.prof),
                                               PL ? 0u : (uint32_t)(L * PW));
    const uint32_t pa = (uint32_t)prow & ~3u, psh = (uint32_t)prow & 3u;
    g4u nx0 = {0, 0, 0, 0}, nx1 = {0, 0, 0, 0};
    uint32_t nx2 = 0;
    auto prof_fetch = [&](int tb) {
        nx0 = __builtin_amdgcn_raw_buffer_load_b128(rprof, pa + (uint32_t)tb, 0, 0);
        nx1 = __builtin_amdgcn_raw_buffer_load_b128(rprof, pa + (uint32_t)tb + 16u, 0, 0);
        nx2 = __builtin_amdgcn_raw_buffer_load_b32(rprof, pa + (uint32_t)tb + 32u, 0, 0);
    };
    if (!PL) prof_fetch(0);
    for (int t0 = 0; t0 <= n + 64; t0 += GBLK) {
        stamp(S, 0, u, t0 / GBLK, 0);
        uint32_t pb[8];                           // !PL: profile bytes t0 .. t0 + 31 of this lane
        if (!PL) {
            const uint32_t c[9] = {nx0.x, nx0.y, nx0.z, nx0.w, nx1.x, nx1.y, nx1.z, nx1.w, nx2};
            for (int x = 0; x < 8; ++x) pb[x] = __builtin_amdgcn_alignbyte(c[x + 1], c[x], psh);
            if (t0 + GBLK <= n + 64) prof_fetch(t0 + GBLK);
        }
        int aR = 0, aP = G_INF;
        if (consume && t0 <= n) {
            // this block of the row above: poll its cells until they carry
            // the strip above's tag
            const uint32_t want = strip_tag(k - 1);
            const unsigned long long w = poll_block(above + t0, lane, lane < GBLK && t0 + lane < W1,
                                                    [&](unsigned long long x) { return rp_tag(x) == want; },
                                                    (int *)flags, S.wait_ticks);
            aR = rp_r(w);
            aP = rp_p(w);
        }
        if (lane < GBLK) brd[lane] = make_int2(aR, aP);
        stamp(S, 0, u, t0 / GBLK, 1);
        // lane q: the plane base of the diagonal s - 1 stored at step t0 + q
        int vb1;
        {
            const int64_t sd = (int64_t)64 * k + t0 + lane - 1;
            const int64_t sc = sd < 0 ? 0 : sd;
            vb1 = (int)(doff_of(sc, m + 1, n + 1) - (sc - (n + 1) > 0 ? sc - (n + 1) : 0));
        }
        const int pbase = prow + t0;
        // rowde is stored by n - j (k_gotoh_bwd reads it forward): lane 0 at
        // step t0 + q writes n - t0 - q = side_v + GBLK - 1 - q
        const uint32_t side_v = lane == 0 ? (uint32_t)(n - t0 - (GBLK - 1)) : GOOB;
        const uint32_t side_r = lane == 0 ? (uint32_t)(n - t0) : GOOB;   // a right block: n - t0 - q, exact
        const uint32_t lrow_v = i == m ? 4u * (uint32_t)(t0 - lane) : GOOB;
        const int j0 = t0 - lane;
        // LEFT: a lane may be at column 0; RIGHT: at column n or past it
        // PRED: a lane's column may lie off the grid (its store is dropped)
        // the score of step q: q a constant (the unrolled blocks) from the
        // realigned dwords, else (short rows) a load
        auto score = [&](auto qc) {
            constexpr int Q = decltype(qc)::value;
            if constexpr (PL) return (int)prof[pbase + Q];
            else return (int)__builtin_amdgcn_sbfe(pb[Q >> 2], 8u * (Q & 3), 8u);
        };
        auto step = [&](auto leftc, auto rightc, auto tlc, auto predc, int q, int sc) {
            constexpr bool LEFT = decltype(leftc)::value, RIGHT = decltype(rightc)::value;
            constexpr bool TL = decltype(tlc)::value, PRED = LEFT || RIGHT || decltype(predc)::value;
            const int j = j0 + q;
            const int2 bd = brd[q];
            const int Rup = __builtin_amdgcn_update_dpp(bd.x, Rme, 0x138, 0xF, 0xF, false);
            const int Pup = __builtin_amdgcn_update_dpp(bd.y, Pme, 0x138, 0xF, 0xF, false);
            const int dg = Rdg - sc;
            const int Ru = Rup + v, Rv = Rme + v;
            const int pm = gmin(Pup, Ru), qm = gmin(Qme, Rv);
            int p = uu + pm, qv = uu + qm;
            // de of (i - 1, j) and fg of (i, j - 1); a P or Q of infinity
            // never equals its finite minimum
            const int de = (pm == Pup ? GD : 0) | (pm == Ru ? GE_ : 0);
            int fg = (qm == Qme ? GF : 0) | (qm == Rv ? GG : 0);
            int r = gmin(gmin(dg, p), qv), ctie = r == dg ? GC : 0;
            if constexpr (TL) {   // row 0: P infinite, R the border
                p = top ? G_INF : p;
                r = top ? (glob ? qv : 0) : r;
                ctie = top ? 0 : ctie;
            }
            if constexpr (LEFT) {   // column 0: Q infinite, R the border
                const bool left = j == 0;
                qv = left ? G_INF : qv;
                fg = left ? 0 : fg;
                r = left ? (left_p ? p : 0) : r;
                ctie = left ? 0 : ctie;
            }
            if constexpr (RIGHT) fg = j > n ? 0 : fg;   // no f/g past column n
            const int abc = (r == p ? GA : 0) | (r == qv ? GB : 0) | ctie;
            // the byte of (i, j - 1): its abc (last step), fg (this lane now)
            // and de (the lane below now; the strip's last row: rowde)
            int deb = __builtin_amdgcn_mov_dpp(de, 0x130, 0xF, 0xF, true);
            if constexpr (TL) deb &= de_keep;
            uint32_t off = plane_off;
            if constexpr (PRED) off = (uint32_t)(j - 1) <= (uint32_t)n ? off : GOOB;
            __builtin_amdgcn_raw_buffer_store_b8((uint8_t)(abcp | fg | deb), rbits, off,
                                                 __builtin_amdgcn_readlane(vb1, q), 0);
            // the first lane's de belongs to the strip above's last row
            if constexpr (RIGHT)   // n - t below 0 is past the side row
                __builtin_amdgcn_raw_buffer_store_b8((uint8_t)de, rside, side_r - (uint32_t)q, 0, 0);
            else
                __builtin_amdgcn_raw_buffer_store_b8((uint8_t)de, rside, side_v + (GBLK - 1 - q), 0, 0);
            if constexpr (RIGHT) __builtin_amdgcn_raw_buffer_store_b32(r, rcol, j == n ? col_off : GOOB, 0, 0);
            if constexpr (TL) __builtin_amdgcn_raw_buffer_store_b32(r, rrow, lrow_v + 4 * q, 0, 0);
            abcp = abc;
            Rdg = Rup;
            Rme = r;
            Pme = p;
            Qme = qv;
            pR = shift_in63(r, pR);
            pP = shift_in63(p, pP);
        };
        // the block's kind (every kind unrolled: a slow block anywhere in a
        // strip delays every strip below it)
        const bool left = t0 < 64, right = t0 + GBLK > n;
        constexpr std::true_type Y{};
        constexpr std::false_type N{};
        if (right && left) {   // n < 64 + GBLK - 1: short rows
            if (tl) {
                for (int q = 0; q < GBLK; ++q) step(Y, Y, Y, N, q, prof[pbase + q]);
            } else {
                for (int q = 0; q < GBLK; ++q) step(Y, Y, N, N, q, prof[pbase + q]);
            }
        } else if (right) {
            if (tl) unroll<GBLK>([&](auto qc) { step(N, Y, Y, N, decltype(qc)::value, score(qc)); });
            else unroll<GBLK>([&](auto qc) { step(N, Y, N, N, decltype(qc)::value, score(qc)); });
        } else if (left) {
            // a middle strip of a global alignment: column 0 comes out of
            // the huge start values, only the stores test their column
            if (tl) unroll<GBLK>([&](auto qc) { step(Y, N, Y, N, decltype(qc)::value, score(qc)); });
            else if (glob) unroll<GBLK>([&](auto qc) { step(N, N, N, Y, decltype(qc)::value, score(qc)); });
            else unroll<GBLK>([&](auto qc) { step(Y, N, N, N, decltype(qc)::value, score(qc)); });
        } else {
            if (tl) unroll<GBLK>([&](auto qc) { step(N, N, Y, N, decltype(qc)::value, score(qc)); });
            else unroll<GBLK>([&](auto qc) { step(N, N, N, N, decltype(qc)::value, score(qc)); });
        }
        // the strip's last row (lane 63 at column t - 63) to the strip below
        const int jp = t0 + lane - (64 - GBLK) - 63;
        if (produce && lane >= 64 - GBLK && jp >= 0 && jp <= n) dev_store(below + jp, rp_pack(pR, pP, tag));
    }
}

// Edge assignment of one strip (bottom-up, right to left): lane l at step t
// is at column j = n + 63 - l - t.  Each block of GBLK steps first takes the
// row below's final bits for its steps (polled; to LDS, read back by every
// lane as a broadcast), then computes from the block's plane bytes (loaded
// during the block before, with lane 63's de side bits), then stores the
// block's final bytes: loads and stores never interleave inside a block, so
// no step waits on a store.  Lane 0's results are shifted into lanes 0..31
// as they come and published to the strip above by one store per block.
// As in k_gotoh_fwd, lanes off the grid compute garbage that only reaches
// off-grid cells; a block away from the columns n and below 0 (EDGE false)
// tests nothing per lane, and only the last strip (row m, TL) tests its row.
__global__ __launch_bounds__(64) void k_gotoh_bwd(GotohStrips S)
{
    extern __shared__ __attribute__((aligned(16))) unsigned char gsm[];
    int *bw = (int *)gsm;   // the row below's final abc at the block's steps
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
    const int bnd = A.is_global ? 0 : GC;
    const int i = 64 * k + lane;
    const bool rowok = i <= m, lastr = i == m;
    const bool produce = k > 0, consume = k + 1 < ns;
    const bool tl = !consume;                  // the last strip: row m and past it
    const int *under = A.brow2 + (size_t)(k + 1) * W1;   // row 64k + 64, by tau = n - j
    int *mytop = A.brow2 + (size_t)k * W1;
    // de bits of this strip's last row (stored by the strip below), by n - j
    const __amdgpu_buffer_rsrc_t rside = brsrc(A.rowde + (size_t)k * W1, consume ? (uint32_t)W1 : 0u);
    const uint32_t plane_off = rowok ? (uint32_t)i : GOOB;
    const uint32_t side_off = lane == 63 ? 0u : GOOB;   // + t: lane 63 is at column n - t
    const int *flags = A.flags;
    const int s0 = 64 * k + n + 63;            // the diagonal of step 0
    const int tagk = (k % 0xFFFFFF + 1) << 8;
    int mine = 0;        // final abc of (i, j + 1): this lane, one step ago
    int dnp = 0;         // final abc of (i + 1, j + 1): the lane below, two steps ago
    int pub = 0;         // lanes 0..31: lane 0's final abc at the block's steps (last step in lane 0)
    int cx[BBLK], sx[BBLK], nx[BBLK], nsx[BBLK], ox[BBLK];
    // lane q: the plane base of the diagonal of step t0 + q
    auto bases = [&](int t0b) {
        const int64_t sd = (int64_t)s0 - t0b - lane;
        const int64_t sc = sd < 0 ? 0 : sd;
        return (int)(doff_of(sc, m + 1, n + 1) - (sc - (n + 1) > 0 ? sc - (n + 1) : 0));
    };
    // the plane bytes and lane 63's side bits of steps t0b .. t0b + BBLK - 1
    // (a lane off the grid reads some other byte or 0: it only feeds garbage)
    auto load_block = [&](int t0b, int vb, int *dst, int *dsts) {
        unroll<BBLK>([&](auto qc) {
            constexpr int q = decltype(qc)::value;
            dst[q] = __builtin_amdgcn_raw_buffer_load_b8(rbits, plane_off, __builtin_amdgcn_readlane(vb, q), 0);
            dsts[q] = __builtin_amdgcn_raw_buffer_load_b8(rside, side_off + (uint32_t)t0b + q, 0, 0);
        });
    };
    int vb = bases(0);
    load_block(0, vb, cx, sx);
    for (int t0 = 0; t0 <= n + 63; t0 += BBLK) {
        stamp(S, 1, u, t0 / BBLK, 0);
        // the strip below's first row for this block (lane 63's cells below),
        // tagged with the strip below's tag
        int d = 0;
        if (consume && t0 <= n) {
            const int want = (k + 1) % 0xFFFFFF + 1;
            d = poll_block(under + t0, lane, lane < BBLK && t0 + lane < W1,
                           [&](int w) { return (w >> 8) == want; }, (int *)flags, S.wait_ticks) & 0xFF;
        }
        if (lane < BBLK) bw[lane] = d;
#pragma unroll
        for (int q = 0; q < BBLK; ++q) asm volatile("; touch %0 %1" : "+v"(cx[q]), "+v"(sx[q]));
        stamp(S, 1, u, t0 / BBLK, 1);
        const int vbn = bases(t0 + BBLK);
        load_block(t0 + BBLK, vbn, nx, nsx);
        const int j0 = n + 63 - lane - t0;
        auto step = [&](auto edgec, auto tlc, int q) {
            constexpr bool EDGE = decltype(edgec)::value, TL = decltype(tlc)::value;
            const int j = j0 - q;
            const int dnb = __builtin_amdgcn_update_dpp(bw[q], mine, 0x130, 0xF, 0xF, false);   // (i + 1, j)
            const int c = cx[q] | sx[q];
            int dn = dnb, rt = mine, dgn = dnp;
            if constexpr (EDGE || TL) {
                const bool lastc = EDGE && j == n, lr = TL && lastr;
                dn = lr ? (lastc ? GC : bnd) : dn;
                rt = lastc ? (lr ? GC : bnd) : rt;
                dgn = (lr || lastc) ? ((lr && lastc) ? GC : bnd) : dgn;
            }
            // Altschul-Erickson steps 8-11 of the cell, bitwise: keep a/b/c
            // unless no edge reaches the cell; add a (b) through d (f)
            const int dA = dn & GA, rB = rt & GB, dC = dgn & GC;
            const int c3 = c >> 3, c4 = c >> 4, c5 = c >> 5;
            const int add = (c3 & dA) | (c4 & rB);
            const int keep = (c4 & dA) | (c5 & rB) | dC;
            const int x = (keep ? c : (c & ~(GA | GB | GC))) | add;
            ox[q] = x;
            dnp = dnb;
            mine = x;
            pub = __builtin_amdgcn_update_dpp(x, pub, 0x138, 0xF, 0xF, false);   // lane 0 <- x
        };
        constexpr std::true_type Y{};
        constexpr std::false_type N{};
        const bool edge = t0 < 64 || t0 + BBLK - 1 > n;
        if (tl) {
            if (edge) unroll<BBLK>([&](auto qc) { step(Y, Y, decltype(qc)::value); });
            else unroll<BBLK>([&](auto qc) { step(N, Y, decltype(qc)::value); });
        } else {
            if (edge) unroll<BBLK>([&](auto qc) { step(Y, N, decltype(qc)::value); });
            else unroll<BBLK>([&](auto qc) { step(N, N, decltype(qc)::value); });
        }
        // the block's final bytes; the strip's first row (lane 0) to the strip above
        unroll<BBLK>([&](auto qc) {
            constexpr int q = decltype(qc)::value;
            const int j = j0 - q;
            const uint32_t off = (!edge || (uint32_t)j <= (uint32_t)n) ? plane_off : GOOB;
            __builtin_amdgcn_raw_buffer_store_b8((uint8_t)ox[q], rbits, off, __builtin_amdgcn_readlane(vb, q), 0);
        });
        const int tp = t0 + (BBLK - 1 - lane) - 63;
        if (produce && lane < BBLK && tp >= 0 && tp <= n) dev_store(mytop + tp, tagk | pub);
        unroll<BBLK>([&](auto qc) {
            constexpr int q = decltype(qc)::value;
            cx[q] = nx[q];
            sx[q] = nsx[q];
        });
        vb = vbn;
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
    // stages a TBD x TBR window of abc (diagonals s0 .. s0-TBD+1, rows
    // ii .. ii-TBR+1 of the current cell (ii, jj), which holds every cell the
    // path can reach before it leaves the window) and the TBR / TBD characters of
    // each sequence before ii / jj into LDS; wave 0 walks the window and
    // writes the output characters; repeat.  The gap runs at both ends are
    // written by the whole block.
    uint8_t *win = gsm;
    char *wc1 = (char *)win + TBD * TBR, *wc2 = wc1 + TBR;
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
    // built back to front, reversed by the host; global (not flat) stores:
    // a flat store counts in lgkmcnt too, so the walk's next LDS read of the
    // window waited for the last step's two output stores
    typedef __attribute__((address_space(1))) char gchar;
    typedef const __attribute__((address_space(1))) uint8_t gbyte;
    gchar *r1 = (gchar *)A.out1, *r2 = (gchar *)A.out2;
    gbyte *bits = (gbyte *)A.bits;
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
        for (int x = threadIdx.x; x < TBD * TBR; x += blockDim.x) {
            const int t = x / TBR, r = x % TBR;
            const int sd = s0 - t, i = i0 - r, j = sd - i;
            uint8_t vv = 0;
            if (i >= 1 && j >= 1 && j <= n) vv = bits[dbase(sd, m, n) + i];   // (r <= t on the path)
            win[x] = vv;
        }
        for (int x = threadIdx.x; x < TBD; x += blockDim.x) {
            if (x < TBR) wc1[x] = i0 - 1 - x >= 0 ? A.s1[i0 - 1 - x] : 0;
            wc2[x] = j0 - 1 - x >= 0 ? A.s2[j0 - 1 - x] : 0;
        }
        __syncthreads();
        if (threadIdx.x < 64) {
            // Wave 0 walks by runs: a cell's move is up (GA), else left (GB),
            // else diagonal (GC), and a run of one move is found in one LDS
            // round trip: lane l reads the l-th cell of the run that each of
            // the three moves would make from the current cell (its l = 0 cell
            // is the current one for all three) and both characters; the
            // current cell's move picks the run, and a ballot its length (the
            // first lane whose cell moves otherwise, or the window's, the
            // grid's or the wave's end).  The lanes write the run's output
            // characters together.
            const int lane = threadIdx.x;
            int i = i0, j = j0, len = tb_len, status = 0;
            while (i > 0 && j > 0) {
                const int t = s0 - (i + j), r = i0 - i, c = j0 - j;
                if (t >= TBD || r >= TBR || c >= TBD) break;
                // cells available to each run from here (the current one included)
                const int nd = min(min((TBD - 1 - t) / 2, TBR - 1 - r), min(TBD - 1 - c, min(i, j) - 1)) + 1;
                const int nu = min(min(TBD - 1 - t, TBR - 1 - r), i - 1) + 1;
                const int nl = min(min(TBD - 1 - t, TBD - 1 - c), j - 1) + 1;
                const uint8_t xd = lane < nd ? win[(t + 2 * lane) * TBR + r + lane] : 0;
                const uint8_t xu = lane < nu ? win[(t + lane) * TBR + r + lane] : 0;
                const uint8_t xl = lane < nl ? win[(t + lane) * TBR + r] : 0;
                const int ch1 = r + lane < TBR ? wc1[r + lane] : 0;
                const int ch2 = c + lane < TBD ? wc2[c + lane] : 0;
                const int x = __builtin_amdgcn_readfirstlane((int)xd);
                if (!(x & (GA | GB | GC))) { status = -1; break; }
                const bool up = x & GA, left = !up && (x & GB);
                int run;
                if (up) {
                    const uint64_t stop = __builtin_amdgcn_ballot_w64(lane >= min(nu, 64) || !(xu & GA));
                    run = (int)__builtin_ctzll(stop | (1ull << 63));
                    run = run < 1 ? 1 : run;
                    if (lane < run) { r1[len + lane] = (char)ch1; r2[len + lane] = '-'; }
                    i -= run;
                } else if (left) {
                    const uint64_t stop =
                        __builtin_amdgcn_ballot_w64(lane >= min(nl, 64) || (xl & GA) || !(xl & GB));
                    run = (int)__builtin_ctzll(stop | (1ull << 63));
                    run = run < 1 ? 1 : run;
                    if (lane < run) { r1[len + lane] = '-'; r2[len + lane] = (char)ch2; }
                    j -= run;
                } else {
                    const uint64_t stop =
                        __builtin_amdgcn_ballot_w64(lane >= min(nd, 64) || (xd & (GA | GB)) || !(xd & GC));
                    run = (int)__builtin_ctzll(stop | (1ull << 63));
                    run = run < 1 ? 1 : run;
                    if (lane < run) { r1[len + lane] = (char)ch1; r2[len + lane] = (char)ch2; }
                    i -= run;
                    j -= run;
                }
                len += run;
            }
            if (lane == 0) { tb_ii = i; tb_jj = j; tb_len = len; tb_status = status; }
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

// ---------------------------------------------------------------------------
// The distance filter's edit distances on the device (remap.py:249-251):
// Levenshtein.distance(extract_relevant_seed(aligned_conseq, aligned_seed),
// relevant) for every alignment of the batch, straight from k_gotoh_tb's
// output (nothing is fetched but one distance per alignment).
//
// The aligned strings are stored back to front, and an edit distance is the
// same for both strings reversed, so the pattern is taken as it lies: seq1's
// characters over the span of seq2's non-gap columns, gaps dropped
// (k_lev_prep), and the text (relevant) is uploaded reversed.  k_lev runs the
// bit-parallel recurrence of Myers / Hyyro (as mh_levenshtein on the host):
// pattern rows in 64-row blocks, one block per lane, 64 blocks per strip,
// one wave per strip; lane l is at column t - l at step t, so the horizontal
// delta into its block's top row is the lane above's output of the step
// before, one DPP lane shift.  A strip's last lane hands its bottom deltas
// to the next strip through global memory in blocks of GBLK columns, each
// word carrying a tag bit, and strips are taken by ticket in their
// dependency order (as k_gotoh_fwd's).  The last block is padded to 64 rows
// that match every character; their vertical deltas in the last column are
// taken off the bottom score at the end.
// ---------------------------------------------------------------------------
struct LevArgs {
    const char *o1, *o2;   // k_gotoh_tb's aligned seq1 / seq2 (reversed)
    const int *result;     // k_gotoh_tb's [status, score, length]
    const uint8_t *text;   // the second string, reversed (n bytes)
    int n;
    uint8_t *pcode;        // the pattern's codes (<= m + 64 bytes)
    int *bnd;              // (strips - 1) x n boundary words: delta bits | 4
    int *meta;             // [0] pattern length, [1] status
    int *res;              // [0] status, [1] score, [2] distance
};

struct LevBatch {
    const LevArgs *args;
    const int2 *tick;      // (alignment, strip) in ticket order
    int strips;
    int *ticket;
    const uint8_t *lut;    // character -> 1 + alphabet code, 0 (none)
    int ncodes;            // alphabet size + 1
    int *flags;            // [0] a wait timed out
    unsigned long long wait_ticks;
};

constexpr int LEV_STRIP_ROWS = 64 * 64;

// One wave per alignment: the span of seq2's non-gap columns, and seq1's
// characters over it without gaps, as codes.
__global__ __launch_bounds__(64) void k_lev_prep(LevBatch B)
{
    const LevArgs A = B.args[blockIdx.x];
    const int lane = threadIdx.x;
    const int status = A.result[0], score = A.result[1], len = A.result[2];
    typedef const __attribute__((address_space(1))) char gcc;
    const gcc *o1 = (const gcc *)A.o1, *o2 = (const gcc *)A.o2;
    int lo = len, hi = -1;
    if (status == 0) {
        for (int k0 = 0; k0 < len; k0 += 64) {
            const int k = k0 + lane;
            const uint64_t b = __builtin_amdgcn_ballot_w64(k < len && o2[k] != '-');
            if (b) { lo = k0 + __builtin_ctzll(b); break; }
        }
        for (int k0 = len - 1; k0 >= 0; k0 -= 64) {
            const int k = k0 - lane;
            const uint64_t b = __builtin_amdgcn_ballot_w64(k >= 0 && o2[k] != '-');
            if (b) { hi = k0 - __builtin_ctzll(b); break; }
        }
    }
    int base = 0;
    if (status == 0 && lo <= hi) {
        const uint64_t below = lane ? ~0ull >> (64 - lane) : 0ull;
        for (int k0 = lo; k0 <= hi; k0 += 64) {
            const int k = k0 + lane;
            const char c = k <= hi ? o1[k] : '-';
            const uint64_t b = __builtin_amdgcn_ballot_w64(c != '-');
            if (c != '-') A.pcode[base + __builtin_popcountll(b & below)] = B.lut[(uint8_t)c];
            base += __builtin_popcountll(b);
        }
    }
    if (lane == 0) {
        // -2: no non-gap column (extract_relevant_seed's match is None)
        const int st = status == -4 ? -4 : status ? -1 : lo > hi ? -2 : 0;
        A.meta[0] = base;
        A.meta[1] = st;
        A.res[0] = st;
        A.res[1] = score;
        A.res[2] = base == 0 ? A.n : A.n == 0 ? base : -1;
    }
}

// the Myers / Hyyro step of one 64-row block at one column: eq the block's
// match bits for the column's character, (hp, hn) the horizontal delta into
// its top row; returns the delta out of its bottom row (bit 0: +1, bit 1: -1)
__device__ __forceinline__ int lev_step(uint64_t eq, int hin, uint64_t &Pv, uint64_t &Mv)
{
    const uint64_t hp = (uint64_t)(hin & 1), hn = (uint64_t)((hin >> 1) & 1);
    const uint64_t Xv = eq | Mv;
    const uint64_t Eq = eq | hn;
    const uint64_t Xh = (((Eq & Pv) + Pv) ^ Pv) | Eq;
    uint64_t Ph = Mv | ~(Xh | Pv);
    uint64_t Mh = Pv & Xh;
    const int out = (int)(Ph >> 63) | (int)(Mh >> 63) << 1;
    Ph = (Ph << 1) | hp;
    Mh = (Mh << 1) | hn;
    Pv = Mh | ~(Xv | Ph);
    Mv = Ph & Xv;
    return out;
}

__global__ __launch_bounds__(64) void k_lev(LevBatch B)
{
    extern __shared__ __attribute__((aligned(16))) unsigned char lsm[];
    uint64_t *peq = (uint64_t *)lsm;                  // [code][lane]
    uint8_t *lut = lsm + (size_t)B.ncodes * 64 * 8;   // 256 bytes
    const int lane = threadIdx.x;
    __shared__ int tk;
    if (lane == 0) tk = atomicAdd(B.ticket, 1);
    for (int x = lane; x < 256; x += 64) lut[x] = B.lut[x];
    __syncthreads();
    const int u = tk;
    if (u >= B.strips) return;
    int t, s;
    {
        const int2 x = B.tick[u];
        t = __builtin_amdgcn_readfirstlane(x.x);
        s = __builtin_amdgcn_readfirstlane(x.y);
    }
    const LevArgs A = B.args[t];
    const int mlen = __builtin_amdgcn_readfirstlane(A.meta[0]);
    const int st = __builtin_amdgcn_readfirstlane(A.meta[1]);
    const int n = A.n;
    if (st != 0 || mlen == 0 || n == 0) return;   // k_lev_prep wrote the result
    const int nb = (mlen + 63) / 64, nstr = (nb + 63) / 64;
    if (s >= nstr) return;
    const bool last = s == nstr - 1;
    const int b = 64 * s + lane;                      // this lane's block
    const bool blk = b < nb;
    const int lastw = (nb - 1 - 64 * s) < 63 ? nb - 1 - 64 * s : 63;
    const int pad = nb * 64 - mlen;
    const uint64_t padmask = (b == nb - 1 && pad) ? ~0ull << (64 - pad) : 0ull;
    // match bits of this lane's block, one word per code (lane-private column)
    for (int c = 0; c < B.ncodes; ++c) peq[c * 64 + lane] = padmask;
    if (blk) {
        const int r_end = mlen - 64 * b < 64 ? mlen - 64 * b : 64;
        for (int r = 0; r < r_end; ++r) peq[A.pcode[64 * b + r] * 64 + lane] |= 1ull << r;
    }
    uint64_t Pv = ~0ull, Mv = 0;
    const int *prev = s > 0 ? A.bnd + (size_t)(s - 1) * n : nullptr;
    int *mine = last ? nullptr : A.bnd + (size_t)s * n;
    const int steps = n + (last ? lastw : 63);
    typedef const __attribute__((address_space(1))) uint8_t gbyte;
    const gbyte *text = (const gbyte *)A.text;
    // the next block's text codes and boundary words, loaded one block ahead
    int cw_next = lane < GBLK && lane < n ? lut[text[lane]] : 0;
    // (strip 0: every column's delta into row 0 is +1)
    int bw_next = !prev ? 1 : lane < GBLK && lane < n ? dev_load(prev + lane) : 0;
    // cc: the code of this lane's column; eqn: the match bits of the next
    // step, read from LDS a step ahead (the column's code is known then)
    int cc = lane == 0 ? __builtin_amdgcn_readlane(cw_next, 0) : 0;
    uint64_t eqn = peq[cc * 64 + lane];
    int hout = 0, acc = 0, pr = 0;
    for (int t0 = 0; t0 < steps; t0 += GBLK) {
        const int cw = cw_next;
        int bw = bw_next;
        const bool need = lane < GBLK && t0 + lane < n;
        if (prev && __builtin_amdgcn_ballot_w64(need && !(bw & 4)))
            bw = poll_block(prev + t0, lane, need, [](int v) { return (v & 4) != 0; }, B.flags, B.wait_ticks);
        const int t1 = t0 + GBLK + lane;
        cw_next = lane < GBLK && t1 < n ? lut[text[t1]] : 0;
        bw_next = !prev ? 1 : lane < GBLK && t1 < n ? dev_load(prev + t1) : 0;
        // A block where some lane is off its columns (the first 64 steps,
        // the last ones) keeps such a lane's state as it is; elsewhere every
        // lane steps (a lane past the pattern only feeds lanes past it, and
        // a lane's output only reaches the next lane at the same column, so
        // off-grid outputs never meet on-grid cells).
        auto block = [&](auto edge_c) {
            constexpr bool EDGE = decltype(edge_c)::value;
            unroll<GBLK>([&](auto qc) {
                constexpr int q = decltype(qc)::value;
                const uint64_t eq = eqn;
                const int nx = q + 1 < GBLK ? __builtin_amdgcn_readlane(cw, q + 1 < GBLK ? q + 1 : 0)
                                            : __builtin_amdgcn_readlane(cw_next, 0);
                cc = from_prev_lane(nx, cc);
                eqn = peq[cc * 64 + lane];
                const int h0 = __builtin_amdgcn_readlane(bw, q) & 3;
                const int hin = from_prev_lane(h0, hout);
                if constexpr (EDGE) {
                    uint64_t nP = Pv, nM = Mv;
                    hout = lev_step(eq, hin, nP, nM);
                    const bool act = blk && (uint32_t)(t0 + q - lane) < (uint32_t)n;
                    Pv = act ? nP : Pv;
                    Mv = act ? nM : Mv;
                    acc += act ? (hout & 1) - (hout >> 1) : 0;
                } else {
                    hout = lev_step(eq, hin, Pv, Mv);
                    acc += (hout & 1) - (hout >> 1);
                }
                pr = shift_in63(hout, pr);
            });
        };
        if (t0 < 64 || t0 + GBLK > n) block(std::true_type{});
        else block(std::false_type{});
        if (!last) {
            // lanes 64 - GBLK .. 63 hold lane 63's outputs of the block's steps
            const int col = t0 + (lane - (64 - GBLK)) - 63;
            if (lane >= 64 - GBLK && col >= 0 && col < n) dev_store(mine + col, (pr & 3) | 4);
        }
    }
    // lane lastw of the last strip: the bottom row's score
    if (last && lane == lastw) {
        const int corr = __builtin_popcountll(Pv & padmask) - __builtin_popcountll(Mv & padmask);
        A.res[2] = nb * 64 + acc - corr;
    }
}

static size_t align16(size_t x) { return (x + 15) & ~(size_t)15; }

// Uploaded "in" blocks, one per distinct sequence (a filter batch aligns K
// consensuses against the same K seeds: K + K blocks, not 2 K^2): seq1's
// codes and text; seq2's codes, text and score profile.  Per alignment an
// "out" block (output strings, result: what is fetched) and a "work" block
// (diagonal buffers, last row / column and the three tie planes, zeroed on
// the device).
static size_t gotoh_in1_bytes(int m) { return align16(m + 8) + align16(m + 1); }
static size_t gotoh_in2_bytes(int n, int L) { return align16(n + 8) + align16(n + 1) + (size_t)L * prof_width(n); }

// distinct pointers of ptr[0 .. count) in first-seen order: idx[t] = the
// distinct index of ptr[t]; returns the distinct pointers
static std::vector<const char *> distinct_ptrs(int count, const char *const *ptr, std::vector<int> &idx)
{
    std::vector<const char *> uniq;
    std::unordered_map<const char *, int> at;
    idx.resize((size_t)count);
    for (int t = 0; t < count; ++t) {
        auto it = at.emplace(ptr[t], (int)uniq.size());
        if (it.second) uniq.push_back(ptr[t]);
        idx[(size_t)t] = it.first->second;
    }
    return uniq;
}

static size_t gotoh_out_bytes(int m, int n)            // aligned strings, result (fetched)
{
    return 2 * align16(m + n + 1) + 64;
}

// fn(t) for t = 0 .. count - 1 on up to 16 host threads
static void gotoh_par(int count, const std::function<void(int)> &fn)
{
    const int nt = std::max(1, std::min({count, 16, (int)std::thread::hardware_concurrency()}));
    std::atomic<int> next(0);
    auto run = [&]() { for (int t; (t = next.fetch_add(1)) < count;) fn(t); };
    std::vector<std::thread> th;
    try {
        for (int k = 1; k < nt; ++k) th.emplace_back(run);
    } catch (const std::system_error &) {
        // fewer threads: the ones started and this one share the work
    }
    run();
    for (auto &x : th) x.join();
}

// the zeroed work block (without the tie planes, which k_gotoh_fwd writes
// in full -- every cell (i <= m, j <= n) -- before anything reads them)
static size_t gotoh_work_bytes(int m, int n)
{
    const size_t strips = (size_t)(m + 1 + 63) / 64;
    return align16(sizeof(int) * (m + 2)) + align16(sizeof(int) * (n + 2)) + align16(8 * strips * (n + 1)) +
           align16(sizeof(int) * strips * (n + 1)) + align16(strips * (n + 1)) + 16;
}

// Retained scratch above an eighth of the device's memory (36 GB of an
// MI355X's 288) is released after the call: one very long alignment must not
// pin device memory for the rest of the session, but a batch the size of
// C4-all's filter (16 GB of tie planes) keeps its buffer -- allocating it
// afresh cost 0.4 s per call on a box's first processes (fresh VRAM pages)
static size_t gotoh_keep_bytes()
{
    static const size_t keep = [] {
        size_t fr = 0, tot = 0;
        if (hipMemGetInfo(&fr, &tot) != hipSuccess || tot == 0) return (size_t)1 << 30;
        return std::max((size_t)1 << 30, tot / 8);
    }();
    return keep;
}

// lev_text non-null: the filter's edit distances instead of the aligned
// strings (out1 / out2 / cap unused): lev_dist[t] = the distance between
// alignment t's relevant seed and lev_text[t] (status -2: no non-gap column)
static int gotoh_batch_once(Ctx &c, int count, const char *const *s1, const char *const *s2, int gop,
                            int gep, int is_global, const char *alphabet, const int *matrix,
                            char *const *out1, char *const *out2, const int *cap, int *score,
                            int *status, unsigned long long wait_ticks, const char *const *lev_text,
                            int *lev_dist)
{
    const bool lev = lev_text != nullptr;
    const int L = (int)strlen(alphabet);
    if (count < 0 || L == 0 || L > 64) { set_error("mh_gotoh_align: bad arguments"); return -3; }
    if (count == 0) return 0;
    int code[256];
    for (int k = 0; k < 256; ++k) code[k] = -1;
    for (int k = 0; k < L; ++k) code[(unsigned char)alphabet[k]] = k;
    int64_t mat_max = 0;
    for (int x = 0; x < L * L; ++x) mat_max = std::max<int64_t>(mat_max, std::abs((int64_t)matrix[x]));
    if (mat_max > 127) { set_error("mh_gotoh_align: scores outside -127..127"); return -3; }
    if (gop < 0 || gep < 0 || gop > (1 << 16) || gep > (1 << 16)) { set_error("mh_gotoh_align: bad gap penalties"); return -3; }
    std::vector<int> ms(count), ns(count), nt(count, 0), lstr(count, 0);
    std::vector<size_t> oo(count + 1, 0), work(count + 1, 0), planes(count + 1, 0);
    for (int t = 0; t < count; ++t)
        if (!s1[t] || !s2[t] || (lev ? !lev_text[t] : !out1[t] || !out2[t])) {
            set_error("mh_gotoh_align: null argument");
            return -3;
        }
    // the distinct sequences (by pointer): lengths and the alphabet check of
    // each on host threads; the first offending character (by alignment,
    // then position) is reported
    std::vector<int> i1, i2, i3;
    const std::vector<const char *> u1 = distinct_ptrs(count, s1, i1), u2 = distinct_ptrs(count, s2, i2);
    const std::vector<const char *> u3 = lev ? distinct_ptrs(count, lev_text, i3) : std::vector<const char *>();
    const int n1 = (int)u1.size(), n2 = (int)u2.size(), n3 = (int)u3.size();
    std::vector<int> len1(n1), len2(n2), len3(n3), bad1(n1, -1), bad2(n2, -1);
    gotoh_par(n1 + n2 + n3, [&](int x) {
        if (x < n1) {
            const char *p = u1[x];
            len1[x] = (int)strlen(p);
            for (int i = 0; i < len1[x] && bad1[x] < 0; ++i)
                if (code[(unsigned char)p[i]] < 0) bad1[x] = (unsigned char)p[i];
        } else if (x < n1 + n2) {
            const int y = x - n1;
            const char *p = u2[y];
            len2[y] = (int)strlen(p);
            for (int j = 0; j < len2[y] && bad2[y] < 0; ++j)
                if (code[(unsigned char)p[j]] < 0) bad2[y] = (unsigned char)p[j];
        } else {
            len3[x - n1 - n2] = (int)strlen(u3[x - n1 - n2]);
        }
    });
    std::vector<int> badc(count, -1);
    for (int t = 0; t < count; ++t) {
        ms[t] = len1[i1[t]];
        ns[t] = len2[i2[t]];
        if (lev) nt[t] = len3[i3[t]];
        badc[t] = bad1[i1[t]] >= 0 ? bad1[i1[t]] : bad2[i2[t]];
    }
    // in blocks: [distinct seq1][distinct seq2][distinct texts]
    std::vector<size_t> io1(n1 + 1, 0), io2(n2 + 1, 0), io3(n3 + 1, 0);
    for (int x = 0; x < n1; ++x) io1[x + 1] = io1[x] + gotoh_in1_bytes(len1[x]);
    io2[0] = io1[n1];
    for (int y = 0; y < n2; ++y) io2[y + 1] = io2[y] + gotoh_in2_bytes(len2[y], L);
    io3[0] = io2[n2];
    for (int z = 0; z < n3; ++z) io3[z + 1] = io3[z] + align16((size_t)len3[z] + 16);
    const size_t io_total = io3[n3];
    for (int t = 0; t < count; ++t) {
        if (ms[t] == 0 || ns[t] == 0 || (!lev && cap[t] < ms[t] + ns[t] + 1)) {
            set_error("mh_gotoh_align: bad arguments (alignment %d)", t);
            return -3;
        }
        if (badc[t] >= 0) { set_error("mh_gotoh_align: '%c' not in alphabet", badc[t]); return -3; }
        oo[t + 1] = oo[t] + gotoh_out_bytes(ms[t], ns[t]);
        // boundary cells carry R and P in 26 bits (k_gotoh_fwd rp_pack)
        if ((int64_t)(ms[t] + ns[t] + 2) * (mat_max + gop + gep + 1) >= ((int64_t)1 << 24)) {
            set_error("mh_gotoh_align: alignment %d too long for the score range", t);
            return -3;
        }
        if ((uint64_t)(ms[t] + 2) * (uint64_t)(ns[t] + 2) >= (uint64_t)GOOB) {
            set_error("mh_gotoh_align: alignment %d too large (%d x %d)", t, ms[t], ns[t]);
            return -3;
        }
        // the pattern is at most seq1 long: its strips of LEV_STRIP_ROWS rows
        lstr[t] = (ms[t] + LEV_STRIP_ROWS - 1) / LEV_STRIP_ROWS;
        work[t + 1] = work[t] + gotoh_work_bytes(ms[t], ns[t]) +
                      (lev ? align16((size_t)ms[t] + 64) + align16(sizeof(int) * (size_t)(lstr[t] - 1) * nt[t]) + 16
                           : 0);
        planes[t + 1] = planes[t] + align16((size_t)(ms[t] + 2) * (ns[t] + 2));
    }
    // strips in ticket order, the longest remaining critical path first:
    // strip q of an alignment (q-th in its pass's dependency order) still has
    // (strips - 1 - q) strips after it, each starting about GLAG steps after
    // the one before (the 64-lane skew plus a block), and then its own n + 64
    // steps.  A strip's predecessor always has the longer path, so it holds
    // a lower ticket (every wait is for a strip already started), and a
    // resident wave rarely waits: the strips that can run next across all the
    // alignments are the ones handed out (alignment-major tickets left the
    // later strips of a long alignment resident and idle, ~half the waves)
    constexpr int64_t GLAG = 128;
    std::vector<int2> tick;
    std::vector<int64_t> key;
    for (int t = 0; t < count; ++t) {
        const int nsx = (ms[t] + 1 + 63) / 64;
        for (int q = 0; q < nsx; ++q) {
            tick.push_back(make_int2(t, q));
            key.push_back((int64_t)(nsx - 1 - q) * GLAG + ns[t] + 64);
        }
    }
    {
        std::vector<int> idx(tick.size());
        for (size_t x = 0; x < idx.size(); ++x) idx[x] = (int)x;
        std::stable_sort(idx.begin(), idx.end(), [&](int x, int y) { return key[(size_t)x] > key[(size_t)y]; });
        std::vector<int2> sorted(tick.size());
        for (size_t x = 0; x < idx.size(); ++x) sorted[x] = tick[(size_t)idx[x]];
        tick.swap(sorted);
    }
    // the edit distances' strips, in the same critical-path order
    std::vector<int2> ltick;
    if (lev) {
        std::vector<int64_t> lkey;
        for (int t = 0; t < count; ++t)
            for (int q = 0; q < lstr[t]; ++q) {
                ltick.push_back(make_int2(t, q));
                lkey.push_back((int64_t)(lstr[t] - 1 - q) * GLAG + nt[t] + 64);
            }
        std::vector<int> idx(ltick.size());
        for (size_t x = 0; x < idx.size(); ++x) idx[x] = (int)x;
        std::stable_sort(idx.begin(), idx.end(), [&](int x, int y) { return lkey[(size_t)x] > lkey[(size_t)y]; });
        std::vector<int2> sorted(ltick.size());
        for (size_t x = 0; x < idx.size(); ++x) sorted[x] = ltick[(size_t)idx[x]];
        ltick.swap(sorted);
    }
    const size_t sz_mat = align16(sizeof(int) * L * L), sz_args = align16(sizeof(GotohArgs) * count);
    const size_t sz_first = align16(sizeof(int2) * tick.size()) + 16;   // the ticket table, the two ticket counters
    // edit distances: [LevArgs][lut][strip table][ticket, flags][results]
    const size_t sz_lev = lev ? align16(sizeof(LevArgs) * count) + 256 + align16(sizeof(int2) * ltick.size()) + 16 +
                                    align16((size_t)16 * count)
                              : 0;
    // device buffer: [in blocks][out blocks][matrix][arguments][strip table, tickets][edit distances][work blocks]
    // [tie planes]
    const size_t off_out = io_total;
    const size_t off_mat = off_out + oo[count], off_args = off_mat + sz_mat, off_first = off_args + sz_args,
                 off_lev = off_first + sz_first, off_work = off_lev + sz_lev, off_planes = off_work + work[count];
    const size_t off_lut = off_lev + align16(sizeof(LevArgs) * count), off_ltick = off_lut + 256,
                 off_lctr = off_ltick + align16(sizeof(int2) * ltick.size()), off_lres = off_lctr + 16;
    const size_t total = off_planes + planes[count] + 256;
    std::lock_guard<std::mutex> guard(c.gotoh_mutex);   // the scratch is per context
    if (c.gotoh_cap < total) {
        hipFree(c.gotoh_buf);
        c.gotoh_buf = nullptr;
        c.gotoh_cap = 0;
        MH_HIP(hipMalloc(&c.gotoh_buf, total));
        c.gotoh_cap = total;
    }
    char *d = c.gotoh_buf;
    hipStream_t st = c.stream;
    // the device zeroes the work and out areas while the host builds the images
    // (the tie planes are not zeroed: 16 GB at C4-all size; a test poisons
    // them instead, MH_GOTOH_POISON_PLANES=1)
    MH_HIP(hipMemsetAsync(d + off_work, 0, work[count], st));
    if (const char *pz = getenv("MH_GOTOH_POISON_PLANES"); pz && *pz == '1')
        MH_HIP(hipMemsetAsync(d + off_planes, 0xA5, planes[count], st));
    MH_HIP(hipMemsetAsync(d + off_first, 0, sz_first, st));
    MH_HIP(hipMemsetAsync(d + off_out, 0, oo[count], st));
    // host images of the in blocks (uploaded) and the out blocks (fetched):
    // each distinct sequence's block, then each alignment's arguments, built
    // on host threads
    std::unique_ptr<char[]> img(new char[io_total + 16]);
    std::unique_ptr<char[]> oimg(new char[oo[count] + 16]);
    gotoh_par(n1 + n2 + n3, [&](int x) {
        if (x < n1) {   // seq1: codes, text
            const int m = len1[x];
            const char *p = u1[x];
            char *b = &img[io1[x]];
            memset(b, 0, io1[x + 1] - io1[x]);
            for (int i = 0; i < m; ++i) b[i] = (char)code[(unsigned char)p[i]];
            memcpy(b + align16(m + 8), p, m);
        } else if (x < n1 + n2) {   // seq2: codes, text, the score profile (prof_width)
            const int y = x - n1, n = len2[y];
            const char *p = u2[y];
            char *b = &img[io2[y]];
            memset(b, 0, io2[y + 1] - io2[y]);
            for (int j = 0; j < n; ++j) b[j] = (char)code[(unsigned char)p[j]];
            memcpy(b + align16(n + 8), p, n);
            const int PW = prof_width(n);
            int8_t *prof = (int8_t *)(b + align16(n + 8) + align16(n + 1));
            for (int cc = 0; cc < L; ++cc) {
                int8_t *row = prof + (size_t)cc * PW;
                for (int j = 1; j <= n; ++j) row[PROF_PAD + j] = (int8_t)matrix[cc * L + code[(unsigned char)p[j - 1]]];
            }
        } else {   // the edit distance's text, reversed
            const int z = x - n1 - n2, nx = len3[z];
            const char *p = u3[z];
            char *b = &img[io3[z]];
            memset(b, 0, io3[z + 1] - io3[z]);
            for (int j = 0; j < nx; ++j) b[j] = p[nx - 1 - j];
        }
    });
    std::vector<GotohArgs> args(count);
    std::vector<LevArgs> largs(lev ? count : 0);
    gotoh_par(count, [&](int t) {
        const int m = ms[t], n = ns[t];
        size_t q = off_out + oo[t], w = off_work + work[t];
        auto take_out = [&](size_t sz) { const size_t at = q; q += align16(sz); return at; };
        auto take_w = [&](size_t sz) { char *at = d + w; w += align16(sz); return at; };
        GotohArgs &A = args[t];
        const size_t oa = io1[i1[t]], o1 = oa + align16(m + 8);
        const size_t ob = io2[i2[t]], o2 = ob + align16(n + 8), oprof = o2 + align16(n + 1);
        const size_t oo1 = take_out(m + n + 1), oo2 = take_out(m + n + 1), ores = take_out(64);
        A.lastcol = (int *)take_w(sizeof(int) * (m + 2));
        A.lastrow = (int *)take_w(sizeof(int) * (n + 2));
        A.bits = (uint8_t *)(d + off_planes + planes[t]);
        const size_t strips = (size_t)(m + 1 + 63) / 64;
        A.brow1 = (unsigned long long *)take_w(8 * strips * (n + 1));
        A.brow2 = (int *)take_w(sizeof(int) * strips * (n + 1));
        A.rowde = (uint8_t *)take_w(strips * (n + 1));
        A.flags = (int *)take_w(16);
        A.prof = (const int8_t *)(d + oprof);
        A.a = (const int8_t *)(d + oa);
        A.b = (const int8_t *)(d + ob);
        A.s1 = d + o1;
        A.s2 = d + o2;
        A.out1 = d + oo1;
        A.out2 = d + oo2;
        A.result = (int *)(d + ores);
        A.m = m; A.n = n; A.L = L; A.mat = (const int *)(d + off_mat);
        A.u = gep; A.v = gop; A.is_global = is_global ? 1 : 0;
        if (lev) {
            LevArgs &E = largs[t];
            const int nx = nt[t];
            const size_t otx = io3[i3[t]];
            E.o1 = A.out1;
            E.o2 = A.out2;
            E.result = A.result;
            E.text = (const uint8_t *)(d + otx);
            E.n = nx;
            E.pcode = (uint8_t *)take_w((size_t)m + 64);
            E.bnd = (int *)take_w(sizeof(int) * (size_t)(lstr[t] - 1) * nx);
            E.meta = (int *)take_w(16);
            E.res = (int *)(d + off_lres + (size_t)16 * t);
        }
    });
    MH_HIP(hipMemcpyAsync(d, img.get(), io_total, hipMemcpyHostToDevice, st));
    MH_HIP(hipMemcpyAsync(d + off_mat, matrix, sizeof(int) * L * L, hipMemcpyHostToDevice, st));
    MH_HIP(hipMemcpyAsync(d + off_args, args.data(), sizeof(GotohArgs) * count,
                          hipMemcpyHostToDevice, st));
    MH_HIP(hipMemcpyAsync(d + off_first, tick.data(), sizeof(int2) * tick.size(), hipMemcpyHostToDevice, st));
    if (lev) {
        uint8_t lut[256];
        for (int k = 0; k < 256; ++k) lut[k] = (uint8_t)(code[k] + 1);
        MH_HIP(hipMemsetAsync(d + off_lctr, 0, 16, st));
        MH_HIP(hipMemcpyAsync(d + off_lev, largs.data(), sizeof(LevArgs) * count, hipMemcpyHostToDevice, st));
        MH_HIP(hipMemcpyAsync(d + off_lut, lut, 256, hipMemcpyHostToDevice, st));
        MH_HIP(hipMemcpyAsync(d + off_ltick, ltick.data(), sizeof(int2) * ltick.size(), hipMemcpyHostToDevice, st));
    }
    const int strips = (int)tick.size();
    GotohStrips S;
    S.args = (const GotohArgs *)(d + off_args);
    S.tick = (const int2 *)(d + off_first);
    S.strips = strips;
    S.ticket = (int *)(d + off_first + sz_first - 16);
    S.stamps = nullptr;
    S.stamp_blocks = 0;
    S.wait_ticks = wait_ticks;
    const char *stamp_path = getenv("MH_GOTOH_STAMPS");
    if (stamp_path && *stamp_path) {
        int nmx = 0;
        for (int t = 0; t < count; ++t) nmx = std::max(nmx, ns[t]);
        S.stamp_blocks = (nmx + 64) / BBLK + 2;   // the smaller of the two passes' blocks
        MH_HIP(hipMalloc(&S.stamps, sizeof(unsigned long long) * 4 * strips * S.stamp_blocks));
        MH_HIP(hipMemsetAsync(S.stamps, 0, sizeof(unsigned long long) * 4 * strips * S.stamp_blocks, st));
    }
    const int pf = prof_begin(c, "k_gotoh_fwd");
    int nmax = 0;
    for (int t = 0; t < count; ++t) nmax = std::max(nmax, ns[t]);
    const size_t prof_bytes = (size_t)L * prof_width(nmax);
    // MH_GOTOH_PROF_LDS_MAX (diagnostics): another limit for the LDS profile
    size_t lds_max = GPROF_LDS_MAX;
    if (const char *e = getenv("MH_GOTOH_PROF_LDS_MAX"); e && *e) lds_max = (size_t)strtoull(e, nullptr, 10);
    if (prof_bytes <= lds_max) {
        const size_t lds_fwd = sizeof(int2) * GBLK + prof_bytes;
        MH_HIP(hipFuncSetAttribute((const void *)k_gotoh_fwd<true>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                   (int)lds_fwd));
        hipLaunchKernelGGL(k_gotoh_fwd<true>, dim3((unsigned)strips), dim3(64), lds_fwd, st, S);
    } else {
        hipLaunchKernelGGL(k_gotoh_fwd<false>, dim3((unsigned)strips), dim3(64), sizeof(int2) * GBLK, st, S);
    }
    prof_end(c, pf);
    const int pb = prof_begin(c, "k_gotoh_bwd");
    hipLaunchKernelGGL(k_gotoh_bwd, dim3((unsigned)strips), dim3(64), sizeof(int) * BBLK, st, S);
    prof_end(c, pb);
    const int pg = prof_begin(c, "k_gotoh");
    hipLaunchKernelGGL(k_gotoh_tb, dim3((unsigned)count), dim3(GOTOH_THREADS), TB_LDS, st,
                       (const GotohArgs *)(d + off_args));
    prof_end(c, pg);
    std::vector<int> lres(lev ? 4 * (size_t)count : 0);
    int lflag = 0;
    if (lev) {
        LevBatch LB;
        LB.args = (const LevArgs *)(d + off_lev);
        LB.tick = (const int2 *)(d + off_ltick);
        LB.strips = (int)ltick.size();
        LB.ticket = (int *)(d + off_lctr);
        LB.flags = (int *)(d + off_lctr + 4);
        LB.lut = (const uint8_t *)(d + off_lut);
        LB.ncodes = L + 1;
        LB.wait_ticks = wait_ticks;
        const int pl = prof_begin(c, "k_lev");
        hipLaunchKernelGGL(k_lev_prep, dim3((unsigned)count), dim3(64), 0, st, LB);
        if (LB.strips > 0)
            hipLaunchKernelGGL(k_lev, dim3((unsigned)LB.strips), dim3(64), (size_t)LB.ncodes * 64 * 8 + 256, st, LB);
        prof_end(c, pl);
    }
    hipError_t e = hipGetLastError();
    if (lev) {
        if (e == hipSuccess) e = hipMemcpyAsync(lres.data(), d + off_lres, sizeof(int) * lres.size(), hipMemcpyDeviceToHost, st);
        if (e == hipSuccess) e = hipMemcpyAsync(&lflag, d + off_lctr + 4, sizeof(int), hipMemcpyDeviceToHost, st);
    } else if (e == hipSuccess) {
        e = hipMemcpyAsync(oimg.get(), d + off_out, oo[count], hipMemcpyDeviceToHost, st);
    }
    if (e == hipSuccess) e = hipStreamSynchronize(st);
    if (e != hipSuccess) return hip_fail(e, "k_gotoh");
    if (S.stamps) {   // header: strips, blocks per strip; then fwd and bwd stamps
        std::vector<unsigned long long> h((size_t)4 * strips * S.stamp_blocks);
        MH_HIP(hipMemcpy(h.data(), S.stamps, h.size() * sizeof(h[0]), hipMemcpyDeviceToHost));
        MH_HIP(hipFree(S.stamps));
        if (FILE *f = fopen(stamp_path, "wb")) {
            const int64_t hdr[2] = {strips, S.stamp_blocks};
            fwrite(hdr, sizeof(hdr), 1, f);
            fwrite(h.data(), sizeof(h[0]), h.size(), f);
            fclose(f);
        }
    }
    if (lev) {
        for (int t = 0; t < count; ++t) {
            const int *r = &lres[(size_t)4 * t];
            if (r[0] == -4 || lflag) {
                set_error("k_gotoh: a strip's wait for its neighbour timed out (alignment %d)", t);
                return -4;
            }
            status[t] = r[0];
            score[t] = r[1];
            lev_dist[t] = r[0] ? 0 : r[2];
        }
    }
    for (int t = 0; t < count && !lev; ++t) {
        const GotohArgs &A = args[t];
        int res[3];
        memcpy(res, &oimg[(const char *)A.result - d - off_out], sizeof(res));
        if (res[0] == -4) { set_error("k_gotoh: a strip's wait for its neighbour timed out (alignment %d)", t); return -4; }
        status[t] = res[0] ? -1 : 0;
        score[t] = res[1];
        const int len = res[0] ? 0 : res[2];
        const char *t1 = &oimg[A.out1 - d - off_out], *t2 = &oimg[A.out2 - d - off_out];
        for (int k = 0; k < len; ++k) { out1[t][k] = t1[len - 1 - k]; out2[t][k] = t2[len - 1 - k]; }
        out1[t][len] = out2[t][len] = '\0';
    }
    if (c.gotoh_cap > gotoh_keep_bytes()) {
        hipFree(c.gotoh_buf);
        c.gotoh_buf = nullptr;
        c.gotoh_cap = 0;
    }
    return 0;
}

// A strip that waited past its limit for its neighbour (a broken protocol,
// or a producer starved for that long) fails the whole launch with -4; the
// batch is then run once more before the error is reported.  The test
// entry mh_test_set_capacities can impose a first-attempt limit (ticks of
// the 100 MHz clock) so the retry is exercised.
int run_gotoh_batch(Ctx &c, int count, const char *const *s1, const char *const *s2, int gop,
                    int gep, int is_global, const char *alphabet, const int *matrix,
                    char *const *out1, char *const *out2, const int *cap, int *score, int *status)
{
    const unsigned long long first = c.test_caps.gotoh_wait_ticks > 0
                                         ? (unsigned long long)c.test_caps.gotoh_wait_ticks
                                         : GWAIT_TICKS;
    int st = gotoh_batch_once(c, count, s1, s2, gop, gep, is_global, alphabet, matrix, out1, out2,
                              cap, score, status, first, nullptr, nullptr);
    if (st != -4) return st;
    ++c.retries[RETRY_GOTOH_WAIT];
    return gotoh_batch_once(c, count, s1, s2, gop, gep, is_global, alphabet, matrix, out1, out2,
                            cap, score, status, GWAIT_TICKS, nullptr, nullptr);
}

// The batch's alignments reduced on the device to the filter's edit
// distances (k_lev_prep, k_lev); the same timeout-and-retry as above.
int run_gotoh_distance_batch(Ctx &c, int count, const char *const *s1, const char *const *s2,
                             const char *const *text, int gop, int gep, int is_global,
                             const char *alphabet, const int *matrix, int *dist, int *score, int *status)
{
    const unsigned long long first = c.test_caps.gotoh_wait_ticks > 0
                                         ? (unsigned long long)c.test_caps.gotoh_wait_ticks
                                         : GWAIT_TICKS;
    int st = gotoh_batch_once(c, count, s1, s2, gop, gep, is_global, alphabet, matrix, nullptr, nullptr,
                              nullptr, score, status, first, text, dist);
    if (st != -4) return st;
    ++c.retries[RETRY_GOTOH_WAIT];
    return gotoh_batch_once(c, count, s1, s2, gop, gep, is_global, alphabet, matrix, nullptr, nullptr,
                            nullptr, score, status, GWAIT_TICKS, text, dist);
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
