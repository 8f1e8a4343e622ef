// mh_map.hip -- the read mapper that replaces bowtie2 on MiCall-Lite's remap
// path (prelim_map.py:114-140 end-to-end, remap.py:701-755 --local), written
// for gfx950.  Bit-for-bit specification: oracle/og_mapper.c.
//
// Kernels, in launch order for one mapping pass:
//   k_pack_reads  ASCII reads -> 2-bit bases + N mask + qualities (ingest only)
//   k_seed        one wave64 per read: 2x32 exact seeds (one lane each),
//                 hash lookups, hit sort (LDS bitonic), diagonal clustering,
//                 top-4 candidates + work list
//   k_dp          two candidates per wave64 (32 lanes each): banded affine-gap
//                 DP over the seeded diagonal +- 15 (bowtie2's maxhalf), lane
//                 = diagonal, rows = read bases; vertical moves by a DPP wave
//                 shift, horizontal gaps by a DPP prefix-max scan within the
//                 half; 4 traceback bits per cell in LDS; wave-uniform
//                 traceback -> CIGAR; an exact ungapped fast path first
//   k_rescue      paired reads with one aligned mate: the other mate's best
//                 diagonal in the -X window next to it (mate rescue), then
//                 k_dp again over those candidates
//   k_pair        one thread per pair: concordance, flags, MAPQ, SAM fields,
//                 per-reference line tallies
#include <cstring>

#include "mh_internal.h"

namespace mh {

// ---------------------------------------------------------------------------
// small wave helpers
// ---------------------------------------------------------------------------
template <int CTRL, int ROWMASK = 0xF>
__device__ __forceinline__ int dpp(int old, int v)
{
    return __builtin_amdgcn_update_dpp(old, v, CTRL, ROWMASK, 0xF, false);
}
constexpr int DPP_ROW_SHR1 = 0x111, DPP_ROW_SHR2 = 0x112, DPP_ROW_SHR4 = 0x114,
              DPP_ROW_SHR8 = 0x118, DPP_WAVE_SHL1 = 0x130, DPP_WAVE_SHR1 = 0x138;

__device__ __forceinline__ int wave_uniform(int v) { return __builtin_amdgcn_readfirstlane(v); }

__device__ __forceinline__ void wave_sync()
{
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// Wave-wide scans and reductions on DPP (row shifts, then the two row
// broadcasts), register to register: __shfl goes through the LDS crossbar
// (ds_bpermute) and pays its latency on every step.  A lane with no source,
// or in a row a step does not write, takes the identity.  Full wave only.
template <class Op>
__device__ __forceinline__ int wave_scan_dpp(int v, int identity, Op op)
{
    v = op(v, dpp<0x111>(identity, v));           // row_shr:1
    v = op(v, dpp<0x112>(identity, v));           // row_shr:2
    v = op(v, dpp<0x114>(identity, v));           // row_shr:4
    v = op(v, dpp<0x118>(identity, v));           // row_shr:8
    v = op(v, dpp<0x142, 0xA>(identity, v));      // row_bcast:15 into rows 1, 3
    v = op(v, dpp<0x143, 0xC>(identity, v));      // row_bcast:31 into rows 2, 3
    return v;
}

__device__ __forceinline__ int op_add(int x, int y) { return x + y; }
__device__ __forceinline__ int op_min(int x, int y) { return x < y ? x : y; }
__device__ __forceinline__ int op_max(int x, int y) { return x > y ? x : y; }

__device__ __forceinline__ int wave_sum(int v)
{
    return __builtin_amdgcn_readlane(wave_scan_dpp(v, 0, op_add), 63);
}

__device__ __forceinline__ int wave_excl_scan(int v, int /*lane*/)
{
    return wave_scan_dpp(v, 0, op_add) - v;
}

__device__ __forceinline__ int wave_min(int v)
{
    return __builtin_amdgcn_readlane(wave_scan_dpp(v, INT32_MAX, op_min), 63);
}

__device__ __forceinline__ int wave_max(int v)
{
    return __builtin_amdgcn_readlane(wave_scan_dpp(v, INT32_MIN, op_max), 63);
}

// signed 64-bit max: the high words first, then the low words (as unsigned,
// sign bit flipped) among the lanes holding the high maximum
__device__ __forceinline__ long long wave_max64(long long v)
{
    const int hi = (int)(v >> 32);
    const int mhi = wave_max(hi);
    const int lo = (int)((uint32_t)v ^ 0x80000000u);
    const int mlo = wave_max(hi == mhi ? lo : INT32_MIN);
    return (long long)(((uint64_t)(uint32_t)mhi << 32) | (uint32_t)(mlo ^ (int)0x80000000u));
}

__device__ __forceinline__ int imax(int a, int b) { return a > b ? a : b; }

// A load through the constant address space: from a wave-uniform address it
// is a scalar (SMEM) load, counted in lgkmcnt, so waiting for it does not
// wait for the wave's vector loads in flight.  Only for data no kernel of the
// launch writes (descriptors and tables written by earlier launches).
template <class T>
__device__ __forceinline__ T ldc(const T *p)
{
#if defined(__HIP_DEVICE_COMPILE__)
    return *(const __attribute__((address_space(4))) T *)p;
#else
    return *p;
#endif
}

// a candidate's strand, reference and centre as three 4-byte scalar loads
// (volatile: merged into one 12-byte load, which only the vector unit has,
// they would cost a vector round trip)
__device__ __forceinline__ Cand ldc_cand(const Cand *p)
{
#if defined(__HIP_DEVICE_COMPILE__)
    const volatile __attribute__((address_space(4))) int *q =
        (const volatile __attribute__((address_space(4))) int *)p;
    return Cand{q[0], q[1], q[2], 0};
#else
    return *p;
#endif
}

// ---------------------------------------------------------------------------
// k_pack_reads: one wave per read, one lane per base, 64 bases a step: the
// loads of seq and qual are coalesced, and the 2-bit words and N masks are
// assembled from three ballots (code bit 0, code bit 1, N) instead of a lane
// walking 32 bytes of its own
// ---------------------------------------------------------------------------
__device__ __forceinline__ uint32_t base_code(uint8_t c, uint32_t &isn)
{
    switch (c) {
    case 'A': case 'a': isn = 0; return 0;
    case 'C': case 'c': isn = 0; return 1;
    case 'G': case 'g': isn = 0; return 2;
    case 'T': case 't': isn = 0; return 3;
    default: isn = 1; return 0;
    }
}

// the 16 low bits of x to the even bit positions
__device__ __forceinline__ uint32_t spread16(uint32_t x)
{
    x &= 0xffffu;
    x = (x | (x << 8)) & 0x00ff00ffu;
    x = (x | (x << 4)) & 0x0f0f0f0fu;
    x = (x | (x << 2)) & 0x33333333u;
    x = (x | (x << 1)) & 0x55555555u;
    return x;
}

__global__ __launch_bounds__(256) void k_pack_reads(DevReads R, const uint8_t *__restrict__ seq,
                                                    const uint8_t *__restrict__ qual,
                                                    const int64_t *__restrict__ src_off)
{
    const int lane = threadIdx.x & 63;
    const int64_t wave = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    const int64_t nwaves = (int64_t)gridDim.x * 4;
    for (int64_t r = wave; r < R.n; r += nwaves) {
        const int m = R.len[r];
        const int64_t so = src_off[r], dofs = R.off[r];
        const int words = 2 * ((m + 31) >> 5);   // 16-base words the read's slot holds
        for (int g = 0; 64 * g < m; ++g) {
            const int b = 64 * g + lane;
            uint32_t c = 0, isn = 0;
            if (b < m) {
                c = base_code(seq[so + b], isn);
                R.qual[dofs + b] = qual[so + b];
            }
            const uint64_t b0 = __builtin_amdgcn_ballot_w64((c & 1u) != 0);
            const uint64_t b1 = __builtin_amdgcn_ballot_w64((c & 2u) != 0);
            const uint64_t bn = __builtin_amdgcn_ballot_w64(isn != 0);
            if (lane < 4 && 4 * g + lane < words) {
                const int sh = 16 * lane;
                R.seq2[(dofs >> 4) + 4 * g + lane] =
                    spread16((uint32_t)(b0 >> sh)) | (spread16((uint32_t)(b1 >> sh)) << 1);
            } else if (lane >= 4 && lane < 6 && 4 * g + 2 * (lane - 4) < words) {   // 32-base N words
                R.nmask[(dofs >> 5) + 2 * g + (lane - 4)] = (uint32_t)(bn >> (32 * (lane - 4)));
            }
        }
    }
}

hipError_t launch_pack_reads(DevReads &r, const uint8_t *d_seq, const uint8_t *d_qual,
                             const int64_t *d_src_off, hipStream_t s)
{
    if (r.n == 0) return hipSuccess;
    int64_t blocks = (r.n + 3) / 4;
    if (blocks > 65536) blocks = 65536;
    hipLaunchKernelGGL(k_pack_reads, dim3((unsigned)blocks), dim3(256), 0, s, r, d_seq, d_qual,
                       d_src_off);
    return hipGetLastError();
}

// ---------------------------------------------------------------------------
// read access helpers
// ---------------------------------------------------------------------------
__device__ __forceinline__ uint32_t read_code(const DevReads &R, int64_t off, int b)
{
    const int64_t g = off + b;
    if ((R.nmask[g >> 5] >> (g & 31)) & 1) return 4;
    return (R.seq2[g >> 4] >> (2 * (g & 15))) & 3;
}

// Word w (bases 16w .. 16w+15) of read (off, m) on strand s, taken from the
// packed words: code = the 2-bit codes (0 where ambiguous or past the read),
// nmk = 1 in the low bit of every such base's pair.  The reverse complement
// reverses 16 pairs of the forward bases m-16w-16 .. m-16w-1 (a funnel of two
// words; indices before the read's start only feed bases past its end).
__device__ __forceinline__ void read_word2(const DevReads &R, int64_t off, int m, int s, int w,
                                           uint32_t &code, uint32_t &nmk)
{
    const int nv = m - 16 * w < 16 ? (m - 16 * w > 0 ? m - 16 * w : 0) : 16;   // bases of the read
    const uint32_t valid = nv >= 16 ? 0xffffffffu : ((1u << (2 * nv)) - 1u);
    uint32_t c, nb;
    if (!s) {
        const int64_t g = off + 16 * w;   // off is a multiple of 32
        c = R.seq2[g >> 4];
        nb = (R.nmask[g >> 5] >> (g & 31)) & 0xffffu;
    } else {
        const int64_t g = off + m - 16 * w - 16;
        // word indices clamped into the read (arithmetic shifts: before the
        // first read g is negative); a clamped word only feeds bits that are
        // past the read or shifted out
        const int64_t wlast = (off + m - 1) >> 4, nlast = (off + m - 1) >> 5;
        const int64_t wl = g >> 4, nl = g >> 5;
        const int64_t w0 = wl > 0 ? wl : 0, w1 = wl + 1 < wlast ? (wl + 1 > 0 ? wl + 1 : 0) : wlast;
        const int64_t n0i = nl > 0 ? nl : 0, n1i = nl + 1 < nlast ? (nl + 1 > 0 ? nl + 1 : 0) : nlast;
        const uint32_t c0 = R.seq2[w0], c1 = R.seq2[w1];
        const uint32_t n0 = R.nmask[n0i], n1 = R.nmask[n1i];
        const uint32_t cf = __builtin_amdgcn_alignbit(c1, c0, (uint32_t)(2 * (g & 15)));
        const uint32_t nf = __builtin_amdgcn_alignbit(n1, n0, (uint32_t)(g & 31));
        // reverse the 16 pairs (bit reverse, then swap the bits of each pair), complement
        uint32_t r = __builtin_bitreverse32(cf);
        r = ((r >> 1) & 0x55555555u) | ((r & 0x55555555u) << 1);
        c = ~r;
        nb = __builtin_bitreverse32(nf & 0xffffu) >> 16;
    }
    // spread the 16 N bits to the low bit of each pair
    uint32_t sp = nb;
    sp = (sp | (sp << 8)) & 0x00ff00ffu;
    sp = (sp | (sp << 4)) & 0x0f0f0f0fu;
    sp = (sp | (sp << 2)) & 0x33333333u;
    sp = (sp | (sp << 1)) & 0x55555555u;
    sp = (sp & valid) | (~valid & 0x55555555u);
    nmk = sp;
    code = c & ~(sp * 3u) & valid;
}

// SL (<= 32) consecutive 2-bit codes starting at absolute base g, base x at
// bits 2x+1:2x; and the N-mask bits of the same window.
__device__ __forceinline__ uint64_t window_key(const DevReads &R, int64_t g, int SL)
{
    const int64_t w = g >> 4;
    const int sh = 2 * (int)(g & 15);
    const uint64_t lo = (uint64_t)R.seq2[w] | ((uint64_t)R.seq2[w + 1] << 32);
    const uint64_t hi = R.seq2[w + 2];
    uint64_t k = sh ? (lo >> sh) | (hi << (64 - sh)) : lo;
    return SL >= 32 ? k : (k & ((1ull << (2 * SL)) - 1));
}

__device__ __forceinline__ uint32_t window_nmask(const DevReads &R, int64_t g, int SL)
{
    const int64_t w = g >> 5;
    const int sh = (int)(g & 31);
    const uint64_t v = ((uint64_t)R.nmask[w] | ((uint64_t)R.nmask[w + 1] << 32)) >> sh;
    return (uint32_t)(v & ((1ull << SL) - 1));
}

__device__ __forceinline__ uint64_t revcomp_key(uint64_t k, int SL)
{
    uint64_t x = ~k;
    x = ((x >> 2) & 0x3333333333333333ull) | ((x & 0x3333333333333333ull) << 2);
    x = ((x >> 4) & 0x0F0F0F0F0F0F0F0Full) | ((x & 0x0F0F0F0F0F0F0F0Full) << 4);
    x = ((x >> 8) & 0x00FF00FF00FF00FFull) | ((x & 0x00FF00FF00FF00FFull) << 8);
    x = ((x >> 16) & 0x0000FFFF0000FFFFull) | ((x & 0x0000FFFF0000FFFFull) << 16);
    x = (x >> 32) | (x << 32);
    return x >> (64 - 2 * SL);
}

// ---------------------------------------------------------------------------
// k_seed
// ---------------------------------------------------------------------------
struct SeedArgs {
    DevReads R;
    DevIndex I;
    int mode;
    const int32_t *len_tab;  // [0]: seed interval, [1]: min score, [2]: n ceil
    Cand *cand;
    int32_t *n_cand;
    int32_t *yf;
    int32_t *work;
    int32_t *counters;
    int64_t plane;           // slot planes' stride (slot_at)
};

__device__ __forceinline__ bool cand_before(const Cand &x, const Cand &y)
{
    if (x.support != y.support) return x.support > y.support;
    if (x.strand != y.strand) return x.strand < y.strand;
    if (x.ref != y.ref) return x.ref < y.ref;
    return x.center < y.center;
}

__device__ __forceinline__ uint64_t shfl_xor64(uint64_t v, int m)
{
    const int lo = __shfl_xor((int)(uint32_t)v, m), hi = __shfl_xor((int)(v >> 32), m);
    return ((uint64_t)(uint32_t)hi << 32) | (uint32_t)lo;
}

__device__ __forceinline__ uint64_t readlane64(uint64_t v, int l)
{
    const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)v, l);
    const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(v >> 32), l);
    return ((uint64_t)hi << 32) | lo;
}

// Candidate clustering of <= 64 seed hits, one per lane (v; ~0 past total):
// a bitonic sort across the lanes, then cluster and run boundaries as
// ballots, and per cluster (a wave-uniform loop over the boundary bits) the
// centre as the longest run of equal hits (the first on ties), by one wave
// max.  The same clusters, centres, supports and top-MAXCAND order as the
// serial walk below (og_mapper.c find_candidates); writes the candidates.
// The hit of lane ^ J.  J = 1, 2, 8 are one DPP move per word (quad_perm,
// row_ror:8), J = 4 two moves and a select; J = 16, 32 go through
// ds_bpermute.  Register to register where DPP reaches: a bpermute is an LDS
// crossbar round trip, and the sort is a chain of them.
template <int J>
__device__ __forceinline__ uint64_t xor_lane64(uint64_t v, int lane)
{
    const int lo = (int)(uint32_t)v, hi = (int)(v >> 32);
    int xl, xh;
    if (J == 1) {
        xl = dpp<0xB1>(lo, lo); xh = dpp<0xB1>(hi, hi);       // quad_perm [1,0,3,2]
    } else if (J == 2) {
        xl = dpp<0x4E>(lo, lo); xh = dpp<0x4E>(hi, hi);       // quad_perm [2,3,0,1]
    } else if (J == 4) {
        const bool up = (lane & 4) != 0;                      // take lane - 4, else lane + 4
        const int ll = dpp<0x104>(lo, lo), lr = dpp<0x114>(lo, lo);   // row_shl:4, row_shr:4
        const int hl = dpp<0x104>(hi, hi), hr = dpp<0x114>(hi, hi);
        xl = up ? lr : ll;
        xh = up ? hr : hl;
    } else if (J == 8) {
        xl = dpp<0x128>(lo, lo); xh = dpp<0x128>(hi, hi);     // row_ror:8
    } else {
        return shfl_xor64(v, J);
    }
    return ((uint64_t)(uint32_t)xh << 32) | (uint32_t)xl;
}

template <int K, int J>
__device__ __forceinline__ void bitonic_step(uint64_t &v, int lane)
{
    const uint64_t o = xor_lane64<J>(v, lane);
    const bool take_min = ((lane & J) == 0) == ((lane & K) == 0);
    v = take_min ? (o < v ? o : v) : (o > v ? o : v);
}

// Bitonic sort of one 64-bit hit per lane over the first N lanes (N a power
// of two <= 64; the stages of every block size k <= N, as the loop
// for k in 2..N, j in k/2..1 runs them).
__device__ __forceinline__ uint64_t bitonic_lanes(uint64_t v, int lane, int N)
{
    bitonic_step<2, 1>(v, lane);
    if (N >= 4) { bitonic_step<4, 2>(v, lane); bitonic_step<4, 1>(v, lane); }
    if (N >= 8) { bitonic_step<8, 4>(v, lane); bitonic_step<8, 2>(v, lane); bitonic_step<8, 1>(v, lane); }
    if (N >= 16) {
        bitonic_step<16, 8>(v, lane); bitonic_step<16, 4>(v, lane);
        bitonic_step<16, 2>(v, lane); bitonic_step<16, 1>(v, lane);
    }
    if (N >= 32) {
        bitonic_step<32, 16>(v, lane); bitonic_step<32, 8>(v, lane); bitonic_step<32, 4>(v, lane);
        bitonic_step<32, 2>(v, lane); bitonic_step<32, 1>(v, lane);
    }
    if (N >= 64) {
        bitonic_step<64, 32>(v, lane); bitonic_step<64, 16>(v, lane); bitonic_step<64, 8>(v, lane);
        bitonic_step<64, 4>(v, lane); bitonic_step<64, 2>(v, lane); bitonic_step<64, 1>(v, lane);
    }
    return v;
}

__device__ int cluster_lanes(const SeedArgs &A, int64_t r, int lane, uint64_t v, int total,
                             Cand *best)
{
    // every hit the same (strand, reference, diagonal) -- a read without an
    // indel against a reference it maps to once: one cluster of one run,
    // the candidate the sort and the walk below would give
    {
        const uint64_t v0 = readlane64(v, 0);
        if (__builtin_amdgcn_ballot_w64(lane < total && v != v0) == 0) {
            if (lane == 0) {
                A.cand[r] = Cand{(int)(v0 >> 62), (int)((v0 >> 32) & 0x3fffffff),
                                 (int)(uint32_t)v0 - (1 << 30), total};   // candidate 0: plane 0
                A.n_cand[r] = 1;
            }
            wave_sync();
            return 1;
        }
    }
    int N = 2;
    while (N < total) N <<= 1;
    {
        // hits arrive in seed order, already sorted when the read's diagonal
        // only grows along it (a deletion): the sort is then the identity
        const uint64_t qv = ((uint64_t)(uint32_t)dpp<DPP_WAVE_SHR1>(0, (int)(v >> 32)) << 32) |
                            (uint32_t)dpp<DPP_WAVE_SHR1>(0, (int)(uint32_t)v);   // lane - 1's hit
        if (__builtin_amdgcn_ballot_w64(lane > 0 && lane < total && v < qv) != 0) v = bitonic_lanes(v, lane, N);
    }
    const uint64_t pv = ((uint64_t)(uint32_t)dpp<DPP_WAVE_SHR1>(0, (int)(v >> 32)) << 32) |
                        (uint32_t)dpp<DPP_WAVE_SHR1>(0, (int)(uint32_t)v);   // lane - 1's hit
    const bool valid = lane < total;
    const int dg = (int)(uint32_t)v - (1 << 30), pdg = (int)(uint32_t)pv - (1 << 30);
    const bool bnd = valid && (lane == 0 || (v >> 32) != (pv >> 32) || dg - pdg > CLUSTER_GAP);
    const bool rst = valid && (lane == 0 || v != pv);
    uint64_t bm = __builtin_amdgcn_ballot_w64(bnd);
    const uint64_t rm = __builtin_amdgcn_ballot_w64(rst);
    const uint64_t above = lane == 63 ? 0ull : rm & (~0ull << (lane + 1));
    const int runlen = (above ? (int)__builtin_ctzll(above) : total) - lane;
    int nc = 0;
    while (bm) {
        const int cs = (int)__builtin_ctzll(bm);
        bm &= bm - 1;
        const int ce = bm ? (int)__builtin_ctzll(bm) : total;
        const int key = (rst && lane >= cs && lane < ce) ? (runlen << 6) | (63 - lane) : -1;
        const int cl = 63 - (wave_max(key) & 63);
        const uint64_t v0 = readlane64(v, cs);
        const int center = (int)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)v, cl) - (1 << 30);
        const Cand c{(int)(v0 >> 62), (int)((v0 >> 32) & 0x3fffffff), center, ce - cs};
        if (lane == 0) {
            int at = nc;
            while (at > 0 && cand_before(c, best[at - 1])) --at;
            if (at < MAXCAND) {
                const int last = nc < MAXCAND ? nc : MAXCAND - 1;
                for (int z = last; z > at; --z) best[z] = best[z - 1];
                best[at] = c;
                if (nc < MAXCAND) ++nc;
            }
        }
    }
    if (lane == 0) {
        for (int c = 0; c < nc; ++c) A.cand[(int64_t)c * A.plane + r] = best[c];
        A.n_cand[r] = nc;
    }
    wave_sync();
    return __builtin_amdgcn_readfirstlane(nc);
}

// The raw words a read's seeding starts from, loaded one read ahead: lane
// (strand s = lane >> 5, seed t = lane & 31) holds the three 2-bit words and
// two N-mask words under its seed window, and lane w < 32 the read's N-mask
// word w for the N count.  k_seed issues the next read's loads right after
// the current read's first hash probe, so they land while the probe chain
// waits (loads return in order: issued after the probe, they hold no wait
// of its back).
struct SeedPre {
    uint32_t s0, s1, s2, n0, n1, nw;
    int m, iv, ns;
    int64_t off;
};

__device__ __forceinline__ SeedPre seed_prefetch(const SeedArgs &A, int m, int64_t off, int lane)
{
    const int SL = A.I.seedlen;
    SeedPre P;
    P.m = m;
    P.off = off;
    P.iv = m >= SL ? ldc(&A.len_tab[m]) : 1;
    int ns = m >= SL ? 1 + (m - SL) / P.iv : 0;
    P.ns = ns > MAXSEEDS ? MAXSEEDS : ns;
    // unconditional loads (lanes without a window read the read's first
    // words): a load under a branch ends in a copy at the join, and the copy
    // waits for it
    const int s = lane >> 5, t = lane & 31;
    const int o = t * P.iv;
    const int64_t g = t < P.ns ? off + (s == 0 ? o : m - o - SL) : off;
    const uint32_t *sq = A.R.seq2 + (g >> 4), *nq = A.R.nmask + (g >> 5);
    P.s0 = sq[0]; P.s1 = sq[1]; P.s2 = sq[2];
    P.n0 = nq[0]; P.n1 = nq[1];
    P.nw = A.R.nmask[(off >> 5) + (lane * 32 < m ? lane : 0)];   // m <= MAXLEN: one word per lane
    return P;
}

// Seeds, hit sort and candidate clustering of read r (its words in P) by one
// wave; writes the candidates, n_cand and yf, returns the candidate count
// (wave-uniform).  Q receives the next read's words (m_next, off_next).
__device__ int seed_read(const SeedArgs &A, int64_t r, const SeedPre &P, int lane, uint64_t *hits,
                         Cand *best, SeedPre &Q, int m_next, int64_t off_next)
{
    const int SL = A.I.seedlen;
    const int m = P.m, iv = P.iv, ns = P.ns;
    bool fetched = false;
    auto fetch_next = [&]() {
        if (!fetched) Q = seed_prefetch(A, m_next, off_next, lane);
        fetched = true;
    };
    if (m == 0) {
        fetch_next();
        if (lane == 0) { A.n_cand[r] = 0; A.yf[r] = 2; }
        return 0;
    }
    const int s = lane >> 5, t = lane & 31;
    const int o = t * iv;
    uint32_t wnm = 1;
    uint64_t wkey = 0;
    if (t < ns) {
        const int64_t g = P.off + (s == 0 ? o : m - o - SL);
        const int sh2 = 2 * (int)(g & 15), sh1 = (int)(g & 31);
        const uint64_t lo = (uint64_t)P.s0 | ((uint64_t)P.s1 << 32);
        const uint64_t k = sh2 ? (lo >> sh2) | ((uint64_t)P.s2 << (64 - sh2)) : lo;
        wkey = SL >= 32 ? k : (k & ((1ull << (2 * SL)) - 1));
        const uint64_t v = ((uint64_t)P.n0 | ((uint64_t)P.n1 << 32)) >> sh1;
        wnm = (uint32_t)(v & ((1ull << SL) - 1));
    }
    int nn = 0;
    if (lane * 32 < m) {
        uint32_t bits = P.nw;
        const int rem = m - lane * 32;
        if (rem < 32) bits &= (1u << rem) - 1;
        nn = __popc(bits);
    }
    nn = wave_sum(nn);
    if (nn > ldc(&A.len_tab[2 * (MAXLEN + 1) + m])) {
        fetch_next();
        if (lane == 0) { A.n_cand[r] = 0; A.yf[r] = 1; }
        return 0;
    }
    if (lane == 0) A.yf[r] = 0;
    if (m < SL) {
        fetch_next();
        if (lane == 0) A.n_cand[r] = 0;
        return 0;
    }
    int cnt = 0;
    uint32_t start = 0;
    // the first probe of every seed, then the next read's loads, then the
    // rest of the probe chains (an entry holds its key and its hits' range)
    const bool probe = t < ns && wnm == 0;
    uint64_t key = 0, h = 0;
    uint4 e = make_uint4(~0u, ~0u, 0u, 0u);
    if (probe) {
        key = s ? revcomp_key(wkey, SL) : wkey;
        h = hash_key(key) & A.I.hmask;
        e = A.I.hent[h];
    }
    fetch_next();
    if (probe) {
        for (;;) {
            const uint64_t k = (uint64_t)e.x | ((uint64_t)e.y << 32);
            if (k == HEMPTY) break;
            if (k == key) {
                start = e.z;
                cnt = (int)e.w;
                break;
            }
            h = (h + 1) & A.I.hmask;
            e = A.I.hent[h];
        }
        if (cnt > MAXHITS_SEED) cnt = 0;
    }
    const int pre = wave_excl_scan(cnt, lane);
    int total = wave_sum(cnt);
    if (total > MAXHITS_MATE) total = MAXHITS_MATE;
    for (int e = 0; e < cnt && pre + e < MAXHITS_MATE; ++e) {
        const int2 h = A.I.hits[start + e];
        const int diag = h.y - o;
        hits[pre + e] = ((uint64_t)s << 62) | ((uint64_t)h.x << 32) |
                        (uint64_t)(uint32_t)(diag + (1 << 30));
    }
    if (total == 0) {
        if (lane == 0) A.n_cand[r] = 0;
        return 0;
    }
    if (total <= 64) {   // one hit per lane: register sort, lane-parallel clusters
        wave_sync();
        return cluster_lanes(A, r, lane, lane < total ? hits[lane] : ~0ull, total, best);
    }
    int N = 1;
    while (N < total) N <<= 1;
    for (int x = total + lane; x < N; x += 64) hits[x] = ~0ull;
    wave_sync();
    // bitonic sort, ascending
    for (int k = 2; k <= N; k <<= 1) {
        for (int j = k >> 1; j > 0; j >>= 1) {
            for (int tt = lane; tt < (N >> 1); tt += 64) {
                const int i = 2 * j * (tt / j) + (tt % j);
                const int q = i + j;
                const uint64_t a = hits[i], b = hits[q];
                const bool up = (i & k) == 0;
                if ((a > b) == up) { hits[i] = b; hits[q] = a; }
            }
            wave_sync();
        }
    }
    int nc = 0;
    if (lane == 0) {
        int h0 = 0;
        while (h0 < total) {
            const uint64_t k0 = hits[h0];
            const int st = (int)(k0 >> 62), rf = (int)((k0 >> 32) & 0x3fffffff);
            int h1 = h0 + 1;
            int prev = (int)(uint32_t)k0 - (1 << 30);
            while (h1 < total) {
                const uint64_t k1 = hits[h1];
                const int d1 = (int)(uint32_t)k1 - (1 << 30);
                if ((k1 >> 32) != (k0 >> 32) || d1 - prev > CLUSTER_GAP) break;
                prev = d1;
                ++h1;
            }
            int center = (int)(uint32_t)k0 - (1 << 30), center_n = 0;
            for (int a = h0; a < h1;) {
                int b = a + 1;
                while (b < h1 && hits[b] == hits[a]) ++b;
                if (b - a > center_n) {
                    center_n = b - a;
                    center = (int)(uint32_t)hits[a] - (1 << 30);
                }
                a = b;
            }
            Cand c{st, rf, center, h1 - h0};
            int at = nc;
            while (at > 0 && cand_before(c, best[at - 1])) --at;
            if (at < MAXCAND) {
                const int last = nc < MAXCAND ? nc : MAXCAND - 1;
                for (int z = last; z > at; --z) best[z] = best[z - 1];
                best[at] = c;
                if (nc < MAXCAND) ++nc;
            }
            h0 = h1;
        }
        for (int c = 0; c < nc; ++c) A.cand[(int64_t)c * A.plane + r] = best[c];
        A.n_cand[r] = nc;
    }
    wave_sync();
    return __builtin_amdgcn_readfirstlane(nc);
}

// One wave per chunk of SEED_CHUNK consecutive reads: the chunk's extension
// work items are collected in LDS and appended to the work list with one
// atomic (a returning same-address atomic costs ~11 ns device-wide).
constexpr int SEED_CHUNK = 32;

// k_seed is latency-bound (hash probes): built for 8 waves per SIMD (<= 64 VGPRs).
constexpr int SEED_WAVES_PER_SIMD = 8;
__global__ __launch_bounds__(256, SEED_WAVES_PER_SIMD) void k_seed(SeedArgs A)
{
    __shared__ uint64_t sh_hits[4][MAXHITS_MATE];
    __shared__ Cand sh_best[4][MAXCAND];
    __shared__ int32_t sh_work[4][SEED_CHUNK * MAXCAND];
    const int lane = threadIdx.x & 63;
    const int wv = wave_uniform(threadIdx.x >> 6);
    const int64_t n_chunks = (A.R.n + SEED_CHUNK - 1) / SEED_CHUNK;
    for (int64_t ch = (int64_t)blockIdx.x * 4 + wv; ch < n_chunks; ch += (int64_t)gridDim.x * 4) {
        int n_work = 0;
        const int64_t r0 = ch * SEED_CHUNK;
        const int64_t r1 = r0 + SEED_CHUNK < A.R.n ? r0 + SEED_CHUNK : A.R.n;
        // the chunk's read lengths and offsets in one round trip (lane = read)
        int my_m = 0;
        int64_t my_off = 0;
        if (r0 + lane < r1) {
            my_m = A.R.len[r0 + lane];
            my_off = A.R.off[r0 + lane];
        }
        SeedPre P = seed_prefetch(A, __builtin_amdgcn_readlane(my_m, 0),
                                  (int64_t)readlane64((uint64_t)my_off, 0), lane);
        for (int64_t r = r0; r < r1; ++r) {
            const int l = (int)(r - r0);
            // the next read of the chunk (past its end: an empty read, no loads)
            const int ln = l + 1 < (int)(r1 - r0) ? l + 1 : 0;
            const int mn = l + 1 < (int)(r1 - r0) ? __builtin_amdgcn_readlane(my_m, ln) : 0;
            const int64_t offn = (int64_t)readlane64((uint64_t)my_off, ln);
            SeedPre Q;
            const int nc = seed_read(A, r, P, lane, sh_hits[wv], sh_best[wv], Q, mn, offn);
            P = Q;
            if (lane < nc) sh_work[wv][n_work + lane] = (int32_t)(r * MAXCAND + lane);
            n_work += nc;
        }
        wave_sync();
        int base = 0;
        if (lane == 0 && n_work) base = atomicAdd(&A.counters[0], n_work);
        base = __builtin_amdgcn_readfirstlane(base);
        for (int x = lane; x < n_work; x += 64) A.work[base + x] = sh_work[wv][x];
        wave_sync();
    }
}

// ---------------------------------------------------------------------------
// k_dp: banded affine-gap DP, two candidates per wave64 (32 lanes each)
// ---------------------------------------------------------------------------
struct DpArgs {
    DevReads R;
    DevIndex I;
    const int32_t *len_tab;
    const Cand *cand;
    const int32_t *work;
    const int32_t *counters;  // [0] = number of work items
    SlotKey *skey;
    SlotInfo *sinfo;
    uint32_t *pool;
    unsigned long long *pool_used;  // words claimed so far (64-bit: never wraps)
    int32_t *pool_ctr;        // [1] overflow, [2] fast-path extensions
    int32_t *queue;           // work-queue counter (chunks past the static first ones), zeroed
    int64_t pool_cap;
    int rows_pad;             // per-wave LDS row capacity (multiple of 8)
    int wave_lds;             // bytes of LDS per wave
    int oeI, exI, oeD, exD;
    int64_t plane;            // slot planes' stride (slot_at)
};

__device__ __forceinline__ int mm_pen(int qchar)
{
    int q = qchar - 33;
    q = q < 0 ? 0 : (q > 40 ? 40 : q);
    return 2 + ((q * 205) >> 11);   // q / 10 for 0 <= q <= 40
}

// Scores inside the row recurrence carry a bias of 2^20, so every live value
// is positive and the 0 that a DPP move with bound_ctrl shifts in at the band
// edges acts as minus infinity.  The moves then fold into the ALU op that uses
// them (v_max_i32_dpp, v_add_u32_dpp) instead of costing a mov + a fill each.
constexpr int BIAS = 1 << 20;
constexpr int DP_WAVES_PER_BLOCK = 4;   // k_dp workgroup size in waves (measured best of 1-4)
// CIGAR runs kept by the traceback.  A path with more runs cannot end up
// with <= MH_MAXOPS - 1 ops: overhang trimming removes at most ~2 x 64 runs.
constexpr int RUNS_CAP = 256;
// CIGAR ops are reserved per wave in chunks (one atomic per chunk, not per
// extension); the pool is sized for every resident wave's partial chunk.
constexpr int POOL_CHUNK = 256;
constexpr int DP_MAX_BLOCKS = 256 * 48;
constexpr int DP_QUEUE_CHUNK = 8;       // k_dp work items per queue chunk

template <int CTRL>
__device__ __forceinline__ int dppz(int v)
{
    return __builtin_amdgcn_update_dpp(0, v, CTRL, 0xF, 0xF, true);
}

__device__ __forceinline__ uint32_t umin1(int v) { return (uint32_t)v < 1u ? (uint32_t)v : 1u; }

// inclusive prefix max within each 32-lane half (x > 0): the row shifts,
// then lane 15 of rows 0 and 2 into rows 1 and 3
__device__ __forceinline__ int scan_max(int x)
{
    x = imax(x, dppz<DPP_ROW_SHR1>(x));
    x = imax(x, dppz<DPP_ROW_SHR2>(x));
    x = imax(x, dppz<DPP_ROW_SHR4>(x));
    x = imax(x, dppz<DPP_ROW_SHR8>(x));
    // the cross-row step in place: rows it does not write keep x (measured on
    // gfx950 with profiles/diag/dpp_probe.hip); the hazard nops of the
    // VALU-write -> DPP-read pair are inside the string
    asm volatile("s_nop 1\n\t"
                 "v_max_i32_dpp %0, %0, %0 row_bcast:15 row_mask:0xa bank_mask:0xf\n\t"
                 "s_nop 1"
                 : "+v"(x));
    return x;
}

// Row values are kept shifted so that the deletion scan needs no per-lane
// add: lane k holds H~ = H + exD * k (and E~ the same), so X = H1~ directly
// and F~ = P(k-1) - (oeD - exD) with one constant.  In end-to-end mode every
// value of row i also carries + 8 (i + 1), the bias of the score nibbles, so
// the diagonal move is one add (local mode keeps the - 8: its floor and the
// best-cell key must not drift by row).  Lane-uniform offsets cancel in every
// traceback bit; the best score subtracts them once at the end.
// All but dIE are per lane: a lane outside its extension's band (and, for
// E, the band's top lane) holds HUGE_NEG in mexI / cF and 0 as its floor.
struct DpConst {
    int mexI;           // E~ = dpp(q) + mexI: -(exI + exD), + 8 end-to-end
    int dIE;            // exI - oeI: h1 - e1 = (Hp + dIE) - Ep on the source lane
    int cF;             // F~ = dpp(P) + cF: -(oeD - exD)
    int floor;          // local: BIAS + exD * lane, the shifted zero
};

// acc = 2 acc + (d < 0): the sign bit of d shifted into the traceback word
__device__ __forceinline__ uint32_t push_sign(uint32_t acc, int d)
{
    return __builtin_amdgcn_alignbit(acc, (uint32_t)d, 31u);
}

// Traceback nibble of cell (i, k), four sign bits in this order (bit 3 first;
// row t of an 8-row group sits at nibble 7 - t):
//   bit 3  eb'  on lane k: E(i, k-1) extends (oracle eb of cell k-1: the
//               extension beat the opening on lane k of row i-1)
//   bit 2  fb'  on lane k: F(i, k+1) extends (oracle fb of cell k+1:
//               X(k) < P(k), the prefix max came from a lane left of k)
//   bit 1  Hd < H  (0: the diagonal is the source)
//   bit 0  E  < H  (0: E is the source when the diagonal is not)
// Each bit is one subtraction and one v_alignbit; no lane-mask compare.  The
// local stop (H == 0) is not stored: the traceback knows H along its path.
constexpr uint32_t TB_EB = 8u, TB_FB = 4u, TB_NE = 1u;   // (bit 1: Hd < H, tested as TB_ND_ALL)
constexpr uint32_t TB_ND_ALL = 0x22222222u;   // bit 1 of every nibble

// One DP row inside the gap window (oracle dp_extend, og_mapper.c:289-328).
template <int LOCAL>
__device__ __forceinline__ void dp_row_gap(uint32_t tbv, int rc, int &Hp, int &Ep,
                                           uint32_t &bestKey, int ci, const DpConst &K,
                                           uint32_t &acc)
{
    const int nib = (int)__builtin_amdgcn_ubfe(tbv, (uint32_t)rc, 4);
    const int Hd = LOCAL ? Hp + nib - 8 : Hp + nib;
    // vertical (insertion) move from lane k+1 of the previous row: on the
    // source lane q = max(Ep - exI, Hp - oeI) + exI, moved one lane down by
    // the fused DPP add; ties open (eb needs h1 < e1 strictly)
    const int hc = Hp + K.dIE;
    const int q = imax(Ep, hc);
    const int E = dppz<DPP_WAVE_SHL1>(q) + K.mexI;
    acc = push_sign(acc, hc - Ep);
    int H1 = imax(Hd, E);
    if (LOCAL) H1 = imax(H1, K.floor);
    // horizontal (deletion) moves: prefix max of X = H1~ over the lanes
    const int P = scan_max(H1);
    const int F = dppz<DPP_WAVE_SHR1>(P) + K.cF;
    const int H = imax(H1, F);
    acc = push_sign(acc, H1 - P);
    acc = push_sign(acc, Hd - H);
    acc = push_sign(acc, E - H);
    if (LOCAL) {
        const uint32_t key = ((uint32_t)H << 10) | (uint32_t)ci;   // ci < 1024
        bestKey = bestKey > key ? bestKey : key;
    }
    Hp = H;
    Ep = E;
}

// dp_row_gap with the traceback bits software-pipelined: the row's four
// sign differences are left in pd and pushed into acc during the next row's
// deletion scan (between its dependent DPP steps, where the wave would
// otherwise wait out the DPP hazards); the caller pushes the last row's.
// The bits land in acc in the same order as dp_row_gap's.
template <int LOCAL, bool HAVE>
__device__ __forceinline__ void dp_row_gap_pipe(uint32_t tbv, int rc, int &Hp, int &Ep,
                                                uint32_t &bestKey, int ci, const DpConst &K,
                                                uint32_t &acc, int (&pd)[4])
{
    const int nib = (int)__builtin_amdgcn_ubfe(tbv, (uint32_t)rc, 4);
    const int Hd = LOCAL ? Hp + nib - 8 : Hp + nib;
    const int hc = Hp + K.dIE;
    const int q = imax(Ep, hc);
    const int E = dppz<DPP_WAVE_SHL1>(q) + K.mexI;
    const int de = hc - Ep;
    int H1 = imax(Hd, E);
    if (LOCAL) H1 = imax(H1, K.floor);
    int x = H1;
    x = imax(x, dppz<DPP_ROW_SHR1>(x));
    if (HAVE) acc = push_sign(acc, pd[0]);
    x = imax(x, dppz<DPP_ROW_SHR2>(x));
    if (HAVE) acc = push_sign(acc, pd[1]);
    x = imax(x, dppz<DPP_ROW_SHR4>(x));
    if (HAVE) acc = push_sign(acc, pd[2]);
    x = imax(x, dppz<DPP_ROW_SHR8>(x));
    if (HAVE) acc = push_sign(acc, pd[3]);
    asm volatile("s_nop 1\n\t"
                 "v_max_i32_dpp %0, %0, %0 row_bcast:15 row_mask:0xa bank_mask:0xf\n\t"
                 "s_nop 1"
                 : "+v"(x));
    const int P = x;
    const int F = dppz<DPP_WAVE_SHR1>(P) + K.cF;
    const int H = imax(H1, F);
    pd[0] = de;
    pd[1] = H1 - P;
    pd[2] = Hd - H;
    pd[3] = E - H;
    if (LOCAL) {
        const uint32_t key = ((uint32_t)H << 10) | (uint32_t)ci;   // ci < 1024
        bestKey = bestKey > key ? bestKey : key;
    }
    Hp = H;
    Ep = E;
}

// A row outside the gap window (first / last GBAR rows): no E, no F.  Its
// nibble is 0: a local cell at H == 0 is a stop the traceback sees from H.
template <int LOCAL>
__device__ __forceinline__ void dp_row_nogap(uint32_t tbv, int rc, int &Hp, int &Ep,
                                             uint32_t &bestKey, int ci, int floor, uint32_t &acc)
{
    const int nib = (int)__builtin_amdgcn_ubfe(tbv, (uint32_t)rc, 4);
    int H = LOCAL ? Hp + nib - 8 : Hp + nib;
    if (LOCAL) {
        H = imax(H, floor);
        const uint32_t key = ((uint32_t)H << 10) | (uint32_t)ci;   // ci < 1024
        bestKey = bestKey > key ? bestKey : key;
    }
    acc <<= 4;
    Hp = H;
    Ep = 0;
}

// exclusive prefix min, init at lane 0
__device__ __forceinline__ int wave_excl_scan_min(int v, int /*lane*/, int init)
{
    return dpp<DPP_WAVE_SHR1>(init, wave_scan_dpp(v, INT32_MAX, op_min));
}

// ---------------------------------------------------------------------------
// Two extensions per wave.  Lanes 0-31 hold one extension and lanes 32-63
// another; lane kl = lane & 31 of a half is diagonal d0 + kl, d0 = center -
// XCENTER.  The band is the seeded diagonal +- hb (og_band_half: the gap
// limit bowtie2 puts on its DP rectangle, at most its maxhalf of 15), so
// lanes 1 .. 31 cover the widest band and lane 0 of a half is never live.  A
// lane outside its band holds values near 0 (minus infinity under the bias)
// and its E and F constants are HUGE_NEG; the same constants sit on the top
// live lane for E and on every dead lane for F, so the two moves that cross
// between the halves (E into lane 31 from lane 32, F into lane 32 from lane
// 31) carry nothing.  The deletion scan stops at 32 lanes (no row_bcast:31).
// ---------------------------------------------------------------------------
constexpr int XCENTER = 16;            // lane of the seeded diagonal within a half
constexpr int HUGE_NEG = -(1 << 24);   // an E / F constant that can never win
constexpr int XREFW_PAD = 48;          // ref window bytes past the last row

// One extension's LDS tables (a wave holds two, after the traceback bits).
// Rows are allocated for at least one staging round (256 rows and 320
// reference bytes), so the one-round staging writes them unguarded.
struct XView {
    uint32_t *tab;    // max(rows, RUNS_CAP): score nibbles per row, then CIGAR runs
    uint8_t *refw;    // rows + 64 (>= rows_pad + XREFW_PAD): ref code * 4 of diagonal d0 + x
    uint8_t *rdc;     // rows: read code | mismatch penalty << 3
    uint8_t *rowk;    // rows: band lane of the M cell of each row, 255 none
};

// rows of the tables: a one-round staging (rows_pad <= 256 or <= 320, see
// stage_raw) writes all of its rows unguarded
__host__ __device__ constexpr int xview_rows(int rows_pad)
{
    return rows_pad <= 256 ? 256 : rows_pad <= 320 ? 320 : rows_pad;
}

__host__ __device__ constexpr int xview_tab_words(int rows_pad)
{
    return xview_rows(rows_pad) > RUNS_CAP ? xview_rows(rows_pad) : RUNS_CAP;
}

__host__ __device__ constexpr int xview_bytes(int rows_pad)
{
    return (4 * xview_tab_words(rows_pad) + 3 * xview_rows(rows_pad) + 64 + 15) & ~15;
}

__device__ __forceinline__ XView xview(unsigned char *base, int rows_pad, int h)
{
    unsigned char *p = base + (size_t)h * xview_bytes(rows_pad);
    const int rows = xview_rows(rows_pad);
    XView X;
    X.tab = (uint32_t *)p;
    p += 4 * xview_tab_words(rows_pad);
    X.refw = p;
    p += rows + 64;
    X.rdc = p;
    X.rowk = p + rows;
    return X;
}

// One work item (a candidate extension), wave-uniform.
struct XItem {
    int sid, m, reflen, d0, hb, strand, ref;
    int64_t roff, gref;
};

// inclusive prefix max within each 32-lane half (rows 0-1 and rows 2-3)
__device__ __forceinline__ int half_scan_max(int v)
{
    v = op_max(v, dpp<0x111>(INT32_MIN, v));
    v = op_max(v, dpp<0x112>(INT32_MIN, v));
    v = op_max(v, dpp<0x114>(INT32_MIN, v));
    v = op_max(v, dpp<0x118>(INT32_MIN, v));
    v = op_max(v, dpp<0x142, 0xA>(INT32_MIN, v));
    return v;
}

// signed 64-bit max of each half (high words, then low words as unsigned
// among the lanes holding the high maximum); k0 / k1 wave-uniform
__device__ __forceinline__ void half_max64(long long v, int lane, long long &k0, long long &k1)
{
    const int hi = (int)(v >> 32);
    const int s = half_scan_max(hi);
    const int h0 = __builtin_amdgcn_readlane(s, 31), h1 = __builtin_amdgcn_readlane(s, 63);
    const int mine = lane < 32 ? h0 : h1;
    const int lo = (int)((uint32_t)v ^ 0x80000000u);
    const int s2 = half_scan_max(hi == mine ? lo : INT32_MIN);
    const int l0 = __builtin_amdgcn_readlane(s2, 31), l1 = __builtin_amdgcn_readlane(s2, 63);
    k0 = (long long)(((uint64_t)(uint32_t)h0 << 32) | (uint32_t)(l0 ^ (int)0x80000000u));
    k1 = (long long)(((uint64_t)(uint32_t)h1 << 32) | (uint32_t)(l1 ^ (int)0x80000000u));
}

// ---------------------------------------------------------------------------
// Exact ungapped fast path of k_dp.
//
// Every path through the band that contains a gap pays at least one open +
// extend, gmin = min(oeI, oeD) (13 with --rdg/--rfg 10,3), and scores at most
// ma per M row, so the DP value of any cell (i, k) is
//     H(i, k) = max(U(i, k), g)   with g <= Gb(i) = ma * (i + 1) - gmin,
// where U is the ungapped recurrence along diagonal k alone (no gap can open
// before row GBAR, so Gb only applies from there).  Hence if the best
// ungapped cell (S, i*, kb) satisfies
//   (A) S > Gb(m - 1)                      (no gapped cell reaches S),
//   (B) U(i, k) < S for every k != kb      (bounded by ma * matches(k) in
//       local mode, -non_matches(k) at the last row end-to-end),
//   (C) U(r, kb) >= Gb(r) on every row r of the traced segment (so H = U
//       there and the traceback's "diagonal first" choice is the same),
// the full DP picks the same best cell and traces the same all-M path.  The
// fast path then hands that path (and its local stop) to finish_ext, and
// k_dp skips the DP and the traceback walk; otherwise (any condition false,
// read > 512 nt) it runs the full DP.
// The candidate is the seeded diagonal (band lane XCENTER): its exact
// ungapped recurrence decides (A) first, then a per-diagonal non-match count
// (4 rows per LDS word; wave lane L counts band lane L - 16) bounds every
// other live diagonal for (B) and stops once all are below.  The whole wave
// works on the one extension.  The result is bit-identical to the full DP
// (tests/test_gpu_parity.py runs both and compares them with the oracle,
// og_mapper.c:dp_extend).
// ---------------------------------------------------------------------------
// Local mode, up to three non-matches on the seeded diagonal kb (rows x_t,
// each scoring s_t, e_t = ma - s_t): the crude bound Gb prices a gapped path
// as matching every row, and fails as soon as two non-matches cost more than
// one gap.  Against kb, a path P over rows [a, b] gains per row s_P(i) -
// s(i, kb): at most e_t at a non-match row x_t, and -ma or less at any other
// row where P's diagonal does not match the read or P inserts the row (kb
// matches there, P scores <= 0); kb's own sum over [a, b] is <= S (and <=
// U(r, kb) when P ends at (r, kb)).  So P beats kb only by covering a run
// x_j .. x_l (j < l) of the non-match rows (one e_t < gmin never pays a
// gap), and then gains at most
//     sum_{t=j..l} e_t - ma * (penalty rows strictly inside, x_t excluded)
//                      - (its gaps).
// Two or more gaps: G = sum e_t - 2 gmin < 0 is required.  One gap, three
// shapes (the band lanes are diagonals; a gap of d lanes costs at least
// gc(d) = min(oeI + exI (d-1), oeD + exD (d-1)) >= gmin):
//  (i)  kb, then one other diagonal k (or k, then kb): the rows of the run
//       off kb are one interval at an end, all of them on k or inserted, so
//       the penalty is at least c_k = k's non-matches in the whole run; it
//       is enough that sum e - ma c_k < gc(|k - kb|) for every live k;
//  (ii) k1, then k2, both off kb (k1 covering the run up to a row c, k2
//       after, any inserted rows between are penalty rows too): the penalty
//       is at least P_k1(c) + Q_k2(c), k1's non-matches in (x_j, c] and k2's
//       in (c, x_l).  With R = sum e - gmin and n = floor(R / ma) + 1, P can
//       only gain if some c has P_k1(c) <= n - 1 and Q_k2(c) <= n - 1, i.e.
//       c < f_k1 (the row of k1's n-th non-match from x_j, or x_l) and
//       c >= g_k2 (the row of k2's n-th from x_l, or x_j); it is enough that
//       min over lanes of g < max over lanes of f never holds (k1 = k2 is
//       let in: only more conservative).
// One wave, lane = diagonal as in (B).  Each run is scanned word by word from
// both ends and the scans stop as soon as every other live lane has met its
// count (n non-matches), which is a few words on ordinary sequence; a
// low-complexity stretch (every diagonal matching long stretches) scans the
// whole run or fails.

// offset (0 .. 3) of the k-th (1-based) set row of a per-row mask (one bit per
// byte), from the low end
__device__ __forceinline__ int sel_row(uint32_t x, int k)
{
    uint32_t b = (x | x >> 7 | x >> 14 | x >> 21) & 0xFu;
    if (k > 1) b &= b - 1;
    if (k > 2) b &= b - 1;
    if (k > 3) b &= b - 1;
    return __builtin_ctz(b);
}

// bytes u of the word at row i with i + u in (lo, hi)
__device__ __forceinline__ uint32_t rows_between(int i, int lo, int hi)
{
    const int a = lo + 1 - i, b = hi - i;
    const uint32_t ma_ = a <= 0 ? ~0u : a >= 4 ? 0u : ~0u << (8 * a);
    const uint32_t mb_ = b >= 4 ? ~0u : b <= 0 ? 0u : ~0u >> (8 * (4 - b));
    return ma_ & mb_;
}

// this lane's non-match rows at rows i .. i+3 of its diagonal (one bit per byte)
__device__ __forceinline__ uint32_t nonmatch_word(const uint8_t *rdc, const uint8_t *rp, uint32_t sh, int i)
{
    const uint32_t rd = *(const uint32_t *)(rdc + i) & 0x07070707u;
    const uint32_t rv = __builtin_amdgcn_alignbyte(*(const uint32_t *)(rp + i + 4), *(const uint32_t *)(rp + i), sh) >> 2;
    uint32_t x = (rd ^ rv) | ((rd | rv) & 0x04040404u);
    return (x | (x >> 1) | (x >> 2)) & 0x01010101u;
}

// One run (lo, hi) of a lane's diagonal, row ex (a non-match row of kb inside
// the run, or -1) left out.  Forward: cnt = the lane's non-matches counted
// (all of the run's unless every other lane had reached n first), f = the row
// of its n-th (hi if none).  Backward: g = the row of its n-th from hi (lo if
// none).  Live lanes only; the loops end together.
__device__ __forceinline__ void scan_run(const uint8_t *rdc, const uint8_t *rp, uint32_t sh, bool other,
                                         int lo, int hi, int ex, int n, int &cnt, int &f, int &g)
{
    const uint32_t exm = ex >= 0 ? ~(1u << (8 * (ex & 3))) : ~0u;
    const int exw = ex & ~3;
    cnt = 0;
    f = hi;
    for (int i = (lo + 1) & ~3; i < hi; i += 4) {
        uint32_t x = nonmatch_word(rdc, rp, sh, i) & rows_between(i, lo, hi);
        if (i == exw) x &= exm;
        const int p = __builtin_popcount(x);
        if (cnt < n && cnt + p >= n) f = i + sel_row(x, n - cnt);
        cnt += p;
        if (__builtin_amdgcn_ballot_w64(other && cnt < n) == 0) break;
    }
    int c = 0;
    g = lo;
    for (int i = (hi - 1) & ~3; i + 3 > lo; i -= 4) {
        uint32_t x = nonmatch_word(rdc, rp, sh, i) & rows_between(i, lo, hi);
        if (i == exw) x &= exm;
        const int p = __builtin_popcount(x);
        if (c < n && c + p >= n) g = i + sel_row(x, p - (n - c) + 1);
        c += p;
        if (__builtin_amdgcn_ballot_w64(other && c < n) == 0) break;
    }
}

template <int LOCAL>
__device__ bool ungapped_wide(const XView &X, int m, int lane, int hb, int nm, uint32_t xm0, uint32_t xm1,
                              int oeI, int exI, int oeD, int exD)
{
    const uint32_t *tab = X.tab;
    const uint8_t *refw = X.refw, *rdc = X.rdc;
    const int ma = 2;
    const int kb = XCENTER;
    const int gmin = oeI < oeD ? oeI : oeD;
    // the non-match rows in order (lane L holds rows 4L .. 4L+3 in xm0 and
    // 256 + 4L .. in xm1, one bit per byte)
    int xs[3] = {0, 0, 0}, es[3] = {0, 0, 0};
    int G = 0;
#pragma unroll
    for (int t = 0; t < 3; ++t) {
        if (t < nm) {
            const int f = xm0 ? 4 * lane + (__builtin_ctz(xm0) >> 3)
                              : xm1 ? 256 + 4 * lane + (__builtin_ctz(xm1) >> 3) : INT32_MAX;
            const int x = __builtin_amdgcn_readfirstlane(wave_min(f));
            if (f == x) {
                if (xm0) xm0 &= xm0 - 1;
                else xm1 &= xm1 - 1;
            }
            xs[t] = x;
            es[t] = ma - ((int)__builtin_amdgcn_ubfe(tab[x], (uint32_t)refw[x + kb], 4) - 8);
            G += es[t];
            if (es[t] >= gmin) return false;
        }
    }
    if (G >= 2 * gmin) return false;
    if (nm <= 1) return true;   // one gap already costs more than the one non-match
    // this lane's diagonal
    const int kl = lane - 16;
    const bool other = kl >= XCENTER - hb && kl <= XCENTER + hb && kl != kb;
    const int kr = other ? kl : 0;
    const uint8_t *rp = refw + (kr & ~3);
    const uint32_t sh = (uint32_t)(kr & 3);
    const int d = kl > kb ? kl - kb : kb - kl;
    const int gI = oeI + exI * (d - 1), gD = oeD + exD * (d - 1);
    const int gc = gI < gD ? gI : gD;
    // the runs: (x0, x1), and with three non-matches (x1, x2) and (x0, x2)
    // without x1
    bool fail = false;
    const int nruns = nm == 3 ? 3 : 1;
    for (int r = 0; r < nruns; ++r) {
        const int lo = r == 1 ? xs[1] : xs[0];
        const int hi = r == 0 ? xs[1] : xs[2];
        const int ex = r == 2 ? xs[1] : -1;
        const int esum = r == 0 ? es[0] + es[1] : r == 1 ? es[1] + es[2] : G;
        const int R = esum - gmin;
        if (R < 0) continue;                 // gc >= gmin: no shape can gain
        const int n = R / ma + 1;
        int cnt, f, g;
        scan_run(rdc, rp, sh, other, lo, hi, ex, n, cnt, f, g);
        // (i): esum - ma * c_k < gc, with cnt = c_k or cnt >= n
        if (esum - ma * cnt >= gc) fail = true;
        // (ii)
        const int gminl = wave_min(other ? g : INT32_MAX);
        const int fmaxl = wave_max(other ? f : INT32_MIN);
        if (gminl < fmaxl) return false;
    }
    return __builtin_amdgcn_ballot_w64(other && fail) == 0;
}

template <int LOCAL>
__device__ bool dp_ungapped(const XView &X, int m, int lane, int gmin, int hb, int &best, int &bi,
                            int &bl, int &low, int oeI, int exI, int oeD, int exD)
{
    const uint32_t *tab = X.tab;
    const uint8_t *refw = X.refw, *rdc = X.rdc;
    const int ma = LOCAL ? 2 : 0;
    const int gb_max = ma * m - gmin;   // Gb(m - 1)
    const int kb = XCENTER;             // the seeded diagonal: the only candidate lane
    // ---- screen for (A): every non-match of the seeded diagonal scores <= -1
    // (end-to-end, where a match scores 0) or loses ma (local), so S <= -nm
    // or S <= ma * (m - nm).  Lane L compares rows 4L .. 4L+3 (and 256 on),
    // one LDS word of read codes against one of reference codes (the window
    // of lane XCENTER is word-aligned). ----
    // (local, <= 3 non-matches: ungapped_wide decides where Gb does not)
    int nm = 0;
    uint32_t xm0 = 0, xm1 = 0;
    {
#pragma unroll
        for (int r = 0; r < 2; ++r) {
            const int i = 4 * lane + 256 * r;
            if (i < m) {
                const uint32_t rd = *(const uint32_t *)(rdc + i) & 0x07070707u;
                const uint32_t rv = *(const uint32_t *)(refw + i + kb) >> 2;
                uint32_t x = (rd ^ rv) | ((rd | rv) & 0x04040404u);
                x = (x | (x >> 1) | (x >> 2)) & 0x01010101u;
                if (m - i < 4) x &= (1u << (8 * (m - i))) - 1u;   // rows past the read
                nm += __builtin_popcount(x);
                if (r == 0) xm0 = x;
                else xm1 = x;
            }
        }
        nm = wave_sum(nm);
    }
    const bool wide = LOCAL && nm <= 3;
    if ((LOCAL ? ma * (m - nm) : -nm) <= gb_max && !wide) return false;
    // ---- exact ungapped recurrence on band lane kb: rows 8*lane .. 8*lane+7 ----
    const int r0 = 8 * lane;
    int s[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
        const int r = r0 + u;
        s[u] = r < m ? (int)__builtin_amdgcn_ubfe(tab[r], (uint32_t)refw[r + kb], 4) - 8 : 0;
    }
    int tot = 0;
#pragma unroll
    for (int u = 0; u < 8; ++u) tot += s[u];
    const int pbase = wave_excl_scan(tot, lane);   // prefix sum before row r0
    int P[8], mn = 0;
    {
        int p = pbase, lm = INT32_MAX;
#pragma unroll
        for (int u = 0; u < 8; ++u) {
            p += s[u];
            P[u] = p;
            lm = p < lm ? p : lm;
        }
        mn = wave_excl_scan_min(lm, lane, 0);      // min(0, prefix sums before r0)
        mn = mn < 0 ? mn : 0;
    }
    int H[8];
    int hbest = -1, rbest = 0;
#pragma unroll
    for (int u = 0; u < 8; ++u) {
        if (LOCAL) {
            mn = P[u] < mn ? P[u] : mn;
            H[u] = P[u] - mn;           // Kadane: max(H(r-1) + s(r), 0)
        } else {
            H[u] = P[u];
        }
        if (LOCAL && r0 + u < m && H[u] > hbest) { hbest = H[u]; rbest = r0 + u; }
    }
    int S, istar;
    if (LOCAL) {
        const int k2 = wave_max(hbest >= 0 ? hbest * 1024 + (1023 - rbest) : -1);
        S = k2 >> 10;
        istar = 1023 - (k2 & 1023);
    } else {
        const int last = m - 1;
        int v = 0;
#pragma unroll
        for (int u = 0; u < 8; ++u) if (r0 + u == last) v = H[u];
        S = __builtin_amdgcn_readlane(v, __builtin_amdgcn_readfirstlane(last >> 3));
        istar = last;
    }
    // (A)
    const bool crude = S > gb_max;
    if (!crude && !wide) return false;
    if (LOCAL && S <= 0) return false;
    // (B): non-matches per diagonal, read bytes rdc[i..i+3] against ref bytes
    // refw[i+kl .. i+kl+3] (codes * 4), 16 rows per step with every LDS read
    // of the step issued before any is used.  The bound ma*(m - nm) (local)
    // or -nm (end-to-end) only falls as rows are counted, so the count stops
    // as soon as every other live diagonal is below S.
    {
        const int kl = lane - 16;
        const bool other = kl >= XCENTER - hb && kl <= XCENTER + hb && kl != kb;
        const int kr = other ? kl : 0;
        const uint8_t *rp = refw + (kr & ~3);
        const uint32_t sh = (uint32_t)(kr & 3);
        int nm = 0;
        bool below = false;
        for (int i = 0; i < m; i += 16) {
            uint32_t rd[4], lo[4], hi[4];
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                rd[u] = *(const uint32_t *)(rdc + i + 4 * u) & 0x07070707u;   // codes without the penalties
                lo[u] = *(const uint32_t *)(rp + i + 4 * u);
                hi[u] = *(const uint32_t *)(rp + i + 4 * u + 4);
            }
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                if (i + 4 * u >= m) break;
                const uint32_t rv = __builtin_amdgcn_alignbyte(hi[u], lo[u], sh) >> 2;
                uint32_t x = (rd[u] ^ rv) | ((rd[u] | rv) & 0x04040404u);
                x = (x | (x >> 1) | (x >> 2)) & 0x01010101u;
                nm += __builtin_popcount(x);
            }
            if (i + 16 <= m) {   // (rows past the read would count as non-matches)
                const int ub = LOCAL ? ma * (m - nm) : -nm;
                if (__builtin_amdgcn_ballot_w64(other && ub >= S) == 0) { below = true; break; }
            }
        }
        if (!below) {
            nm -= (4 - (m & 3)) & 3;   // rows past the read end are coded 4
            const int ub = LOCAL ? ma * (m - nm) : -nm;
            if (__builtin_amdgcn_ballot_w64(other && ub >= S) != 0) return false;
        }
    }
    // start of the traced segment: last row <= i* where H == 0 (local)
    int istop = -1;
    if (LOCAL) {
        int z = -1;
#pragma unroll
        for (int u = 0; u < 8; ++u) if (r0 + u <= istar && H[u] == 0) z = r0 + u;
        istop = wave_max(z);
    }
    // (C)
    bool bad = false;
    const int lo = istop > 0 ? istop : 0;
#pragma unroll
    for (int u = 0; u < 8; ++u) {
        const int r = r0 + u;
        if (r >= lo && r <= istar && r >= GBAR && H[u] < ma * (r + 1) - gmin) bad = true;
    }
    if (!crude || __builtin_amdgcn_ballot_w64(bad) != 0) {
        if (!wide || !ungapped_wide<LOCAL>(X, m, lane, hb, nm, xm0, xm1, oeI, exI, oeD, exD)) return false;
    }
    best = S;
    bi = istar;
    bl = kb;
    low = istop;   // the path is rows istop + 1 .. istar of lane kb, all M
    return true;
}

// Staging of one extension: its per-row score tables, read codes and
// reference window go into its half's LDS tables.

// Row i of the tables from the read's base code c (4: ambiguous, already
// complemented on the reverse strand) and quality character qc; rows past the
// read (live = false) get code 4 and a nibble of 8 (score 0).
template <int LOCAL>
__device__ __forceinline__ void put_row(const XView &X, int i, bool live, uint32_t c, int qc)
{
    const uint32_t ma = LOCAL ? 2 : 0;
    // branch-free (a branch here serialises the staging's LDS reads): lm is
    // all ones on a row of the read
    const uint32_t lm = 0u - (uint32_t)live;
    const uint32_t pen = (uint32_t)mm_pen(qc) & lm;
    c = (c & lm) | (4u & ~lm);
    // nibble g = score(g) + 8: -pen for a mismatch, ma for g == c, -NPEN when
    // either side is ambiguous (g == 4 or c == 4); past the read all 8 (0)
    const uint32_t mis = (8u - pen) * 0x1111u | (uint32_t)(8 - NPEN) << 16;
    const uint32_t hit = mis + (ma + pen) * (1u << (4 * (c & 3)));
    uint32_t tb = c < 4 ? hit : 0x11111u * (uint32_t)(8 - NPEN);
    tb = (tb & lm) | (0x88888u & ~lm);
    X.tab[i] = tb;
    X.rdc[i] = (uint8_t)(c | pen << 3);
    X.rowk[i] = 255;
}

// Reads longer than one round of 256 rows (4 per lane) and 320 reference
// bytes (5 per lane): every load of a round is issued before any is used.
struct StageRegs {
    uint32_t nmw[4], sqw[4], qv[4], gv[5];
};

__device__ __forceinline__ void stage_load(const DpArgs &A, int m, int strand, int64_t roff, int d0,
                                           int reflen, int64_t gref, int i0, int x0, int lane,
                                           StageRegs &S)
{
#pragma unroll
    for (int u = 0; u < 4; ++u) {
        const int i = i0 + 64 * u + lane;
        const int b = i < m ? (strand ? m - 1 - i : i) : 0;
        const int64_t g = roff + b;
        S.nmw[u] = A.R.nmask[g >> 5];
        S.sqw[u] = A.R.seq2[g >> 4];
        S.qv[u] = A.R.qual[g];
    }
#pragma unroll
    for (int u = 0; u < 5; ++u) {
        int j = d0 + x0 + 64 * u + lane;
        j = j < 0 ? 0 : (j >= reflen ? reflen - 1 : j);
        S.gv[u] = A.I.codes[gref + j];
    }
}

template <int LOCAL>
__device__ __forceinline__ void stage_rows(const DpArgs &A, const XItem &it, const XView &X, int i0,
                                           int lane, const StageRegs &S)
{
    const int m = it.m;
#pragma unroll
    for (int u = 0; u < 4; ++u) {
        const int i = i0 + 64 * u + lane;
        if (i >= A.rows_pad) break;
        const int64_t g = it.roff + (it.strand ? m - 1 - i : i);
        uint32_t c = ((S.nmw[u] >> (g & 31)) & 1) ? 4u : ((S.sqw[u] >> (2 * (g & 15))) & 3u);
        if (it.strand && c < 4) c = 3 - c;
        put_row<LOCAL>(X, i, i < m, c, (int)S.qv[u]);
    }
}

__device__ __forceinline__ void stage_ref(const DpArgs &A, const XItem &it, const XView &X, int x0,
                                          int lane, const StageRegs &S)
{
    const int wref = A.rows_pad + XREFW_PAD;
#pragma unroll
    for (int u = 0; u < 5; ++u) {
        const int x = x0 + 64 * u + lane, j = it.d0 + x;
        const uint32_t g = (j >= 0 && j < it.reflen) ? S.gv[u] : 4u;
        if (x < wref) X.refw[x] = (uint8_t)(g * 4);
    }
}

// Reads of more than one round (rows_pad > 320) load and store 256 rows and
// 320 reference bytes per round (stage_ext)
constexpr int STAGE_ROWS = 256;

// Reads of one round (rows_pad <= ROUND, 256 or 320) are staged in two
// halves: k_dp issues the next item's raw bytes into a per-wave raw area by
// LDS-DMA (global_load_lds_dword: no VGPR destination, so nothing in the
// compiler's waits depends on them) before the current item's DP and
// traceback, and builds the tables from the raw area when the item's turn
// comes.  Raw area (RawLayout<ROUND>): the qualities (one dword per lane per
// 256 rows); the 2-bit words (16 bases each, lanes 0 .. ROUND/16 - 1) and
// N-mask words (32 bases each, the next ROUND/32 lanes) of the read; 128
// dwords of reference codes from the aligned dword below the window's first
// byte (the window is rows_pad + XREFW_PAD <= 368 bytes).
template <int ROUND>
struct RawLayout {
    static constexpr int QUAL = ROUND <= 256 ? 256 : 512;   // quality bytes
    static constexpr int WORDS = QUAL;                      // offset of the read's words
    static constexpr int NSEQ = ROUND / 16;                 // lanes loading 2-bit words
    static constexpr int NMASK = ROUND / 32;                // lanes loading N-mask words
    static constexpr int REF = WORDS + 256;                 // offset of the reference dwords
    static constexpr int BYTES = REF + 512;
    static constexpr int ROW_ROUNDS = ROUND / 64;           // rows per lane
    static constexpr int REF_ROUNDS = ROUND <= 256 ? 5 : 6; // reference bytes per lane
};

__host__ __device__ constexpr int raw_bytes(int rows_pad)
{
    return rows_pad <= 256 ? RawLayout<256>::BYTES : rows_pad <= 320 ? RawLayout<320>::BYTES : 0;
}

// s_waitcnt vmcnt(0): every vector memory operation of the wave, the
// LDS-DMA of stage_dma included, has completed
__device__ __forceinline__ void vm_wait() { __builtin_amdgcn_s_waitcnt(0x3f70); }

__device__ __forceinline__ void dma4(const void *g, unsigned char *lds)
{
    __builtin_amdgcn_global_load_lds((const void *)g, (__attribute__((address_space(3))) void *)lds, 4, 0, 0);
}

template <int ROUND>
__device__ __forceinline__ void stage_dma(const DpArgs &A, const XItem &x, unsigned char *raw, int lane)
{
    using RL = RawLayout<ROUND>;
    // qualities: lane l the bytes 4l .. 4l+3 of each 256 rows of the read (a
    // lane past the read re-reads its first dword)
#pragma unroll
    for (int k = 0; k < RL::QUAL / 256; ++k) {
        const int b = 256 * k + 4 * lane;
        dma4(A.R.qual + x.roff + (b < x.m ? b : 0), raw + 256 * k);
    }
    // 2-bit words (16 bases each) and N-mask words (32 bases each); roff is a
    // multiple of 32
    const int64_t sw = x.roff >> 4, nw = x.roff >> 5;
    const int nl = lane - RL::NSEQ;
    const uint32_t *sp = A.R.seq2 + sw + (16 * lane < x.m && lane < RL::NSEQ ? lane : 0);
    const uint32_t *np = A.R.nmask + nw + (nl >= 0 && nl < RL::NMASK && 32 * nl < x.m ? nl : 0);
    dma4(lane < RL::NSEQ ? (const void *)sp : (const void *)np, raw + RL::WORDS);
    // reference codes: dwords from the aligned dword at or below gref + d0,
    // clamped into the code array (bytes off the reference are masked later)
    const int64_t a0 = (x.gref + x.d0) & ~(int64_t)3;
    const int64_t last = ((A.I.total + 64) & ~(int64_t)3) - 4;
#pragma unroll
    for (int k = 0; k < 2; ++k) {
        int64_t a = a0 + 4 * (64 * k + lane);
        a = a < 0 ? 0 : (a > last ? last : a);
        dma4(A.I.codes + a, raw + RL::REF + 256 * k);
    }
}

// the tables of an item whose raw bytes stage_dma brought in (after a wait
// for the wave's vector memory operations)
template <int LOCAL, int ROUND>
__device__ __forceinline__ void stage_raw(const DpArgs &A, const XItem &it, const XView &X,
                                          const unsigned char *raw, int lane)
{
    using RL = RawLayout<ROUND>;
    constexpr int NR = RL::ROW_ROUNDS, NX = RL::REF_ROUNDS;
    const int m = it.m;
    const uint32_t *sw = (const uint32_t *)(raw + RL::WORDS), *nw = sw + RL::NSEQ;
    // every LDS read first (no branches: rows past the read read base 0)
    int b[NR];
    uint32_t nmw[NR], sqw[NR], qv[NR], gv[NX];
#pragma unroll
    for (int u = 0; u < NR; ++u) {
        const int i = 64 * u + lane;
        b[u] = i < m ? (it.strand ? m - 1 - i : i) : 0;
        nmw[u] = nw[b[u] >> 5];
        sqw[u] = sw[b[u] >> 4];
        qv[u] = raw[b[u]];
    }
    const int sh = (int)((it.gref + it.d0) & 3);
#pragma unroll
    for (int u = 0; u < NX; ++u) gv[u] = raw[RL::REF + sh + 64 * u + lane];
#pragma unroll
    for (int u = 0; u < NR; ++u) {   // rows 0 .. ROUND - 1 (the tables hold them)
        const int i = 64 * u + lane;
        uint32_t c = ((nmw[u] >> (b[u] & 31)) & 1) ? 4u : ((sqw[u] >> (2 * (b[u] & 15))) & 3u);
        if (it.strand && c < 4) c = 3 - c;
        put_row<LOCAL>(X, i, i < m, c, (int)qv[u]);
    }
#pragma unroll
    for (int u = 0; u < NX; ++u) {   // reference bytes 0 .. 64 NX - 1 (the window holds rows + 64)
        const int x = 64 * u + lane, j = it.d0 + x;
        const uint32_t g = (j >= 0 && j < it.reflen) ? gv[u] : 4u;
        X.refw[x] = (uint8_t)(g * 4);
    }
}

// Staging of reads longer than one round: the rounds load and store in turn.
template <int LOCAL>
__device__ __forceinline__ void stage_ext(const DpArgs &A, const XItem &it, const XView &X, int lane)
{
    const int wref = A.rows_pad + XREFW_PAD;
    for (int r0 = 0; r0 < A.rows_pad || 320 * (r0 / STAGE_ROWS) < wref; r0 += STAGE_ROWS) {
        const int x0 = 320 * (r0 / STAGE_ROWS);
        StageRegs S;
        stage_load(A, it.m, it.strand, it.roff, it.d0, it.reflen, it.gref, r0, x0, lane, S);
        if (r0 < A.rows_pad) stage_rows<LOCAL>(A, it, X, r0, lane, S);
        if (x0 < wref) stage_ref(A, it, X, x0, lane, S);
    }
}

// A row that is a gap row on some lanes and not on others, or past the read
// of one half: the gap row with E and F switched off where the row has no
// gap window (its nibble then says "diagonal", as the oracle's does), and no
// update at all past the read.  Only the first and last GBAR-ish rows of an
// extension come here.
template <int LOCAL>
__device__ __forceinline__ void dp_row_any(uint32_t tbv, int rc, int &Hp, int &Ep, uint32_t &bestKey,
                                           int ci, const DpConst &K, uint32_t &acc, bool gap,
                                           bool liverow)
{
    DpConst K2 = K;
    K2.mexI = gap ? K.mexI : HUGE_NEG;
    K2.cF = gap ? K.cF : HUGE_NEG;
    int hp = Hp, ep = Ep;
    uint32_t bk = bestKey, a = acc;
    dp_row_gap<LOCAL>(tbv, rc, hp, ep, bk, ci, K2, a);
    Hp = liverow ? hp : Hp;
    Ep = liverow ? ep : Ep;
    bestKey = liverow ? bk : bestKey;
    acc = liverow ? a : acc << 4;
}

// The banded DP of the wave's two extensions (X0 on lanes 0-31, X1 on lanes
// 32-63) over rows, 8 rows per group (one u32 of traceback bits per lane);
// groups inside both gap windows run branch-free.  Returns each half's best
// cell: max score, then smallest row, then smallest band lane.
template <int LOCAL>
__device__ void dp_pair(const DpArgs &A, const XView &X0, const XView &X1, int m0, int m1, int hb0,
                        int hb1, uint32_t *bits, int lane, int &best0, int &bi0, int &bl0,
                        int &best1, int &bi1, int &bl1)
{
    const int h = lane >> 5, kl = lane & 31;
    const uint32_t *tab = h ? X1.tab : X0.tab;
    const uint8_t *refw = (h ? X1.refw : X0.refw) + kl;
    const int ml = h ? m1 : m0, hb = h ? hb1 : hb0;
    const bool live = kl >= XCENTER - hb && kl <= XCENTER + hb;
    DpConst K;
    K.mexI = (live && kl < XCENTER + hb) ? -(A.exI + A.exD) + (LOCAL ? 0 : 8) : HUGE_NEG;
    K.dIE = A.exI - A.oeI;
    K.cF = live ? -(A.oeD - A.exD) : HUGE_NEG;
    K.floor = live ? BIAS + A.exD * lane : 0;
    int Hp = K.floor, Ep = 0;   // row -1: H = 0 (shifted, see DpConst); dead lanes near 0
    uint32_t bestKey = 0;
    const int mlo = m0 < m1 ? m0 : m1, mhi = m0 < m1 ? m1 : m0;
    for (int i0 = 0; i0 < mhi; i0 += 8) {
        uint32_t tbv[8];
        int rcv[8];
#pragma unroll
        for (int t = 0; t < 8; ++t) {
            tbv[t] = tab[i0 + t];
            rcv[t] = refw[i0 + t];
        }
        uint32_t acc = 0;
        if (i0 >= GBAR && i0 + 8 <= mlo - GBAR) {
            int pd[4];
            dp_row_gap_pipe<LOCAL, false>(tbv[0], rcv[0], Hp, Ep, bestKey, 1023 - i0, K, acc, pd);
#pragma unroll
            for (int t = 1; t < 8; ++t)
                dp_row_gap_pipe<LOCAL, true>(tbv[t], rcv[t], Hp, Ep, bestKey, 1023 - (i0 + t), K, acc, pd);
            acc = push_sign(acc, pd[0]);
            acc = push_sign(acc, pd[1]);
            acc = push_sign(acc, pd[2]);
            acc = push_sign(acc, pd[3]);
        } else if (m0 == m1) {
            // both halves end on the same row: a row's gap window is the same
            // on every lane (wave-uniform branches), rows past the read are
            // skipped
#pragma unroll
            for (int t = 0; t < 8; ++t) {
                const int i = i0 + t;
                if (i >= m0) acc <<= 4;   // past the read: an empty nibble
                else if (i >= GBAR && i < m0 - GBAR)
                    dp_row_gap<LOCAL>(tbv[t], rcv[t], Hp, Ep, bestKey, 1023 - i, K, acc);
                else
                    dp_row_nogap<LOCAL>(tbv[t], rcv[t], Hp, Ep, bestKey, 1023 - i, K.floor, acc);
            }
        } else {
#pragma unroll
            for (int t = 0; t < 8; ++t) {
                const int i = i0 + t;
                dp_row_any<LOCAL>(tbv[t], rcv[t], Hp, Ep, bestKey, 1023 - i, K, acc,
                                  i >= GBAR && i < ml - GBAR, i < ml);
            }
        }
        bits[(i0 >> 3) * 64 + lane] = acc;
    }
    int bestH, bestI;
    if (LOCAL) {
        bestH = (int)(bestKey >> 10) - BIAS - A.exD * lane;
        bestI = 1023 - (int)(bestKey & 1023u);
    } else {
        bestH = Hp - BIAS - A.exD * lane - 8 * ml;   // end-to-end: the last row
        bestI = ml - 1;
    }
    const long long key = (long long)bestH * 1048576ll + (long long)((1023 - bestI) << 6) +
                          (long long)(63 - lane);
    long long k0, k1;
    half_max64(key, lane, k0, k1);
    best0 = (int)(k0 >> 20);
    bi0 = 1023 - (int)((k0 >> 6) & 1023);
    bl0 = (63 - (int)(k0 & 63)) & 31;
    best1 = (int)(k1 >> 20);
    bi1 = 1023 - (int)((k1 >> 6) & 1023);
    bl1 = (63 - (int)(k1 & 63)) & 31;
}

// What a traceback leaves for post_ext besides the CIGAR runs (back to
// front in X.tab) and the band lane of every M row (X.rowk).
struct WalkOut {
    int tb_ok, t_start, t_first, t_nrun;   // wave-uniform
    int path_cnt;                          // per lane: ambiguous << 16 | mismatches of its M rows
};

// Traceback of one extension whose traceback bits sit in columns hcol ..
// hcol + 31 of the wave's bits, with the whole wave.
template <int LOCAL>
__device__ WalkOut walk1(const DpArgs &A, const XItem &it, const XView &X, const uint32_t *bits,
                         int hcol, int best, int bi, int bl, int lane, int fast_low)
{
    const int ma = LOCAL ? 2 : 0;
    const int m = it.m, d0 = it.d0;
    const int klo = XCENTER - it.hb, khi = XCENTER + it.hb;
    uint32_t *runs = X.tab;   // the DP is done with the score tables
    const uint8_t *refw = X.refw, *rdc = X.rdc;
    uint8_t *rowk = X.rowk;
    const int minsc = ldc(&A.len_tab[(MAXLEN + 1) + m]);

    // ---- traceback: CIGAR runs, back to front, and the band lane of every
    // M row (rowk) for the lane-parallel statistics below.  The walk's state
    // is wave-uniform (SGPRs, scalar branches).  A diagonal run is found in
    // one step: lane L tests the traceback word of row group (i >> 3) - L on
    // the current diagonal, and a ballot gives the first group below row i
    // that holds a non-diagonal cell (one LDS round trip per run instead of
    // one per 8 rows).  In local mode the walk carries the value of its cell
    // (hv): down a run the lanes rebuild H row by row (a prefix sum of the
    // run's scores) and the first H == 0 is the stop the oracle takes
    // (og_mapper.c dp_extend, src 0).  Gap moves are single steps.  Only
    // lane 0 writes runs. ----
    int tb_ok = 0, t_start = 0, t_first = 0, t_nrun = 0;
    int path_cnt = 0;   // this lane's M rows of the path: ambiguous << 16 | mismatches
    best = __builtin_amdgcn_readfirstlane(best);
    bi = __builtin_amdgcn_readfirstlane(bi);
    bl = __builtin_amdgcn_readfirstlane(bl);
    fast_low = __builtin_amdgcn_readfirstlane(fast_low);
    if (fast_low > -2) {
        // the fast path's all-M path (rows fast_low + 1 .. bi of band lane
        // bl, its local stop included): the walk would find one M run
        if (!(LOCAL && best <= 0) && best >= __builtin_amdgcn_readfirstlane(minsc)) {
            const int len = bi - fast_low;
            if (lane == 0) runs[0] = ((uint32_t)len << 4) | (uint32_t)MH_OP_M;
            for (int r0 = bi; r0 > fast_low; r0 -= 256) {   // lane L: rows r0 - 4L .. r0 - 4L - 3
                int rb[4], g[4];
#pragma unroll
                for (int u = 0; u < 4; ++u) {
                    const int r = r0 - 4 * lane - u;
                    rb[u] = r > fast_low ? rdc[r] & 7 : 0;
                    g[u] = r > fast_low ? refw[r + bl] >> 2 : 0;
                }
#pragma unroll
                for (int u = 0; u < 4; ++u) {
                    const int r = r0 - 4 * lane - u;
                    if (r > fast_low) {
                        rowk[r] = (uint8_t)bl;
                        const int amb = rb[u] > 3 || g[u] > 3;
                        path_cnt += (amb << 16) + (amb || rb[u] != g[u]);
                    }
                }
            }
            tb_ok = 1;
            t_start = fast_low + 1;
            t_first = fast_low + 1 + d0 + bl;
            t_nrun = 1;
        }
    } else if (!(LOCAL && best <= 0) && best >= __builtin_amdgcn_readfirstlane(minsc)) {
        int i = bi, k = bl, state = 0, ok = 1, hv = best;
        int wr = -1, wk = -1;
        uint32_t word = 0;
        int rop = -1, rlen = 0, nrun = 0, first_j = 0;
        for (;;) {
            if (state == 0) {
                // rf: the highest row <= i on diagonal k whose source is
                // not the diagonal (-1: the run reaches row 0)
                int rf = -1;
                uint32_t wf = 0;
                for (int g0 = i >> 3, top = i & 7; g0 >= 0; g0 -= 64, top = 7) {
                    const int g = g0 - lane;
                    uint32_t w = g >= 0 ? bits[g * 64 + hcol + k] : 0u;
                    if (lane == 0 && top < 7)   // rows above i count as diagonal
                        w &= ~((1u << (4 * (7 - top))) - 1u);
                    const uint32_t nd = w & TB_ND_ALL;
                    const uint64_t hit = __builtin_amdgcn_ballot_w64(nd != 0);
                    if (hit) {
                        const int L = (int)__builtin_ctzll(hit);
                        wf = (uint32_t)__builtin_amdgcn_readlane((int)w, L);
                        const uint32_t ndf = (uint32_t)__builtin_amdgcn_readlane((int)nd, L);
                        rf = (g0 - L) * 8 + 7 - (int)(__builtin_ctz(ndf) >> 2);
                        break;
                    }
                }
                // the rows rf + 1 .. i of the run, 256 per round (lane L: rows
                // r0 - 4L .. r0 - 4L - 3), read once for the local stop, the
                // band lane of every M row (rowk) and the n-ceil / mismatch
                // counts.  Local mode rebuilds H(r) = hv minus the scores of
                // the diagonal moves out of the rows above r; the highest row
                // of rf .. i with H == 0 is the stop, and the run is the rows
                // above it.
                int stop = -1;
                const int lo = LOCAL ? (rf > 0 ? rf : 0) : rf + 1;
                for (int r0 = i; r0 >= lo; r0 -= 256) {
                    int rb[4], gc[4];
#pragma unroll
                    for (int u = 0; u < 4; ++u) {
                        const int r = r0 - 4 * lane - u;
                        rb[u] = r > rf ? rdc[r] : 0;
                        gc[u] = r > rf ? refw[r + k] >> 2 : 0;
                    }
                    int stop_c = -1, run = 0;
                    if (LOCAL) {
                        int sc[4], tot = 0;
#pragma unroll
                        for (int u = 0; u < 4; ++u) {
                            const int r = r0 - 4 * lane - u, c = rb[u] & 7;
                            sc[u] = r <= rf ? 0 : (c > 3 || gc[u] > 3) ? -NPEN
                                                  : (c == gc[u] ? ma : -(rb[u] >> 3));
                            tot += sc[u];
                        }
                        run = wave_excl_scan(tot, lane);
                        int zrow = -1;
#pragma unroll
                        for (int u = 0; u < 4; ++u) {
                            const int r = r0 - 4 * lane - u;
                            if (zrow < 0 && r >= lo && hv - run == 0) zrow = r;
                            run += sc[u];
                        }
                        const uint64_t z = __builtin_amdgcn_ballot_w64(zrow >= 0);
                        if (z) stop_c = __builtin_amdgcn_readlane(zrow, (int)__builtin_ctzll(z));
                    }
#pragma unroll
                    for (int u = 0; u < 4; ++u) {
                        const int r = r0 - 4 * lane - u, c = rb[u] & 7;
                        if (r > rf && r > stop_c) {
                            rowk[r] = (uint8_t)k;
                            const int amb = c > 3 || gc[u] > 3;
                            path_cnt += (amb << 16) + (amb || c != gc[u]);
                        }
                    }
                    if (stop_c >= 0) { stop = stop_c; break; }
                    if (LOCAL) hv -= __builtin_amdgcn_readlane(run, 63);
                }
                const int low = stop >= 0 ? stop : rf;
                if (i > low) {   // rows low+1 .. i: one M run
                    const int len = i - low;
                    if (rop == MH_OP_M) rlen += len;
                    else {
                        if (rlen) {
                            if (nrun >= RUNS_CAP - 1) { ok = 0; break; }
                            if (lane == 0) runs[nrun] = ((uint32_t)rlen << 4) | (uint32_t)rop;
                            ++nrun;
                        }
                        rop = MH_OP_M;
                        rlen = len;
                    }
                    first_j = low + 1 + d0 + k;
                }
                i = low;
                if (stop >= 0 || i < 0) break;   // a local stop starts the alignment at row i + 1
                const uint32_t nib = (wf >> (4 * (7 - (i & 7)))) & 15u;
                state = (nib & TB_NE) ? 2 : 1;
                continue;
            }
            // a gap step: the extend bit of cell (i, k) sits on band lane k + 1
            // (E, eb') or k - 1 (F, fb')
            const int g = i >> 3, kk = state == 1 ? k + 1 : k - 1;
            if (kk < klo || kk > khi) { ok = 0; break; }
            if (g != wr || kk != wk) {
                word = __builtin_amdgcn_readfirstlane(bits[g * 64 + hcol + kk]);
                wr = g; wk = kk;
            }
            const uint32_t nib = (word >> (4 * (7 - (i & 7)))) & 15u;
            const int op = state == 1 ? MH_OP_I : MH_OP_D;
            if (op == rop) ++rlen;
            else {
                if (rlen) {
                    if (nrun >= RUNS_CAP - 1) { ok = 0; break; }
                    if (lane == 0) runs[nrun] = ((uint32_t)rlen << 4) | (uint32_t)rop;
                    ++nrun;
                }
                rop = op;
                rlen = 1;
            }
            if (op == MH_OP_I) {
                const bool ext = (nib & TB_EB) != 0;
                hv += ext ? A.exI : A.oeI;
                state = ext ? 1 : 0;
                --i; ++k;
                if (i < 0 || k > khi) { ok = 0; break; }
            } else {
                const bool ext = (nib & TB_FB) != 0;
                hv += ext ? A.exD : A.oeD;
                state = ext ? 2 : 0;
                --k;
                if (k < klo) { ok = 0; break; }
            }
        }
        if (rlen) {
            if (lane == 0) runs[nrun] = ((uint32_t)rlen << 4) | (uint32_t)rop;
            ++nrun;
        }
        tb_ok = ok;
        t_start = i + 1;
        t_first = first_j;
        t_nrun = nrun;
    }
    return WalkOut{tb_ok, t_start, t_first, t_nrun, path_cnt};
}

// Overhang trimming, statistics, the CIGAR and the slot of one extension
// after its traceback (W's first four fields wave-uniform).
template <int LOCAL>
__device__ void post_ext(const DpArgs &A, const XItem &it, const XView &X, int best, int bi, int bl,
                         int lane, int64_t &ck_base, int &ck_left, const WalkOut &W)
{
    const int m = it.m, reflen = it.reflen, d0 = it.d0;
    const uint32_t *runs = X.tab;
    const uint8_t *refw = X.refw, *rdc = X.rdc, *rowk = X.rowk;
    int tb_ok = W.tb_ok;
    const int t_start = W.t_start, t_first = W.t_first, t_nrun = W.t_nrun, path_cnt = W.path_cnt;
    Slot out{};
    out.valid = 0;
    out.strand = it.strand;
    out.ref = it.ref;
    if (tb_ok) {
        // trim overhanging columns into soft clips, on the runs (lane 0)
        int lo = t_nrun - 1, hi = 0;   // forward order is runs[nrun-1] .. runs[0]
        uint32_t front = 0, back = 0;
        int clipL = t_start, clipR = m - 1 - bi, jL = t_first, jR = bi + d0 + bl;
        if (lane == 0) {
            front = lo >= 0 ? runs[lo] : 0;
            back = runs[0];
            while (lo >= hi) {
                const int op = front & 15, len = (int)(front >> 4);
                if (op == MH_OP_M && jL >= 0) break;
                if (op == MH_OP_M) {
                    const int t = -jL < len ? -jL : len;
                    clipL += t; jL += t;
                    if (t < len) { front = ((uint32_t)(len - t) << 4) | MH_OP_M; continue; }
                } else if (op == MH_OP_I) {
                    clipL += len;
                } else {
                    jL += len;
                }
                if (--lo >= hi) front = runs[lo];
            }
            if (lo == hi) back = front;   // one run left: keep the front's trim
            while (hi <= lo) {
                const int op = back & 15, len = (int)(back >> 4);
                if (op == MH_OP_M && jR < reflen) break;
                if (op == MH_OP_M) {
                    const int t = jR - reflen + 1 < len ? jR - reflen + 1 : len;
                    clipR += t; jR -= t;
                    if (t < len) { back = ((uint32_t)(len - t) << 4) | MH_OP_M; continue; }
                } else if (op == MH_OP_I) {
                    clipR += len;
                } else {
                    jR -= len;
                }
                if (++hi <= lo) back = hi == lo ? front : runs[hi];
            }
        }
        clipL = __builtin_amdgcn_readfirstlane(clipL);
        clipR = __builtin_amdgcn_readfirstlane(clipR);
        // ambiguous positions over the untrimmed alignment (--n-ceil) and
        // mismatches over the trimmed one, summed together (nn << 16 | xm):
        // counted along the path by the traceback, so only a trim that moved
        // a clip (the path overhangs a reference end, or starts / ends with
        // an insertion) needs a pass over the M rows
        int cnt = path_cnt;
        if (clipL != t_start || clipR != m - 1 - bi) {
            cnt = 0;
            for (int i = t_start + lane; i <= bi; i += 64) {
                const int k = rowk[i];
                if (k == 255) continue;
                const int g = refw[i + k] >> 2, rb = rdc[i] & 7;
                if (rb > 3 || g > 3) cnt += 1 << 16;
                if ((rb > 3 || g > 3 || rb != g) && i >= clipL && i <= m - 1 - clipR) ++cnt;
            }
        }
        cnt = wave_sum(cnt);
        if ((cnt >> 16) > ldc(&A.len_tab[2 * (MAXLEN + 1) + m])) tb_ok = 0;
        if (tb_ok && lane == 0 && lo >= hi) {
            const int nc = (clipL > 0) + (clipR > 0) + (lo - hi + 1);
            if (nc <= MH_MAXOPS - 1) {
                if (nc > ck_left) {   // next wave-private chunk of the pool
                    ck_base = (int64_t)atomicAdd(A.pool_used, (unsigned long long)POOL_CHUNK);
                    ck_left = POOL_CHUNK;
                }
                const int64_t base = ck_base;
                ck_base += nc;
                ck_left -= nc;
                if (base + nc > A.pool_cap) {
                    atomicExch(&A.pool_ctr[1], 1);
                } else {
                    uint32_t *cg = A.pool + base;
                    int n = 0, xo = 0, xg = 0, mx = 0;
                    if (clipL) cg[n++] = ((uint32_t)clipL << 4) | MH_OP_S;
                    for (int z = lo; z >= hi; --z) {
                        const uint32_t rr = z == hi ? back : (z == lo ? front : runs[z]);
                        cg[n++] = rr;
                        if ((rr & 15) != MH_OP_M) { ++xo; xg += (int)(rr >> 4); }
                        else if ((int)(rr >> 4) > mx) mx = (int)(rr >> 4);
                    }
                    if (clipR) cg[n++] = ((uint32_t)clipR << 4) | MH_OP_S;
                    out.valid = 1;
                    out.pos = jL;
                    out.end = jR + 1;
                    out.score = best;
                    out.xo = xo; out.xg = xg;
                    out.n_cigar = n;
                    out.cig_off = (int32_t)base;
                    out.xm = cnt & 0xffff;
                    out.nm = out.xm + xg;
                    out.maxm = mx;
                }
            }
        }
    }
    if (lane == 0) {
        const int64_t at = slot_at(it.sid, A.plane);
        A.skey[at] = SlotKey{out.valid ? (out.ref << 1 | out.strand) : -1, out.pos, out.end, out.score};
        A.sinfo[at] = SlotInfo{out.cig_off, (uint32_t)out.xm | (uint32_t)out.xo << 16,
                                   (uint32_t)out.xg | (uint32_t)out.n_cigar << 16, out.maxm};
    }
    wave_sync();
}

// Traceback, overhang trimming, statistics and the slot of one extension.
template <int LOCAL>
__device__ void finish_ext(const DpArgs &A, const XItem &it, const XView &X, const uint32_t *bits,
                           int hcol, int best, int bi, int bl, int lane, int64_t &ck_base,
                           int &ck_left, int fast_low = -2)
{
    best = __builtin_amdgcn_readfirstlane(best);
    bi = __builtin_amdgcn_readfirstlane(bi);
    bl = __builtin_amdgcn_readfirstlane(bl);
    const WalkOut W = walk1<LOCAL>(A, it, X, bits, hcol, best, bi, bl, lane, fast_low);
    wave_sync();
    post_ext<LOCAL>(A, it, X, best, bi, bl, lane, ck_base, ck_left, W);
}

// k_dp: a wave walks its share of the work list.  Each item is staged into
// the free half's tables and tried on the exact ungapped fast path (the
// whole wave); an item that needs the DP waits in half 0 until a second one
// fills half 1, then both run through the rows together.  A last waiting
// item runs with half 1 repeating it.
template <int LOCAL, int ROUND>
__global__ __launch_bounds__(256) void k_dp(DpArgs A)
{
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const int lane = threadIdx.x & 63;
    const int wv = wave_uniform(threadIdx.x >> 6);
    const int wpb = blockDim.x >> 6;
    unsigned char *wbase = smem + (size_t)wv * A.wave_lds;
    uint32_t *bits = (uint32_t *)wbase;                       // rows_pad/8 * 64: 4 bits/cell
    unsigned char *xbase = wbase + (size_t)32 * A.rows_pad;
    const XView X0 = xview(xbase, A.rows_pad, 0), X1 = xview(xbase, A.rows_pad, 1);
    unsigned char *raw = xbase + 2 * xview_bytes(A.rows_pad);   // RawLayout<ROUND> (reads of one round)
    const int n_work = A.counters[0];
    const int gmin = A.oeI < A.oeD ? A.oeI : A.oeD;

    int64_t ck_base = 0;   // lane 0: this wave's current CIGAR pool chunk
    int ck_left = 0;
    int n_fast = 0;        // extensions resolved by dp_ungapped
    // Work items come in chunks of QCH from a queue: a wave's first chunk is
    // its own (wave id), the next ones are taken by one atomic each on lane 0,
    // issued a chunk ahead, so the waves of a launch sized to what is resident
    // finish together.  Item position p of the wave is chunk cA's item p (or,
    // past QCH, chunk cB's item p - QCH).
    // Software pipeline over the items, three deep: while item w is aligned,
    // the candidate and read descriptors of the item after next are loaded
    // (scalar loads; and the work id of the one after that), and the next
    // item, whose descriptors landed during the previous one, gets its
    // reference window and (reads of one staging round) its raw bytes issued
    // by LDS-DMA, so they land while w is aligned.  A wave then waits on no
    // global round trip between items.
    constexpr int QCH = DP_QUEUE_CHUNK;
    const int gwaves = gridDim.x * wpb;
    constexpr bool one_round = ROUND > 0;   // rows_pad <= ROUND
    int cA = (blockIdx.x * wpb + wv) * QCH, cB = 0, qv = 0, p = 0;
    auto grab = [&]() {   // lane 0: the base of a later chunk (in flight until read)
        if (lane == 0) qv = atomicAdd(A.queue, QCH) + gwaves * QCH;
    };
    grab();
    cB = __builtin_amdgcn_readfirstlane(qv);
    grab();
    auto at = [&](int d) {   // item index at position p + d (d <= 3 < QCH)
        const int q = p + d;
        return q < QCH ? cA + q : cB + (q - QCH);
    };
    int w = cA;
    XItem cur{};                       // item w: every field, staging issued
    int sid1 = 0, m1 = 0, sid2 = 0;    // next item: work id, candidate, read; the one after: work id
    Cand cd1{};
    int64_t roff1 = 0;
    auto to_item = [&](int sid, const Cand &cd, int m, int64_t roff) {
        XItem x;
        x.sid = sid;
        x.m = m;
        x.roff = roff;
        x.d0 = cd.center - XCENTER;
        x.strand = cd.strand;
        x.ref = cd.ref;
        x.reflen = ldc(&A.I.ref_len[cd.ref]);
        x.gref = ldc(&A.I.ref_off[cd.ref]);
        x.hb = ldc(&A.len_tab[3 * (MAXLEN + 1) + m]);
        if (one_round) stage_dma<ROUND ? ROUND : 256>(A, x, raw, lane);
        return x;
    };
    if (w < n_work) {
        const int sid = ldc(&A.work[w]);
        cur = to_item(sid, ldc_cand(&A.cand[slot_at(sid, A.plane)]), ldc(&A.R.len[sid / MAXCAND]),
                      ldc(&A.R.off[sid / MAXCAND]));
    }
    if (at(1) < n_work) {
        sid1 = ldc(&A.work[at(1)]);
        cd1 = ldc_cand(&A.cand[slot_at(sid1, A.plane)]);
        m1 = ldc(&A.R.len[sid1 / MAXCAND]);
        roff1 = ldc(&A.R.off[sid1 / MAXCAND]);
    }
    if (at(2) < n_work) sid2 = ldc(&A.work[at(2)]);
    bool pend = false;     // half 0 holds an item waiting for the DP
    bool landed = false;   // the raw bytes of `cur` were waited for
    XItem P{};
    while (w < n_work) {
        const XItem it = cur;
        const int h = pend ? 1 : 0;
        const XView X = h ? X1 : X0;
        if (one_round) {
            if (!landed) vm_wait();   // (after a pending item: nothing ran to cover them)
            stage_raw<LOCAL, ROUND ? ROUND : 256>(A, it, X, raw, lane);
        } else {
            stage_ext<LOCAL>(A, it, X, lane);
        }
        wave_sync();
        int best = 0, bi = 0, bl = 0, low = -1;
        const bool fast = it.m > 2 * GBAR + 8 && it.m <= 512 &&
                          dp_ungapped<LOCAL>(X, it.m, lane, gmin, it.hb, best, bi, bl, low, A.oeI, A.exI,
                                            A.oeD, A.exD);
        n_fast += fast;
        if (at(1) < n_work) cur = to_item(sid1, cd1, m1, roff1);
        if (at(2) < n_work) {
            sid1 = sid2;
            cd1 = ldc_cand(&A.cand[slot_at(sid2, A.plane)]);
            m1 = ldc(&A.R.len[sid2 / MAXCAND]);
            roff1 = ldc(&A.R.off[sid2 / MAXCAND]);
        }
        if (at(3) < n_work) sid2 = ldc(&A.work[at(3)]);
        // The next item's raw bytes are waited for before this item's
        // traceback stores anything: the vector memory counter is in order,
        // so a wait after the stores would also wait for their write acks.
        landed = false;
        if (fast) {
            wave_sync();
            if (one_round) { vm_wait(); landed = true; }
            finish_ext<LOCAL>(A, it, X, bits, 32 * h, best, bi, bl, lane, ck_base, ck_left, low);
        } else if (!pend) {
            P = it;
            pend = true;
        } else {
            int b0, i0, l0, b1, i1, l1;
            dp_pair<LOCAL>(A, X0, X1, P.m, it.m, P.hb, it.hb, bits, lane, b0, i0, l0, b1, i1, l1);
            wave_sync();
            if (one_round) { vm_wait(); landed = true; }
            finish_ext<LOCAL>(A, P, X0, bits, 0, b0, i0, l0, lane, ck_base, ck_left);
            finish_ext<LOCAL>(A, it, X1, bits, 32, b1, i1, l1, lane, ck_base, ck_left);
            pend = false;
        }
        if (++p == QCH) {   // into the next chunk; take the one after it
            p = 0;
            cA = cB;
            cB = __builtin_amdgcn_readfirstlane(qv);
            grab();
        }
        w = at(0);
    }
    if (pend) {
        int b0, i0, l0, b1, i1, l1;
        dp_pair<LOCAL>(A, X0, X0, P.m, P.m, P.hb, P.hb, bits, lane, b0, i0, l0, b1, i1, l1);
        wave_sync();
        finish_ext<LOCAL>(A, P, X0, bits, 0, b0, i0, l0, lane, ck_base, ck_left);
    }
    if (lane == 0 && n_fast) atomicAdd(&A.pool_ctr[2], n_fast);
}

// ---------------------------------------------------------------------------
// k_rescue: mate rescue (og_mapper.c rescue_pair / rescue_diagonal).  When
// exactly one mate of a pair aligned, the other is looked for in the -X
// window next to the aligned mate, on the opposite strand: the diagonal with
// the most base matches over the window (ties: leftmost) becomes the mate's
// only candidate and k_dp extends it like any other.  One wave per 64 pairs:
// lane = pair for the test, then the whole wave scans each selected mate's
// window, lane = diagonal, 4 read bases per LDS word.
// ---------------------------------------------------------------------------
struct RescueArgs {
    DevReads R;
    DevIndex I;
    const SlotKey *skey;
    int32_t *n_cand;
    const int32_t *yf;
    Cand *cand;
    int32_t *work;        // rescue work list (slot ids)
    int32_t *counter;     // [0] rescue work items
    int maxins;
    int64_t plane;        // slot planes' stride (slot_at)
};

// diagonals per staged reference window (the -X window of C2 has ~950)
constexpr int RESCUE_CHUNK = 1024;
constexpr int RESCUE_WORDS = (RESCUE_CHUNK + MAXLEN) / 16 + 4;   // 2-bit words of a staged window
constexpr int RESCUE_W32 = (RESCUE_CHUNK + MAXLEN) / 32 + 4;     // bit-plane words of a staged window

// the 16 low bits of each bit pair of x, packed into 16 bits
__device__ __forceinline__ uint32_t compact16(uint32_t x)
{
    x &= 0x55555555u;
    x = (x | (x >> 1)) & 0x33333333u;
    x = (x | (x >> 2)) & 0x0f0f0f0fu;
    x = (x | (x >> 4)) & 0x00ff00ffu;
    return (x | (x >> 8)) & 0x0000ffffu;
}

__device__ __forceinline__ int best_slot(const SlotKey *skey, int64_t r, int n, int64_t plane)
{
    int best = -1, bs = 0;
    for (int c = 0; c < n; ++c) {
        const SlotKey k = skey[(int64_t)c * plane + r];
        if (k.rs >= 0 && (best < 0 || k.score > bs)) { best = c; bs = k.score; }
    }
    return best;
}

__global__ __launch_bounds__(256) void k_rescue(RescueArgs A)
{
    // the mate and the reference window as 2-bit words (16 bases each) plus
    // "N" masks (01 in the base's bit pair)
    __shared__ uint32_t sh_rd[4][2][MAXLEN / 16 + 1];
    __shared__ uint32_t sh_rf[4][2][RESCUE_WORDS];
    // the same as bit planes (32 bases a word: low code bits, high code bits)
    // for the count without ambiguous bases
    __shared__ uint2 sh_rp[4][MAXLEN / 32 + 1];
    __shared__ uint2 sh_pl[4][RESCUE_W32];
    __shared__ int32_t sh_items[4][64];
    const int lane = threadIdx.x & 63;
    const int wv = wave_uniform(threadIdx.x >> 6);
    uint32_t *rdw = sh_rd[wv][0], *rdn = sh_rd[wv][1];
    uint32_t *rfw = sh_rf[wv][0], *rfn = sh_rf[wv][1];
    uint2 *rp = sh_rp[wv], *pl = sh_pl[wv];
    const int64_t units = A.R.n / 2;
    for (int64_t u0 = ((int64_t)blockIdx.x * 4 + wv) * 64; u0 < units;
         u0 += (int64_t)gridDim.x * 256) {
        const int64_t u = u0 + lane;
        // the mate to rescue and its anchor (the other mate's best slot)
        int need = 0, tgt_mate = 0, a_ref = 0, a_strand = 0, a_pos = 0, a_end = 0;
        int t_len = 0, r_len = 0;
        int64_t t_off = 0, r_off = 0;   // the mate's and the reference's (loaded lane-parallel here)
        if (u < units) {
            const int64_t r1 = 2 * u, r2 = r1 + 1;
            const int b1 = best_slot(A.skey, r1, A.n_cand[r1], A.plane);
            const int b2 = best_slot(A.skey, r2, A.n_cand[r2], A.plane);
            if ((b1 >= 0) != (b2 >= 0)) {
                const int64_t an = b1 >= 0 ? r1 : r2, tg = b1 >= 0 ? r2 : r1;
                if (A.yf[tg] == 0 && A.R.len[tg] > 0) {
                    const SlotKey s = A.skey[(int64_t)(b1 >= 0 ? b1 : b2) * A.plane + an];
                    need = 1;
                    tgt_mate = b1 >= 0 ? 1 : 0;
                    a_ref = s.rs >> 1; a_strand = s.rs & 1; a_pos = s.pos; a_end = s.end;
                    t_len = A.R.len[tg];
                    t_off = A.R.off[tg];
                    r_len = A.I.ref_len[a_ref];
                    r_off = A.I.ref_off[a_ref];
                }
            }
        }
        uint64_t todo = __builtin_amdgcn_ballot_w64(need != 0);
        int n_items = 0;
        while (todo) {
            const int l = __builtin_ctzll(todo);
            todo &= todo - 1;
            const int64_t tg = 2 * (u0 + l) + __builtin_amdgcn_readlane(tgt_mate, l);
            const int ref = __builtin_amdgcn_readlane(a_ref, l);
            const int ast = __builtin_amdgcn_readlane(a_strand, l);
            const int apos = __builtin_amdgcn_readlane(a_pos, l);
            const int aend = __builtin_amdgcn_readlane(a_end, l);
            const int m = __builtin_amdgcn_readlane(t_len, l);
            const int64_t off = readlane64(t_off, l);
            const int reflen = __builtin_amdgcn_readlane(r_len, l);
            const int64_t gref = readlane64(r_off, l);
            int64_t lo = ast == 0 ? (int64_t)apos : (int64_t)aend - A.maxins;
            int64_t hi = ast == 0 ? (int64_t)apos + A.maxins : (int64_t)aend;
            if (lo < 0) lo = 0;
            if (hi > reflen) hi = reflen;
            if (hi - lo < m) continue;
            const int s = 1 - ast;
            // the mate on strand s; bases past its end count as N (never match)
            const int nw = (m + 15) >> 4;
            bool read_n = false;   // an ambiguous base inside the read
            for (int w = lane; w < nw; w += 64) {
                uint32_t code, nmk;
                read_word2(A.R, off, m, s, w, code, nmk);
                const int nv = m - 16 * w < 16 ? m - 16 * w : 16;
                const uint32_t valid = nv >= 16 ? 0xffffffffu : ((1u << (2 * nv)) - 1u);
                read_n |= (nmk & valid) != 0;
                rdw[w] = code;
                rdn[w] = nmk;
            }
            const bool any_read_n = __builtin_amdgcn_ballot_w64(read_n) != 0;
            wave_sync();
            // the read's bit planes (bases past m are masked in the count)
            const int nw32 = (m + 31) >> 5;
            for (int w = lane; w < nw32; w += 64) {
                const uint32_t c0 = rdw[2 * w], c1 = rdw[2 * w + 1];
                rp[w] = make_uint2(compact16(c0) | (compact16(c1) << 16),
                                   compact16(c0 >> 1) | (compact16(c1 >> 1) << 16));
            }
            const int tail = m - 32 * (nw32 - 1);
            const uint32_t tmask = tail >= 32 ? 0xffffffffu : (1u << tail) - 1u;
            int bestM = -1, bestd = 0;
            const int dlast = (int)(hi - m);
            for (int d0 = (int)lo; d0 <= dlast; d0 += RESCUE_CHUNK) {
                const int nd = dlast - d0 + 1 < RESCUE_CHUNK ? dlast - d0 + 1 : RESCUE_CHUNK;
                // the window's bit planes (bases d0 .. d0 + nd + m - 2 are
                // compared; the ones from hi on are never reached)
                const int nrw32 = (nd + m + 31) / 32 + 1;
                const int64_t wend = d0 + nd + m - 1 < hi ? (int64_t)d0 + nd + m - 1 : hi;
                bool win_n = false;   // an ambiguous reference base among the compared ones
#pragma unroll 1
                for (int w = lane; w < nrw32; w += 64) {
                    const int64_t g = gref + d0 + 32 * w;
                    const uint32_t *cp = A.I.cplane + 2 * (g >> 5);
                    const uint32_t sh = (uint32_t)(g & 31);
                    const uint32_t pl0 = __builtin_amdgcn_alignbit(cp[2], cp[0], sh);
                    const uint32_t pl1 = __builtin_amdgcn_alignbit(cp[3], cp[1], sh);
                    const uint32_t nf = __builtin_amdgcn_alignbit(A.I.ncode[(g >> 5) + 1], A.I.ncode[g >> 5], sh);
                    const int64_t nin = wend - (d0 + 32 * (int64_t)w);
                    const uint32_t valid = nin >= 32 ? 0xffffffffu : (nin > 0 ? (1u << nin) - 1u : 0u);
                    win_n |= (nf & valid) != 0;
                    pl[w] = make_uint2(pl0, pl1);
                }
                wave_sync();
                if (!any_read_n && __builtin_amdgcn_ballot_w64(win_n) == 0) {
                    // no ambiguous base on either side: mismatches over 32 bases
                    // per step from the two planes (the window's words aligned to
                    // the diagonal by a funnel shift, carried over a step); the
                    // last word masks the read's tail
                    for (int t = lane; t < nd; t += 64) {
                        const int w0 = t >> 5;
                        const uint32_t sh = (uint32_t)(t & 31);
                        uint2 cur = pl[w0];
                        int mis = 0;
                        for (int i = 0; i < nw32 - 1; ++i) {
                            const uint2 nx = pl[w0 + i + 1], r = rp[i];
                            const uint32_t x0 = __builtin_amdgcn_alignbit(nx.x, cur.x, sh) ^ r.x;
                            const uint32_t x1 = __builtin_amdgcn_alignbit(nx.y, cur.y, sh) ^ r.y;
                            mis += __builtin_popcount(x0 | x1);
                            cur = nx;
                        }
                        {
                            const uint2 nx = pl[w0 + nw32], r = rp[nw32 - 1];
                            const uint32_t x0 = __builtin_amdgcn_alignbit(nx.x, cur.x, sh) ^ r.x;
                            const uint32_t x1 = __builtin_amdgcn_alignbit(nx.y, cur.y, sh) ^ r.y;
                            mis += __builtin_popcount((x0 | x1) & tmask);
                        }
                        const int cnt = m - mis;
                        if (cnt > bestM) { bestM = cnt; bestd = d0 + t; }
                    }
                    wave_sync();
                    continue;
                }
                // reference bases d0 .. d0 + nd + m (+ one word), N past the window
                const int nrw = (nd + m + 15) / 16 + 1;
#pragma unroll 1
                for (int w = lane; w < nrw; w += 64) {
                    // 16 reference bases from the packed copies (a funnel shift of
                    // two words each); bases from hi on count as ambiguous
                    const int64_t g = gref + d0 + 16 * w;
                    const uint32_t cf = __builtin_amdgcn_alignbit(A.I.code2[(g >> 4) + 1], A.I.code2[g >> 4],
                                                                  (uint32_t)(2 * (g & 15)));
                    const uint32_t nf = __builtin_amdgcn_alignbit(A.I.ncode[(g >> 5) + 1], A.I.ncode[g >> 5],
                                                                  (uint32_t)(g & 31)) & 0xffffu;
                    const int64_t nin = hi - (d0 + 16 * (int64_t)w);
                    const uint32_t valid = nin >= 16 ? 0xffffffffu : (nin > 0 ? (1u << (2 * nin)) - 1u : 0u);
                    uint32_t sp = nf;
                    sp = (sp | (sp << 8)) & 0x00ff00ffu;
                    sp = (sp | (sp << 4)) & 0x0f0f0f0fu;
                    sp = (sp | (sp << 2)) & 0x33333333u;
                    sp = (sp | (sp << 1)) & 0x55555555u;
                    sp = (sp & valid) | (~valid & 0x55555555u);
                    rfw[w] = cf & ~(sp * 3u) & valid;
                    rfn[w] = sp;
                }
                wave_sync();
                for (int t = lane; t < nd; t += 64) {
                    // matches on diagonal d0 + t: 16 bases per step, the window
                    // words aligned to the diagonal by a funnel shift
                    const int w0 = t >> 4;
                    const uint32_t sh = (uint32_t)(2 * (t & 15));
                    int cnt = 0;
                    for (int i = 0; i < nw; ++i) {
                        const uint32_t v = __builtin_amdgcn_alignbit(rfw[w0 + i + 1], rfw[w0 + i], sh);
                        const uint32_t vn = __builtin_amdgcn_alignbit(rfn[w0 + i + 1], rfn[w0 + i], sh);
                        const uint32_t x = rdw[i] ^ v;
                        cnt += __builtin_popcount(~(x | (x >> 1) | rdn[i] | vn) & 0x55555555u);
                    }
                    if (cnt > bestM) { bestM = cnt; bestd = d0 + t; }
                }
                wave_sync();
            }
            const int mmax = wave_max(bestM);
            const int dsel = wave_min(bestM == mmax ? bestd : INT32_MAX);
            if (lane == 0) {
                A.cand[tg] = Cand{s, ref, dsel, 0};   // candidate 0: plane 0
                A.n_cand[tg] = 1;
                sh_items[wv][n_items] = (int32_t)(tg * MAXCAND);
            }
            ++n_items;
        }
        wave_sync();
        if (n_items) {
            int base = 0;
            if (lane == 0) base = atomicAdd(A.counter, n_items);
            base = __builtin_amdgcn_readfirstlane(base);
            if (lane < n_items) A.work[base + lane] = sh_items[wv][lane];
        }
        wave_sync();
    }
}

// ---------------------------------------------------------------------------
// k_pair: pairing, flags, MAPQ (unpinned V2-style table, see og_mapq)
// ---------------------------------------------------------------------------
__device__ int mapq_v2(int local, int perfect, int minsc, int best, int has_sec, int sec)
{
    int diff = perfect - minsc;
    if (diff < 1) diff = 1;
    const int over = best - minsc;
#define GE(x, f10) (10ll * (long long)(x) >= (long long)(f10) * diff)
    if (!has_sec) {
        if (GE(over, 8)) return local ? 44 : 42;
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

struct PairArgs {
    DevReads R;
    const int32_t *len_tab;
    const SlotKey *skey;
    const SlotInfo *sinfo;
    const int32_t *n_cand;
    const int32_t *yf;
    const uint32_t *pool;
    Rec *rec;
    int64_t *ref_stats;  // [5][n_refs] lines, filtered, mapped, first_row, first_mapped; unmapped, star
    int n_refs;
    int local;
    int maxins;
    int paired;
    int64_t plane;       // slot planes' stride (slot_at)
};

// A read's candidates: its keys in registers (one 16-B load each, the
// read's MAXCAND keys are one 64-B line), invalid ones and those past
// n_cand as rs = -1.
struct MateView {
    SlotKey k[MAXCAND];
    int64_t base;    // the read (candidate c at c * plane + base)
    int best;
    SlotKey bk;      // k[best] (copied when chosen: a run-time index into k would
                     // put the view in scratch memory)
};

__device__ __forceinline__ void load_mate(const PairArgs &A, int64_t r, MateView &mv)
{
    mv.base = r;
    const int n = A.n_cand[r];
    mv.best = -1;
    mv.bk = SlotKey{-1, 0, 0, 0};
#pragma unroll
    for (int c = 0; c < MAXCAND; ++c) {
        mv.k[c] = c < n ? A.skey[(int64_t)c * A.plane + r] : SlotKey{-1, 0, 0, 0};
        if (mv.k[c].rs >= 0 && (mv.best < 0 || mv.k[c].score > mv.bk.score)) { mv.best = c; mv.bk = mv.k[c]; }
    }
}

__device__ __forceinline__ void clear_rec(Rec &o)
{
    o.ref = -1; o.pos = 0; o.rev = 0; o.score = 0; o.secbest = I32MIN; o.flag = 0; o.mapq = 0;
    o.rnext = -2; o.pnext = 0; o.tlen = 0; o.sam_ref = -1; o.sam_pos = 0; o.xm = 0; o.xo = 0;
    o.xg = 0; o.nm = 0; o.ys = I32MIN; o.yt = 0; o.yf = 0; o.n_cigar = 0; o.cig_off = 0;
    o.maxm = 0;
}

__device__ __forceinline__ void fill_aligned(const PairArgs &A, Rec &o, const MateView &mv, int chosen,
                                             const SlotKey &a, int m)
{
    o.ref = a.rs >> 1; o.pos = a.pos; o.rev = a.rs & 1; o.score = a.score;
    int sec = 0, has = 0;
#pragma unroll
    for (int c = 0; c < MAXCAND; ++c) {
        const SlotKey b = mv.k[c];
        // same place: strand, reference and position
        if (c == chosen || b.rs < 0 || (b.rs == a.rs && b.pos == a.pos)) continue;
        if (!has || b.score > sec) { sec = b.score; has = 1; }
    }
    o.secbest = has ? sec : I32MIN;
    o.mapq = mapq_v2(A.local, A.local ? 2 * m : 0, A.len_tab[(MAXLEN + 1) + m], a.score, has, sec);
    const SlotInfo f = A.sinfo[(int64_t)chosen * A.plane + mv.base];
    o.xm = (int)(f.xm_xo & 0xffffu); o.xo = (int)(f.xm_xo >> 16);
    o.xg = (int)(f.xg_nc & 0xffffu); o.nm = o.xm + o.xg;
    o.n_cigar = (int)(f.xg_nc >> 16);
    o.cig_off = f.cig_off;
    o.maxm = f.maxm;
    o.sam_ref = o.ref;
    o.sam_pos = a.pos + 1;
}

__device__ __forceinline__ bool concordant(const SlotKey &x, const SlotKey &y, int maxins)
{
    // same reference, opposite strands
    if ((x.rs ^ y.rs) != 1) return false;
    const SlotKey &fw = (x.rs & 1) == 0 ? x : y;
    const SlotKey &rv = (x.rs & 1) == 0 ? y : x;
    const int lo = fw.pos < rv.pos ? fw.pos : rv.pos;
    const int hi = fw.end > rv.end ? fw.end : rv.end;
    if (hi - lo > maxins) return false;
    if (rv.pos < fw.pos && rv.end < fw.end) return false;
    return true;
}

// Per-reference line tallies (remap.py:494-506, :743-755).  Almost every
// read of a pass lands on the same one or two references, so the counters
// are reduced per block in LDS and flushed with one global atomic each.
constexpr int TALLY_LDS_REFS = 256;

struct TallyLds {
    unsigned int lines[TALLY_LDS_REFS], filt[TALLY_LDS_REFS], mapped[TALLY_LDS_REFS];
    int first[TALLY_LDS_REFS], firstm[TALLY_LDS_REFS];
    unsigned int unmapped, star;
    int star_first;
};

__device__ __forceinline__ void tally(const PairArgs &A, TallyLds *T, const Rec &o, int64_t row)
{
    const int n = A.n_refs;
    if (T) {
        if (o.sam_ref >= 0) {
            atomicAdd(&T->lines[o.sam_ref], 1u);
            if (!(o.flag & 4)) {
                if (o.maxm > 50) atomicAdd(&T->filt[o.sam_ref], 1u);
                atomicAdd(&T->mapped[o.sam_ref], 1u);
                atomicMin(&T->firstm[o.sam_ref], (int)row);
            }
            atomicMin(&T->first[o.sam_ref], (int)row);
        } else {
            atomicAdd(&T->star, 1u);
            atomicMin(&T->star_first, (int)row);
        }
        if (o.flag & 4) atomicAdd(&T->unmapped, 1u);
        return;
    }
    if (o.sam_ref >= 0) {
        atomicAdd((unsigned long long *)&A.ref_stats[o.sam_ref], 1ull);
        if (!(o.flag & 4)) {
            if (o.maxm > 50) atomicAdd((unsigned long long *)&A.ref_stats[n + o.sam_ref], 1ull);
            atomicAdd((unsigned long long *)&A.ref_stats[2 * n + o.sam_ref], 1ull);
        }
        atomicMin((long long *)&A.ref_stats[3 * n + o.sam_ref], (long long)row);
        if (!(o.flag & 4)) atomicMin((long long *)&A.ref_stats[4 * n + o.sam_ref], (long long)row);
    } else {
        atomicAdd((unsigned long long *)&A.ref_stats[5 * n + 1], 1ull);
        atomicMin((long long *)&A.ref_stats[5 * n + 2], (long long)row);
    }
    if (o.flag & 4) atomicAdd((unsigned long long *)&A.ref_stats[5 * n], 1ull);
}

__device__ void tally_flush(const PairArgs &A, TallyLds *T)
{
    const int n = A.n_refs;
    unsigned long long *S = (unsigned long long *)A.ref_stats;
    for (int r = threadIdx.x; r < n; r += blockDim.x) {
        if (T->lines[r]) atomicAdd(&S[r], (unsigned long long)T->lines[r]);
        if (T->filt[r]) atomicAdd(&S[n + r], (unsigned long long)T->filt[r]);
        if (T->mapped[r]) atomicAdd(&S[2 * n + r], (unsigned long long)T->mapped[r]);
        if (T->first[r] != INT32_MAX) atomicMin((long long *)&A.ref_stats[3 * n + r], (long long)T->first[r]);
        if (T->firstm[r] != INT32_MAX) atomicMin((long long *)&A.ref_stats[4 * n + r], (long long)T->firstm[r]);
    }
    if (threadIdx.x == 0) {
        if (T->unmapped) atomicAdd(&S[5 * n], (unsigned long long)T->unmapped);
        if (T->star) atomicAdd(&S[5 * n + 1], (unsigned long long)T->star);
        if (T->star_first != INT32_MAX) atomicMin((long long *)&A.ref_stats[5 * n + 2], (long long)T->star_first);
    }
}

__global__ __launch_bounds__(256) void k_pair(PairArgs A)
{
    __shared__ TallyLds sT;
    TallyLds *T = (A.n_refs <= TALLY_LDS_REFS && A.R.n < INT32_MAX) ? &sT : nullptr;
    if (T) {
        for (int r = threadIdx.x; r < TALLY_LDS_REFS; r += blockDim.x) {
            T->lines[r] = T->filt[r] = T->mapped[r] = 0;
            T->first[r] = T->firstm[r] = INT32_MAX;
        }
        if (threadIdx.x == 0) { T->unmapped = T->star = 0; T->star_first = INT32_MAX; }
        __syncthreads();
    }
    const int64_t units = A.paired ? A.R.n / 2 : A.R.n;
    // every thread runs the same trip count so the final barrier is uniform
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    const int64_t trips = (units + stride - 1) / stride;
    for (int64_t it = 0; it < trips; ++it) {
        const int64_t u = it * stride + (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
        if (u >= units) continue;
        if (!A.paired) {
            MateView mv;
            load_mate(A, u, mv);
            Rec o;
            clear_rec(o);
            o.yf = A.yf[u];
            o.yt = 3;
            if (mv.best >= 0) {
                fill_aligned(A, o, mv, mv.best, mv.bk, A.R.len[u]);
                o.flag = o.rev ? 0x10 : 0;
            } else {
                o.flag = 0x4;
            }
            A.rec[u] = o;
            tally(A, T, o, u);
            continue;
        }
        const int64_t r1 = 2 * u, r2 = 2 * u + 1;
        MateView m1, m2;
        load_mate(A, r1, m1);
        load_mate(A, r2, m2);
        Rec o1, o2;
        clear_rec(o1);
        clear_rec(o2);
        o1.yf = A.yf[r1];
        o2.yf = A.yf[r2];
        int c1 = m1.best, c2 = m2.best, conc = 0;
        SlotKey k1 = m1.bk, k2 = m2.bk;
        long long best_sum = -9223372036854775807ll - 1;
#pragma unroll
        for (int x = 0; x < MAXCAND; ++x) {
            const SlotKey sx = m1.k[x];
            if (sx.rs < 0) continue;
#pragma unroll
            for (int y = 0; y < MAXCAND; ++y) {
                const SlotKey sy = m2.k[y];
                if (sy.rs < 0) continue;
                if (!concordant(sx, sy, A.maxins)) continue;
                const long long s = (long long)sx.score + sy.score;
                if (s > best_sum) { best_sum = s; c1 = x; c2 = y; k1 = sx; k2 = sy; conc = 1; }
            }
        }
        const int al1 = c1 >= 0, al2 = c2 >= 0;
        if (al1) fill_aligned(A, o1, m1, c1, k1, A.R.len[r1]);
        if (al2) fill_aligned(A, o2, m2, c2, k2, A.R.len[r2]);
        int f1 = 0x1 | 0x40, f2 = 0x1 | 0x80;
        if (conc) { f1 |= 0x2; f2 |= 0x2; }
        if (!al1) { f1 |= 0x4; f2 |= 0x8; }
        if (!al2) { f2 |= 0x4; f1 |= 0x8; }
        if (al1 && o1.rev) { f1 |= 0x10; f2 |= 0x20; }
        if (al2 && o2.rev) { f2 |= 0x10; f1 |= 0x20; }
        o1.flag = f1;
        o2.flag = f2;
        const int yt = conc ? 0 : (al1 && al2) ? 1 : 2;
        o1.yt = o2.yt = yt;
        if (al1 && al2) {
            o1.ys = o2.score;
            o2.ys = o1.score;
            if (o1.ref == o2.ref) {
                o1.rnext = o2.rnext = -1;
                const SlotKey &a = k1, &b = k2;
                const int lo = a.pos < b.pos ? a.pos : b.pos;
                const int hi = a.end > b.end ? a.end : b.end;
                const int t = hi - lo;
                const bool first1 = a.pos <= b.pos;
                o1.tlen = first1 ? t : -t;
                o2.tlen = first1 ? -t : t;
            } else {
                o1.rnext = o2.ref;
                o2.rnext = o1.ref;
            }
            o1.pnext = o2.sam_pos;
            o2.pnext = o1.sam_pos;
        } else if (al1 || al2) {
            // the aligned mate's place for both (no run-time reference to
            // one of the two records: that puts both in scratch memory)
            const int sref = al1 ? o1.sam_ref : o2.sam_ref;
            const int spos = al1 ? o1.sam_pos : o2.sam_pos;
            const int ascore = al1 ? o1.score : o2.score;
            o1.sam_ref = o2.sam_ref = sref;
            o1.sam_pos = o2.sam_pos = spos;
            o1.rnext = o2.rnext = -1;
            o1.pnext = o2.pnext = spos;
            if (al1) o2.ys = ascore;
            else o1.ys = ascore;
        }
        A.rec[r1] = o1;
        A.rec[r2] = o2;
        tally(A, T, o1, r1);
        tally(A, T, o2, r2);
    }
    if (T) {
        __syncthreads();
        tally_flush(A, T);
    }
}

// ---------------------------------------------------------------------------
// host driver of one mapping pass
// ---------------------------------------------------------------------------
// CIGAR pool words for a pass over n reads (or what a retry found demanded)
static int64_t pool_words_for(int64_t n)
{
    return (n > 0 ? n : 1) * 8 + 4096 + 2 * (int64_t)DP_MAX_BLOCKS * DP_WAVES_PER_BLOCK * POOL_CHUNK;
}

static int ensure_map_buffers(Ctx &c)
{
    MapState &M = c.map;
    const int64_t n = c.reads.n;
    if (M.cap_reads < n || M.cand == nullptr) {
        hipFree(M.cand); hipFree(M.n_cand); hipFree(M.yf); hipFree(M.work);
        hipFree(M.rwork); hipFree(M.skey); hipFree(M.sinfo); hipFree(M.rec);
        const int64_t cap = n > 0 ? n : 1;
        MH_HIP(hipMalloc(&M.cand, sizeof(Cand) * cap * MAXCAND));
        MH_HIP(hipMalloc(&M.n_cand, sizeof(int32_t) * cap));
        MH_HIP(hipMalloc(&M.yf, sizeof(int32_t) * cap));
        MH_HIP(hipMalloc(&M.work, sizeof(int32_t) * cap * MAXCAND));
        MH_HIP(hipMalloc(&M.rwork, sizeof(int32_t) * (cap / 2 + 1)));
        MH_HIP(hipMalloc(&M.skey, sizeof(SlotKey) * cap * MAXCAND));
        MH_HIP(hipMalloc(&M.sinfo, sizeof(SlotInfo) * cap * MAXCAND));
        MH_HIP(hipMalloc(&M.rec, sizeof(Rec) * cap));
        M.cap_reads = cap;
    }
    if (M.counters == nullptr) MH_HIP(hipMalloc(&M.counters, sizeof(int32_t) * 8));
    if (M.cap_refs < c.index.n_refs || M.ref_stats == nullptr) {
        hipFree(M.ref_stats);
        const int cr = c.index.n_refs > 0 ? c.index.n_refs : 1;
        MH_HIP(hipMalloc(&M.ref_stats, sizeof(int64_t) * (5 * cr + 3)));
        M.cap_refs = cr;
    }
    if (M.pool_used == nullptr) MH_HIP(hipMalloc(&M.pool_used, sizeof(unsigned long long)));
    // the ops themselves plus every wave's partly used chunk, for both k_dp
    // launches of a pass (main and mate rescue share the pool); grown when a
    // later pass has more reads than the one that sized it.  A capacity
    // imposed by a test is where every pass starts.
    const int64_t test_cap = c.test_caps.cigar_pool_words;
    const int64_t need = test_cap > 0 ? test_cap : pool_words_for(n);
    // slots and records address the pool with int32 offsets (Slot / Rec cig_off)
    if (need > (int64_t)INT32_MAX) {
        set_error("mh_map: %lld reads need a CIGAR pool past 2^31 words; map them in batches",
                  (long long)n);
        return -3;
    }
    if (M.pool == nullptr || (test_cap > 0 ? M.pool_cap != need : M.pool_cap < need)) {
        hipFree(M.pool);
        M.pool = nullptr;
        M.pool_cap = 0;
        MH_HIP(hipMalloc(&M.pool, sizeof(uint32_t) * need));
        M.pool_cap = need;
    }
    return 0;
}

__global__ void k_init_stats(int64_t *s, int n_refs)
{
    for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < 5 * n_refs + 3; i += gridDim.x * blockDim.x)
        s[i] = ((i >= 3 * n_refs && i < 5 * n_refs) || i == 5 * n_refs + 2) ? INT64_MAX : 0;
}

__global__ void k_fix_first(int64_t *s, int n_refs)
{
    for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < 2 * n_refs; i += gridDim.x * blockDim.x)
        if (s[3 * n_refs + i] == INT64_MAX) s[3 * n_refs + i] = -1;
    if (blockIdx.x == 0 && threadIdx.x == 0 && s[5 * n_refs + 2] == INT64_MAX) s[5 * n_refs + 2] = -1;
}

const int64_t *map_stats_host(Ctx &c)
{
    MapState &M = c.map;
    if (!M.stats_host_valid) {
        M.stats_host.resize(5 * (size_t)M.n_refs + 3);
        const size_t bytes = sizeof(int64_t) * M.stats_host.size();
        if (M.stats_pin_ready) {   // copied at the end of the pass: done by now or at this sync
            if (hipStreamSynchronize(c.stream) != hipSuccess) {
                set_error("map_stats_host: copy failed");
                return nullptr;
            }
            std::memcpy(M.stats_host.data(), M.stats_pin, bytes);
        } else if (hipMemcpyAsync(M.stats_host.data(), M.ref_stats, bytes, hipMemcpyDeviceToHost,
                                  c.stream) != hipSuccess ||
                   hipStreamSynchronize(c.stream) != hipSuccess) {
            set_error("map_stats_host: copy failed");
            return nullptr;
        }
        M.stats_host_valid = true;
    }
    return M.stats_host.data();
}

// ---------------------------------------------------------------------------
// Diagnostics: k_probe_ext runs, for caller-given (read, strand, ref, centre)
// extensions, both the exact ungapped fast path (dp_ungapped) and the full
// banded DP (dp_pair) on the same staged tables, one wave per extension, and
// writes [fast, best, row, lane] of the fast path (zeros when it declines),
// the band half, and [best, row, lane] of the full DP.  Whenever the fast path accepts, the
// full DP must find the same best cell (tests/test_gpu_fastpath.py feeds it
// adversarial low-complexity windows).  Not on any product path.
// ---------------------------------------------------------------------------
template <int LOCAL>
__global__ __launch_bounds__(64) void k_probe_ext(DpArgs A, const int32_t *items, int32_t *out, int n)
{
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const int lane = threadIdx.x & 63;
    const int e = blockIdx.x;
    if (e >= n) return;
    uint32_t *bits = (uint32_t *)smem;
    unsigned char *xbase = smem + (size_t)32 * A.rows_pad;
    const XView X0 = xview(xbase, A.rows_pad, 0);
    const int gmin = A.oeI < A.oeD ? A.oeI : A.oeD;
    const int r = items[4 * e];
    XItem it;
    it.sid = 0;
    it.m = A.R.len[r];
    it.roff = A.R.off[r];
    it.strand = items[4 * e + 1];
    it.ref = items[4 * e + 2];
    it.d0 = items[4 * e + 3] - XCENTER;
    it.reflen = A.I.ref_len[it.ref];
    it.gref = A.I.ref_off[it.ref];
    it.hb = A.len_tab[3 * (MAXLEN + 1) + it.m];
    stage_ext<LOCAL>(A, it, X0, lane);
    wave_sync();
    int best = 0, bi = 0, bl = 0, low = -1;
    const bool fast = it.m > 2 * GBAR + 8 && it.m <= 512 &&
                      dp_ungapped<LOCAL>(X0, it.m, lane, gmin, it.hb, best, bi, bl, low, A.oeI, A.exI,
                                        A.oeD, A.exD);
    wave_sync();
    int b0, i0, l0, b1, i1, l1;
    dp_pair<LOCAL>(A, X0, X0, it.m, it.m, it.hb, it.hb, bits, lane, b0, i0, l0, b1, i1, l1);
    if (lane == 0) {
        int32_t *o = out + 8 * e;
        o[0] = fast;
        o[1] = fast ? best : 0;
        o[2] = fast ? bi : 0;
        o[3] = fast ? bl : 0;
        o[4] = it.hb;
        o[5] = b0;
        o[6] = i0;
        o[7] = l0;
    }
}

int run_probe_ext(Ctx &c, const mh_params &par, int n, const int32_t *items, int32_t *out)
{
    if (c.index.n_refs <= 0 || c.reads.n <= 0 || n < 0) { set_error("mh_probe_extend: no index / reads"); return -3; }
    if (par.mode != MH_E2E && par.mode != MH_LOCAL) { set_error("mh_probe_extend: bad mode"); return -3; }
    if (c.len_tab == nullptr || c.len_tab_key != len_tab_key(par)) { set_error("mh_probe_extend: length tables"); return -3; }
    // every item checked on the host before the launch: read, strand, ref
    for (int e = 0; e < n; ++e) {
        if (items[4 * e] < 0 || items[4 * e] >= c.reads.n || (items[4 * e + 1] & ~1) ||
            items[4 * e + 2] < 0 || items[4 * e + 2] >= c.index.n_refs) {
            set_error("mh_probe_extend: item %d out of range", e);
            return -3;
        }
    }
    if (n == 0) return 0;
    const int rows_pad = ((c.reads.max_len + 7) / 8) * 8;
    const int lds = 32 * rows_pad + 2 * xview_bytes(rows_pad);
    if (lds > 160 * 1024) { set_error("mh_probe_extend: reads too long"); return -3; }
    hipStream_t s = c.stream;
    int32_t *d_items = nullptr, *d_out = nullptr;
    MH_HIP(hipMalloc(&d_items, sizeof(int32_t) * 4 * (size_t)n));
    MH_HIP(hipMalloc(&d_out, sizeof(int32_t) * 8 * (size_t)n));
    MH_HIP(hipMemcpyAsync(d_items, items, sizeof(int32_t) * 4 * (size_t)n, hipMemcpyHostToDevice, s));
    DpArgs da{c.reads, c.index, c.len_tab, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr,
              nullptr, nullptr, nullptr, 0, rows_pad, lds,
              par.rfg_open + par.rfg_ext, par.rfg_ext, par.rdg_open + par.rdg_ext, par.rdg_ext};
    const void *kf = par.mode == MH_LOCAL ? (const void *)k_probe_ext<1> : (const void *)k_probe_ext<0>;
    MH_HIP(hipFuncSetAttribute(kf, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
    if (par.mode == MH_LOCAL) hipLaunchKernelGGL((k_probe_ext<1>), dim3(n), dim3(64), lds, s, da, d_items, d_out, n);
    else hipLaunchKernelGGL((k_probe_ext<0>), dim3(n), dim3(64), lds, s, da, d_items, d_out, n);
    MH_HIP(hipGetLastError());
    MH_HIP(hipMemcpyAsync(out, d_out, sizeof(int32_t) * 8 * (size_t)n, hipMemcpyDeviceToHost, s));
    MH_HIP(hipStreamSynchronize(s));
    hipFree(d_items);
    hipFree(d_out);
    return 0;
}

int run_map(Ctx &c, const mh_params &par)
{
    c.map.stats_host_valid = false;
    c.map.stats_pin_ready = false;
    if (c.index.n_refs <= 0 || c.index.hent == nullptr) {
        set_error("mh_map: no reference index (call mh_index_build first)");
        return -3;
    }
    if (par.mode != MH_E2E && par.mode != MH_LOCAL) { set_error("mh_map: bad mode"); return -3; }
    const int SL = par.mode == MH_LOCAL ? 20 : 22;
    if (c.index.seedlen != SL) {
        set_error("mh_map: index seed length %d does not match mode (%d)", c.index.seedlen, SL);
        return -3;
    }
    if (c.len_tab == nullptr || c.len_tab_key != len_tab_key(par)) {
        set_error("mh_map: length tables not prepared");
        return -3;
    }
    if (int st = ensure_map_buffers(c)) return st;
    MapState &M = c.map;
    const int64_t n = c.reads.n;
    M.n_reads = n;
    M.n_refs = c.index.n_refs;
    M.par = par;
    hipStream_t s = c.stream;
    M.last_work = M.last_cigar = 0;
    if (n == 0) hipLaunchKernelGGL(k_init_stats, dim3(64), dim3(256), 0, s, M.ref_stats, M.n_refs);
    if (n > 0) {
        // seeds, candidates and the work list; run again by a retry, since
        // k_rescue replaces the candidates of the mates it rescues
        auto launch_seed = [&]() -> int {
            SeedArgs sa{c.reads, c.index, par.mode, c.len_tab, M.cand, M.n_cand, M.yf, M.work, M.counters, M.cap_reads};
            int64_t blocks = ((n + SEED_CHUNK - 1) / SEED_CHUNK + 3) / 4;
            if (blocks > 1 << 16) blocks = 1 << 16;
            const int pk = prof_begin(c, "k_seed");
            hipLaunchKernelGGL(k_seed, dim3((unsigned)blocks), dim3(256), 0, s, sa);
            prof_end(c, pk);
            MH_HIP(hipGetLastError());
            return 0;
        };

        const int rows_pad = ((c.reads.max_len + 7) / 8) * 8;
        // traceback bits 32 B per row, the tables of the wave's two
        // extensions, the raw area of a one-round staging
        const int wave_lds = 32 * rows_pad + 2 * xview_bytes(rows_pad) + raw_bytes(rows_pad);
        if (wave_lds > 160 * 1024) { set_error("mh_map: reads too long for LDS"); return -3; }
        // waves per workgroup: the most that keeps the CU's resident waves,
        // floor(160 KiB / (wpb wave_lds)) wpb, at its maximum (at 251-nt reads
        // all of 1 .. 4 give 12; at 300-nt reads 4 would leave 8 of 10)
        int wpb = 1;
        for (int w = DP_WAVES_PER_BLOCK; w >= 1; --w)
            if ((160 * 1024 / (w * wave_lds)) * w > (160 * 1024 / (wpb * wave_lds)) * wpb ||
                ((160 * 1024 / (w * wave_lds)) * w == (160 * 1024 / (wpb * wave_lds)) * wpb && w > wpb))
                wpb = w;
        auto launch_dp = [&](const int32_t *work, const int32_t *count, int32_t *queue,
                             int64_t max_items, const char *name) -> int {
            DpArgs da{c.reads, c.index, c.len_tab, M.cand, work, count, M.skey, M.sinfo, M.pool,
                      M.pool_used, M.counters + 1, queue, M.pool_cap, rows_pad, wave_lds,
                      par.rfg_open + par.rfg_ext, par.rfg_ext, par.rdg_open + par.rdg_ext,
                      par.rdg_ext, M.cap_reads};
            const int round = rows_pad <= 256 ? 256 : rows_pad <= 320 ? 320 : 0;
            const void *kf =
                par.mode == MH_LOCAL
                    ? (round == 256 ? (const void *)k_dp<1, 256> : round ? (const void *)k_dp<1, 320> : (const void *)k_dp<1, 0>)
                    : (round == 256 ? (const void *)k_dp<0, 256> : round ? (const void *)k_dp<0, 320> : (const void *)k_dp<0, 0>);
            // the waves that fit at once (the queue balances them), no more
            // than the items need
            const auto okey = std::make_pair(kf, wpb * wave_lds);
            auto occ = M.dp_occ.find(okey);
            if (occ == M.dp_occ.end()) {
                // the cap every k_dp launch fits under (set once per kernel and shape)
                MH_HIP(hipFuncSetAttribute(kf, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
                if (!c.n_cu) MH_HIP(hipDeviceGetAttribute(&c.n_cu, hipDeviceAttributeMultiprocessorCount, c.device));
                int nb = 0;
                MH_HIP(hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, kf, 64 * wpb, (size_t)wpb * wave_lds));
                occ = M.dp_occ.emplace(okey, nb).first;
            }
            const int per_cu = occ->second;
            int64_t dblocks = (int64_t)(c.n_cu > 0 ? c.n_cu : 256) * (per_cu > 0 ? per_cu : 1);
            const int64_t need = (max_items + (int64_t)wpb * DP_QUEUE_CHUNK - 1) / ((int64_t)wpb * DP_QUEUE_CHUNK);
            if (dblocks > need) dblocks = need;
            if (dblocks > DP_MAX_BLOCKS) dblocks = DP_MAX_BLOCKS;
            if (dblocks < 1) dblocks = 1;
            const int pd = prof_begin(c, name);
            const dim3 grid((unsigned)dblocks), block(64 * wpb);
            const size_t lds = (size_t)wpb * wave_lds;
            if (par.mode == MH_LOCAL) {
                if (round == 256) hipLaunchKernelGGL((k_dp<1, 256>), grid, block, lds, s, da);
                else if (round) hipLaunchKernelGGL((k_dp<1, 320>), grid, block, lds, s, da);
                else hipLaunchKernelGGL((k_dp<1, 0>), grid, block, lds, s, da);
            } else {
                if (round == 256) hipLaunchKernelGGL((k_dp<0, 256>), grid, block, lds, s, da);
                else if (round) hipLaunchKernelGGL((k_dp<0, 320>), grid, block, lds, s, da);
                else hipLaunchKernelGGL((k_dp<0, 0>), grid, block, lds, s, da);
            }
            prof_end(c, pd);
            MH_HIP(hipGetLastError());
            return 0;
        };
        const int64_t units = c.reads.paired ? n / 2 : n;
        PairArgs pa{c.reads, c.len_tab, M.skey, M.sinfo, M.n_cand, M.yf, M.pool, M.rec, M.ref_stats,
                    M.n_refs, par.mode == MH_LOCAL, par.maxins, c.reads.paired, M.cap_reads};
        int64_t pblocks = (units + 255) / 256;
        if (pblocks > 1 << 16) pblocks = 1 << 16;
        if (pblocks < 1) pblocks = 1;
        for (int attempt = 0; attempt < 2; ++attempt) {
            // counters: [0] work items, [2] pool overflow, [3] fast path,
            // [4] rescue work items; pool_used: CIGAR words claimed.  The
            // pairing runs before the overflow check (it reads the slots,
            // not the pool; a retry starts the tallies again), so a pass
            // synchronises once.
            hipLaunchKernelGGL(k_init_stats, dim3(64), dim3(256), 0, s, M.ref_stats, M.n_refs);
            MH_HIP(hipMemsetAsync(M.counters, 0, sizeof(int32_t) * 8, s));
            MH_HIP(hipMemsetAsync(M.pool_used, 0, sizeof(unsigned long long), s));
            if (int st = launch_seed()) return st;
            if (int st = launch_dp(M.work, M.counters, M.counters + 5, n * 2, "k_dp")) return st;
            if (c.reads.paired && units > 0) {
                RescueArgs ra{c.reads, c.index, M.skey, M.n_cand, M.yf, M.cand, M.rwork,
                              M.counters + 4, par.maxins, M.cap_reads};
                int64_t rblocks = (units + 255) / 256;
                if (rblocks > 4096) rblocks = 4096;
                const int pr = prof_begin(c, "k_rescue");
                hipLaunchKernelGGL(k_rescue, dim3((unsigned)rblocks), dim3(256), 0, s, ra);
                prof_end(c, pr);
                MH_HIP(hipGetLastError());
                if (int st = launch_dp(M.rwork, M.counters + 4, M.counters + 6, units, "k_dp_rescue")) return st;
            }
            pa.pool = M.pool;
            const int pp = prof_begin(c, "k_pair");
            hipLaunchKernelGGL(k_pair, dim3((unsigned)pblocks), dim3(256), 0, s, pa);
            prof_end(c, pp);
            MH_HIP(hipGetLastError());
            int32_t ctr[5];
            unsigned long long used = 0;
            MH_HIP(hipMemcpyAsync(ctr, M.counters, sizeof(ctr), hipMemcpyDeviceToHost, s));
            MH_HIP(hipMemcpyAsync(&used, M.pool_used, sizeof(used), hipMemcpyDeviceToHost, s));
            MH_HIP(hipStreamSynchronize(s));
            M.last_work = ctr[0] + ctr[4];
            M.last_rescue = ctr[4];
            M.last_cigar = (int64_t)used;
            M.last_fast = ctr[3];
            if (!ctr[2]) break;
            if (attempt == 1) { set_error("mh_map: CIGAR pool overflow after a retry"); return -2; }
            // CIGAR pool overflow: grow to what was asked for and redo the pass
            // from the seeds (k_rescue rewrote the candidates of the mates it
            // rescued, and their slots point into the pool being replaced)
            ++c.retries[RETRY_CIGAR_POOL];
            hipFree(M.pool);
            M.pool = nullptr;
            M.pool_cap = 0;
            int64_t grown = (int64_t)used * 2 + pool_words_for(0);
            if (grown > (int64_t)INT32_MAX) grown = INT32_MAX;   // int32 cig_off
            if ((int64_t)used > grown) {
                set_error("mh_map: CIGAR pool demand %llu words passes the int32 offsets",
                          (unsigned long long)used);
                return -2;
            }
            MH_HIP(hipMalloc(&M.pool, sizeof(uint32_t) * grown));
            M.pool_cap = grown;
        }
    }
    hipLaunchKernelGGL(k_fix_first, dim3(8), dim3(256), 0, s, M.ref_stats, M.n_refs);
    MH_HIP(hipGetLastError());
    {   // the tallies to pinned memory behind the pass (mh_map's sync covers it)
        const size_t bytes = sizeof(int64_t) * (5 * (size_t)M.n_refs + 3);
        if (M.stats_pin_cap < bytes) {
            if (M.stats_pin) hipHostFree(M.stats_pin);
            M.stats_pin = nullptr;
            M.stats_pin_cap = 0;
            if (hipHostMalloc(&M.stats_pin, bytes, hipHostMallocDefault) == hipSuccess)
                M.stats_pin_cap = bytes;
            else
                M.stats_pin = nullptr;   // map_stats_host copies on demand instead
        }
        if (M.stats_pin && hipMemcpyAsync(M.stats_pin, M.ref_stats, bytes, hipMemcpyDeviceToHost, s) == hipSuccess)
            M.stats_pin_ready = true;
    }
    M.valid = true;
    return 0;
}

}  // namespace mh
