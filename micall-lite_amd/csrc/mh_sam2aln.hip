// mh_sam2aln.hip -- sam2aln on gfx950: the read-pair merge and the count of
// identical merged sequences that micall/core/sam2aln.py:395-478 runs in
// Python over remap.csv, behind mh_sam2aln_csv / mh_sam2aln_output.
//
//   host   remap.csv -> rows (DictReader), matchmaker (sam2aln.py:291-312),
//          the row-level failure causes of parse_sam (:340-348) and the
//          apply_cigar checks that raise (:113-151); insert.csv / failed.csv
//          text and the final ordering of aligned.csv (:465-478)
//   k_s2a_merge   one wave64 per pair: apply_cigar of both mates into LDS,
//                 merge_pairs (q_cutoff 15, no insertions, :156-237)
//                 lane-parallel, prop_N test (:381-385), the merged sequence
//                 written to HBM and hashed (two 64-bit position-keyed sums)
//   k_s2a_count   one thread per merged pair: open-addressing table keyed by
//                 the hash, count + first unit per distinct sequence
//   k_s2a_verify  one wave per merged pair: every member of a group is
//                 compared byte for byte with the group's first member
//                 (a hash collision is reported, never merged silently)
//   k_s2a_gather  distinct sequences copied out for the host's sort
// Bit-for-bit specification: the reference itself (tests/golden/e2e/*/aligned.csv
// etc. were produced by running micall.core.sam2aln on the same remap.csv).
#include <fcntl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <cerrno>
#include <chrono>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#include "mh_gunzip.h"
#include "mh_sam2aln.h"

namespace mh {

static void s2a_free_device(S2AState &S)
{
    hipFree(S.d_seq); hipFree(S.d_qual); hipFree(S.d_out); hipFree(S.d_gather);
    hipFree(S.d_soff); hipFree(S.d_units); hipFree(S.d_slot); hipFree(S.d_goff);
    hipFree(S.d_pos); hipFree(S.d_cigoff); hipFree(S.d_ncig);
    hipFree(S.d_uref); hipFree(S.d_res); hipFree(S.d_tcnt); hipFree(S.d_trep);
    hipFree(S.d_uniq); hipFree(S.d_ctr); hipFree(S.d_cig); hipFree(S.d_h); hipFree(S.d_tkey);
    S.d_seq = S.d_qual = S.d_out = S.d_gather = nullptr;
    S.d_soff = S.d_units = S.d_slot = S.d_goff = nullptr;
    S.d_pos = S.d_cigoff = S.d_ncig = S.d_uref = S.d_res = S.d_tcnt = S.d_trep =
        S.d_uniq = S.d_ctr = nullptr;
    S.d_cig = nullptr;
    S.d_h = S.d_tkey = nullptr;
    S.dcap.clear();
}

void s2a_free(Ctx &c)
{
    if (!c.s2a) return;
    s2a_free_device(*c.s2a);
    delete c.s2a;
    c.s2a = nullptr;
}

// ---------------------------------------------------------------------------
// device
// ---------------------------------------------------------------------------
struct S2AArgs {
    const uint8_t *seq, *qual;
    const int64_t *soff;
    const int32_t *pos, *cig_off, *n_cig;
    const uint32_t *cig;
    const int64_t *units;     // per merge unit: row1, row2 (-1: single)
    const int32_t *uref;
    const int64_t *slot;      // byte offset of the unit's output slot in out
    int64_t n;
    int q_cutoff;
    double max_prop_n;
    int span_cap, ops_cap, wave_bytes;
    uint8_t *out;
    int32_t *res;             // 4 per unit
    uint64_t *h;              // 2 per unit
    int32_t *ctr;             // [0] error
};

__device__ __forceinline__ int s2a_scan(int v, int lane)
{
    for (int o = 1; o < 64; o <<= 1) {
        const int y = __shfl_up(v, o, 64);
        if (lane >= o) v += y;
    }
    return v;
}

__device__ __forceinline__ uint64_t mix64(uint64_t z)
{
    z += 0x9e3779b97f4a7c15ull;
    z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
    z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
    return z ^ (z >> 31);
}

struct Mate {
    int row, pad, rf, len;   // len = pad + reference span
    char *c, *q;             // LDS: c[t], q[t] for t < rf
};

// merged character at padded position i (sam2aln.py:186-230); seq1 = a,
// seq2 = b (the longer padded read); single = no mate
__device__ __forceinline__ char s2a_char(int i, const Mate &a, const Mate &b, bool single,
                                         int rev_start, unsigned char cut)
{
    char c2 = '-';
    unsigned char q2 = '!';
    if (i >= b.pad && i < b.len) { c2 = b.c[i - b.pad]; q2 = (unsigned char)b.q[i - b.pad]; }
    if (single) return c2;
    if (i < a.len) {
        char c1 = '-';
        unsigned char q1 = '!';
        if (i >= a.pad) { c1 = a.c[i - a.pad]; q1 = (unsigned char)a.q[i - a.pad]; }
        if (c1 == '-' && c2 == '-') return '-';
        if (c1 == c2) return (q1 > cut || q2 > cut) ? c1 : 'N';
        const int dq = (int)q2 - (int)q1;
        if ((dq < 0 ? -dq : dq) >= 5) {
            const unsigned char m2 = q2 > cut ? q2 : cut, m1 = q1 > cut ? q1 : cut;
            return q1 > m2 ? c1 : (q2 > m1 ? c2 : 'N');
        }
        return 'N';
    }
    if (c2 == '-') return i >= rev_start ? '-' : 'n';
    return q2 > cut ? c2 : 'N';
}

__global__ __launch_bounds__(256) void k_s2a_merge(S2AArgs A)
{
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const int lane = threadIdx.x & 63;
    const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int wpb = blockDim.x >> 6;
    unsigned char *wb = smem + (size_t)wv * A.wave_bytes;
    char *cq = (char *)wb;                                     // c0 q0 c1 q1, span_cap each
    int32_t *opref = (int32_t *)(wb + 4 * (size_t)A.span_cap); // ops_cap + 1 per mate
    int32_t *opread = opref + 2 * (A.ops_cap + 1);
    const unsigned char cut = (unsigned char)(A.q_cutoff + 33);

    for (int64_t u = (int64_t)blockIdx.x * wpb + wv; u < A.n; u += (int64_t)gridDim.x * wpb) {
        const int64_t rows[2] = {A.units[2 * u], A.units[2 * u + 1]};
        const int nm = rows[1] >= 0 ? 2 : 1;
        // every loop over the mates is unrolled: mt[k] with a run-time k
        // would put the array in scratch memory (80 B per lane, ~5 GB of
        // HBM writes per launch at C2)
        Mate mt[2];
#pragma unroll
        for (int k = 0; k < 2; ++k) {
            mt[k].row = -1; mt[k].pad = 0; mt[k].rf = 0; mt[k].len = 0;
            mt[k].c = cq + 2 * k * A.span_cap;
            mt[k].q = cq + (2 * k + 1) * A.span_cap;
        }
        // ---- apply_cigar (sam2aln.py:84-153): op offsets by a lane-parallel
        // scan, then the read expanded into reference coordinates ----
#pragma unroll
        for (int k = 0; k < 2; ++k) {
            if (k >= nm) break;
            const int64_t r = rows[k];
            const int nc = A.n_cig[r];
            const uint32_t *ops = A.cig + A.cig_off[r];
            int32_t *oref = opref + k * (A.ops_cap + 1), *ord = opread + k * (A.ops_cap + 1);
            int rf0 = 0, rd0 = 0;
            for (int o0 = 0; o0 < nc; o0 += 64) {
                const int o = o0 + lane;
                int dref = 0, dread = 0, isd = 0;
                if (o < nc) {
                    const uint32_t op = ops[o];
                    const int n = (int)(op >> 4), t = (int)(op & 15);
                    if (t == MH_OP_M) { dref = n; dread = n; }
                    else if (t == MH_OP_D) { dref = n; isd = 1; }
                    else dread = n;                      // I, S (checked on the host)
                }
                const int iref = s2a_scan(dref, lane), iread = s2a_scan(dread, lane);
                if (o < nc) {
                    oref[o] = rf0 + iref - dref;
                    ord[o] = isd ? -1 : rd0 + iread - dread;
                }
                rf0 += __shfl(iref, 63, 64);
                rd0 += __shfl(iread, 63, 64);
            }
            if (lane == 0) { oref[nc] = rf0; ord[nc] = rd0; }
            const int p = A.pos[r] - 1;
            mt[k].row = (int)r;
            mt[k].pad = p > 0 ? p : 0;
            mt[k].rf = rf0;
            mt[k].len = mt[k].pad + rf0;
        }
        __builtin_amdgcn_wave_barrier();
#pragma unroll
        for (int k = 0; k < 2; ++k) {
            if (k >= nm) break;
            const int64_t r = rows[k];
            const int32_t *oref = opref + k * (A.ops_cap + 1), *ord = opread + k * (A.ops_cap + 1);
            const uint8_t *s = A.seq + A.soff[r], *q = A.qual + A.soff[r];
            for (int t = lane; t < mt[k].rf; t += 64) {
                int o = 0;
                while (oref[o + 1] <= t) ++o;
                const int rd = ord[o];
                char c = '-', qq = ' ';
                if (rd >= 0) {
                    const int x = rd + (t - oref[o]);
                    c = (char)s[x];
                    qq = (char)q[x];
                }
                mt[k].c[t] = c;
                mt[k].q[t] = qq;
            }
        }
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");

        // ---- merge_pairs roles: seq1 = row1 unless it is longer ----
        const bool single = nm == 1;
        Mate a = mt[0], b = mt[0];
        if (!single) {
            if (mt[0].len > mt[1].len) { a = mt[1]; b = mt[0]; }
            else { a = mt[0]; b = mt[1]; }
        }
        const int len2 = b.len;
        // is_reverse_started: first i with seq2[i] != '-'; is_forward_started:
        // first i < len(seq1) where not both are '-'
        int rev_start = 1 << 30, fwd_start = 1 << 30;
        if (!single) {
            for (int i0 = 0; i0 < len2; i0 += 64) {
                const int i = i0 + lane;
                int rs = 1 << 30, fs = 1 << 30;
                if (i < len2) {
                    const char c2 = (i >= b.pad) ? b.c[i - b.pad] : '-';
                    if (c2 != '-') rs = i;
                    if (i < a.len) {
                        const char c1 = (i >= a.pad) ? a.c[i - a.pad] : '-';
                        if (!(c1 == '-' && c2 == '-')) fs = i;
                    }
                }
                for (int o = 32; o > 0; o >>= 1) {
                    rs = min(rs, __shfl_xor(rs, o, 64));
                    fs = min(fs, __shfl_xor(fs, o, 64));
                }
                rev_start = min(rev_start, rs);
                fwd_start = min(fwd_start, fs);
                if (rev_start < (1 << 30) && (fwd_start < (1 << 30) || i0 + 64 >= a.len)) break;
            }
        }
        const bool fwd = single || fwd_start < a.len;
        // mseq[j] = merged char at i = j + i0 (the forward read never
        // starting drops positions < len(seq1), sam2aln.py:191-195)
        const int ibase = fwd ? 0 : a.len;
        const int mlen = len2 - ibase;
        // ---- offset (leading '-'), last non-'-', count of 'N' ----
        int first = 1 << 30, last = -1, nN = 0;
        for (int j0 = 0; j0 < mlen; j0 += 64) {
            const int j = j0 + lane;
            if (j < mlen) {
                const int i = j + ibase;
                char m;
                if (!single && fwd && i < fwd_start) m = '-';
                else m = s2a_char(i, a, b, single, rev_start, cut);
                if (m != '-') { first = min(first, j); last = max(last, j); }
                nN += m == 'N';
            }
        }
        for (int o = 32; o > 0; o >>= 1) {
            first = min(first, __shfl_xor(first, o, 64));
            last = max(last, __shfl_xor(last, o, 64));
            nN += __shfl_xor(nN, o, 64);
        }
        int status = S2A_OK;
        if (last < 0) {
            status = S2A_EMPTY;   // len(mseq.strip('-')) == 0: ZeroDivisionError in the reference
        } else {
            const double prop = (double)nN / (double)(last - first + 1);
            if (prop > A.max_prop_n) status = S2A_MANYNS;
        }
        const int off = status == S2A_EMPTY ? 0 : first;
        const int blen = status == S2A_EMPTY ? 0 : mlen - first;
        uint64_t h1 = 0, h2 = 0;
        if (status == S2A_OK) {
            uint8_t *dst = A.out + A.slot[u];
            for (int j0 = 0; j0 < blen; j0 += 64) {
                const int jj = j0 + lane;
                if (jj < blen) {
                    const int i = jj + off + ibase;
                    const char m = (!single && fwd && i < fwd_start)
                                       ? '-' : s2a_char(i, a, b, single, rev_start, cut);
                    dst[jj] = (uint8_t)m;
                    const uint64_t k1 = mix64(2ull * (uint64_t)jj + 1ull) | 1ull;
                    const uint64_t k2 = mix64((uint64_t)jj ^ 0x5bd1e995ull << 32) | 1ull;
                    h1 += k1 * (uint64_t)(uint8_t)m;
                    h2 += k2 * (uint64_t)(uint8_t)m;
                }
            }
            for (int o = 32; o > 0; o >>= 1) {
                h1 += __shfl_xor(h1, o, 64);
                h2 += __shfl_xor(h2, o, 64);
            }
            const uint64_t meta = ((uint64_t)(uint32_t)A.uref[u] << 40) ^
                                  ((uint64_t)(uint32_t)off << 20) ^ (uint64_t)(uint32_t)blen;
            h1 = mix64(h1 ^ mix64(meta));
            h2 = mix64(h2 + 0x2545f4914f6cdd1dull * mix64(meta + 7));
        }
        if (lane == 0) {
            A.res[4 * u] = status;
            A.res[4 * u + 1] = off;
            A.res[4 * u + 2] = blen;
            A.res[4 * u + 3] = last < 0 ? 0 : last - first + 1;
            A.h[2 * u] = h1;
            A.h[2 * u + 1] = h2;
        }
        __builtin_amdgcn_wave_barrier();
    }
}

__device__ __forceinline__ uint64_t s2a_key(uint64_t h1) { return h1 ? h1 : 1ull; }

__global__ __launch_bounds__(256) void k_s2a_count(const int32_t *res, const uint64_t *h, int64_t n,
                                                   uint64_t *tkey, int32_t *tcnt, int32_t *trep,
                                                   uint64_t mask)
{
    for (int64_t u = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; u < n;
         u += (int64_t)gridDim.x * blockDim.x) {
        if (res[4 * u] != S2A_OK) continue;
        const uint64_t key = s2a_key(h[2 * u]);
        uint64_t s = key & mask;
        for (;;) {
            const unsigned long long old = atomicCAS((unsigned long long *)&tkey[s], 0ull,
                                                     (unsigned long long)key);
            if (old == 0ull || old == key) {
                atomicAdd(&tcnt[s], 1);
                atomicMin(&trep[s], (int32_t)u);
                break;
            }
            s = (s + 1) & mask;
        }
    }
}

__global__ __launch_bounds__(256) void k_s2a_verify(const int32_t *res, const uint64_t *h,
                                                    const int32_t *uref, const int64_t *slot,
                                                    const uint8_t *out, int64_t n,
                                                    const uint64_t *tkey, const int32_t *trep,
                                                    uint64_t mask, int32_t *ctr)
{
    const int lane = threadIdx.x & 63;
    const int wpb = blockDim.x >> 6;
    for (int64_t u = (int64_t)blockIdx.x * wpb + (threadIdx.x >> 6); u < n;
         u += (int64_t)gridDim.x * wpb) {
        if (res[4 * u] != S2A_OK) continue;
        const uint64_t key = s2a_key(h[2 * u]);
        uint64_t s = key & mask;
        while (tkey[s] != key) s = (s + 1) & mask;
        const int64_t r = trep[s];
        if (r == u) continue;
        bool bad = h[2 * r + 1] != h[2 * u + 1] || uref[r] != uref[u] ||
                   res[4 * r + 1] != res[4 * u + 1] || res[4 * r + 2] != res[4 * u + 2];
        if (!bad) {
            const uint8_t *x = out + slot[u], *y = out + slot[r];
            int diff = 0;
            for (int j = lane; j < res[4 * u + 2]; j += 64) diff |= x[j] != y[j];
            bad = __any(diff);
        }
        if (bad && lane == 0) atomicExch(&ctr[0], 1);
    }
}

__global__ __launch_bounds__(256) void k_s2a_compact(const uint64_t *tkey, const int32_t *tcnt,
                                                     const int32_t *trep, uint64_t size,
                                                     int32_t *uniq, int32_t *ctr)
{
    for (uint64_t s = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; s < size;
         s += (uint64_t)gridDim.x * blockDim.x) {
        if (!tkey[s]) continue;
        const int idx = atomicAdd(&ctr[1], 1);
        uniq[2 * idx] = trep[s];
        uniq[2 * idx + 1] = tcnt[s];
    }
}

__global__ __launch_bounds__(256) void k_s2a_gather(const int32_t *uniq, const int64_t *goff,
                                                    const int32_t *res, const int64_t *slot,
                                                    const uint8_t *out, int64_t n_uniq,
                                                    uint8_t *dst)
{
    const int lane = threadIdx.x & 63;
    const int wpb = blockDim.x >> 6;
    for (int64_t k = (int64_t)blockIdx.x * wpb + (threadIdx.x >> 6); k < n_uniq;
         k += (int64_t)gridDim.x * wpb) {
        const int64_t r = uniq[2 * k];
        const int bl = res[4 * r + 2];
        const uint8_t *src = out + slot[r];
        for (int j = lane; j < bl; j += 64) dst[goff[k] + j] = src[j];
    }
}

// ---------------------------------------------------------------------------
// host
// ---------------------------------------------------------------------------
// a device buffer of at least `bytes` behind p: kept between calls and
// reallocated only to grow (a hipFree waits for the device, and large
// allocations map pages: both once per size, not once per call)
template <class T>
static int dev_reserve(S2AState &S, T *&p, size_t bytes)
{
    size_t &cap = S.dcap[(const void *)&p];
    if (p && cap >= bytes) return 0;
    hipFree(p);
    p = nullptr;
    cap = 0;
    MH_HIP(hipMalloc(&p, bytes > 0 ? bytes : 1));
    cap = bytes;
    return 0;
}

template <class T>
static int s2a_upload(S2AState &S, T *&dst, const std::vector<T> &v, hipStream_t s)
{
    if (int st = dev_reserve(S, dst, sizeof(T) * v.size())) return st;
    if (!v.empty()) MH_HIP(hipMemcpyAsync(dst, v.data(), sizeof(T) * v.size(), hipMemcpyHostToDevice, s));
    return 0;
}

template <class Bytes>
static int s2a_upload_bytes(S2AState &S, uint8_t *&dst, const Bytes &v, hipStream_t s)
{
    if (int st = dev_reserve(S, dst, v.size())) return st;
    if (!v.empty()) MH_HIP(hipMemcpyAsync(dst, v.data(), v.size(), hipMemcpyHostToDevice, s));
    return 0;
}

// apply_cigar's checks on one row (sam2aln.py:113-151): the regex, the
// supported ops and the read length; the reference raises RuntimeError.
int s2a_run(Ctx &c, S2AState &S, double max_prop_n)
{
    hipStream_t s = c.stream;
    const int64_t nu = (int64_t)S.u1.size();
    std::vector<int64_t> mu;      // row pairs of merged units
    std::vector<int32_t> mref;
    std::vector<int64_t> slot;
    int64_t total = 0;
    int span_cap = 1, ops_cap = 1;
    for (int64_t u = 0; u < nu; ++u) {
        if (S.ucause[u] >= 0) continue;
        const int64_t r1 = S.u1[u], r2 = S.upaired[u] ? S.u2[u] : -1;
        S.merge_of_unit[u] = (int64_t)mref.size();
        mu.push_back(r1);
        mu.push_back(r2);
        mref.push_back(S.name_id[u]);
        // slot: at most max(len) - min(pad) merged characters
        int hi = 0, lo = 1 << 30;
        for (int64_t r : {r1, r2}) {
            if (r < 0) continue;
            int rf = 0;
            for (int o = 0; o < S.n_cig[r]; ++o) {
                const uint32_t op = S.cig[S.cig_off[r] + o];
                if ((op & 15) == MH_OP_M || (op & 15) == MH_OP_D) rf += (int)(op >> 4);
            }
            const int pad = S.pos[r] - 1 > 0 ? S.pos[r] - 1 : 0;
            hi = std::max(hi, pad + rf);
            lo = std::min(lo, pad);
            span_cap = std::max(span_cap, rf);
            ops_cap = std::max(ops_cap, S.n_cig[r]);
        }
        slot.push_back(total);
        total += std::max(0, hi - lo);
    }
    S.n_merge = (int64_t)mref.size();
    S.n_unique = 0;
    S.res.clear();
    S.uniq.clear();
    S.uniq_off.clear();
    S.gathered.clear();
    if (S.n_merge == 0) return 0;
    span_cap = (span_cap + 15) & ~15;
    const int wave_bytes = ((4 * span_cap + 2 * 4 * 2 * (ops_cap + 1)) + 15) & ~15;
    int wpb = 4;
    while (wpb > 1 && (size_t)wpb * wave_bytes > 160 * 1024) --wpb;
    if ((size_t)wave_bytes > 160 * 1024) {
        set_error("sam2aln: reference span %d too long for LDS", span_cap);
        return -3;
    }
    if (int st = s2a_upload_bytes(S, S.d_seq, S.seq, s)) return st;
    if (int st = s2a_upload_bytes(S, S.d_qual, S.qual, s)) return st;
    if (int st = s2a_upload(S, S.d_soff, S.soff, s)) return st;
    if (int st = s2a_upload(S, S.d_pos, S.pos, s)) return st;
    if (int st = s2a_upload(S, S.d_cigoff, S.cig_off, s)) return st;
    if (int st = s2a_upload(S, S.d_ncig, S.n_cig, s)) return st;
    if (int st = s2a_upload(S, S.d_cig, S.cig, s)) return st;
    if (int st = s2a_upload(S, S.d_units, mu, s)) return st;
    if (int st = s2a_upload(S, S.d_uref, mref, s)) return st;
    if (int st = s2a_upload(S, S.d_slot, slot, s)) return st;
    const int64_t nm = S.n_merge;
    uint64_t tsize = 1024;
    while (tsize < (uint64_t)(2 * nm)) tsize <<= 1;
    if (int st = dev_reserve(S, S.d_out, total > 0 ? (size_t)total : 1)) return st;
    if (int st = dev_reserve(S, S.d_res, sizeof(int32_t) * 4 * nm)) return st;
    if (int st = dev_reserve(S, S.d_h, sizeof(uint64_t) * 2 * nm)) return st;
    if (int st = dev_reserve(S, S.d_ctr, sizeof(int32_t) * 4)) return st;
    if (int st = dev_reserve(S, S.d_tkey, sizeof(uint64_t) * tsize)) return st;
    if (int st = dev_reserve(S, S.d_tcnt, sizeof(int32_t) * tsize)) return st;
    if (int st = dev_reserve(S, S.d_trep, sizeof(int32_t) * tsize)) return st;
    if (int st = dev_reserve(S, S.d_uniq, sizeof(int32_t) * 2 * nm)) return st;
    MH_HIP(hipMemsetAsync(S.d_ctr, 0, sizeof(int32_t) * 4, s));
    MH_HIP(hipMemsetAsync(S.d_tkey, 0, sizeof(uint64_t) * tsize, s));
    MH_HIP(hipMemsetAsync(S.d_tcnt, 0, sizeof(int32_t) * tsize, s));
    MH_HIP(hipMemsetAsync(S.d_trep, 0x7f, sizeof(int32_t) * tsize, s));

    S2AArgs a{S.d_seq, S.d_qual, S.d_soff, S.d_pos, S.d_cigoff, S.d_ncig, S.d_cig,
              S.d_units, S.d_uref, S.d_slot, nm, S.q_cutoff, max_prop_n, span_cap, ops_cap,
              wave_bytes, S.d_out, S.d_res, S.d_h, S.d_ctr};
    int64_t blocks = (nm + wpb - 1) / wpb;
    if (blocks > 256 * 64) blocks = 256 * 64;
    MH_HIP(hipFuncSetAttribute((const void *)k_s2a_merge,
                               hipFuncAttributeMaxDynamicSharedMemorySize, wpb * wave_bytes));
    const int p0 = prof_begin(c, "k_s2a_merge");
    hipLaunchKernelGGL(k_s2a_merge, dim3((unsigned)blocks), dim3(64 * wpb), wpb * wave_bytes, s, a);
    prof_end(c, p0);
    MH_HIP(hipGetLastError());
    int64_t tb = (nm + 255) / 256;
    if (tb > 65536) tb = 65536;
    const int p1 = prof_begin(c, "k_s2a_group");
    hipLaunchKernelGGL(k_s2a_count, dim3((unsigned)tb), dim3(256), 0, s, S.d_res, S.d_h, nm,
                       S.d_tkey, S.d_tcnt, S.d_trep, tsize - 1);
    int64_t vb = (nm + 3) / 4;
    if (vb > 256 * 64) vb = 256 * 64;
    hipLaunchKernelGGL(k_s2a_verify, dim3((unsigned)vb), dim3(256), 0, s, S.d_res, S.d_h, S.d_uref,
                       S.d_slot, S.d_out, nm, S.d_tkey, S.d_trep, tsize - 1, S.d_ctr);
    int64_t cb = (int64_t)((tsize + 255) / 256);
    if (cb > 65536) cb = 65536;
    hipLaunchKernelGGL(k_s2a_compact, dim3((unsigned)cb), dim3(256), 0, s, S.d_tkey, S.d_tcnt,
                       S.d_trep, tsize, S.d_uniq, S.d_ctr);
    prof_end(c, p1);
    MH_HIP(hipGetLastError());
    int32_t ctr[4];
    MH_HIP(hipMemcpyAsync(ctr, S.d_ctr, sizeof(ctr), hipMemcpyDeviceToHost, s));
    MH_HIP(hipStreamSynchronize(s));
    if (ctr[0]) {
        set_error("sam2aln: merged-sequence hash collision (distinct sequences share a key)");
        return -4;
    }
    S.n_unique = ctr[1];
    S.res.resize(4 * nm);
    S.uniq.resize(2 * (size_t)S.n_unique);
    MH_HIP(hipMemcpyAsync(S.res.data(), S.d_res, sizeof(int32_t) * 4 * nm, hipMemcpyDeviceToHost, s));
    if (S.n_unique)
        MH_HIP(hipMemcpyAsync(S.uniq.data(), S.d_uniq, sizeof(int32_t) * 2 * S.n_unique,
                              hipMemcpyDeviceToHost, s));
    MH_HIP(hipStreamSynchronize(s));
    for (int64_t u = 0; u < nm; ++u)
        if (S.res[4 * u] == S2A_EMPTY) {
            set_error("sam2aln: merged sequence of unit %lld is all gaps (float division by zero)",
                      (long long)u);
            return -3;
        }
    // gather the distinct bodies
    S.uniq_off.resize(S.n_unique + 1);
    int64_t g = 0;
    for (int64_t k = 0; k < S.n_unique; ++k) {
        S.uniq_off[k] = g;
        g += S.res[4 * (int64_t)S.uniq[2 * k] + 2];
    }
    S.uniq_off[S.n_unique] = g;
    S.gathered.resize((size_t)g);
    if (S.n_unique && g) {
        if (int st = s2a_upload(S, S.d_goff, S.uniq_off, s)) return st;
        if (int st = dev_reserve(S, S.d_gather, (size_t)g)) return st;
        int64_t gb = (S.n_unique + 3) / 4;
        if (gb > 256 * 64) gb = 256 * 64;
        hipLaunchKernelGGL(k_s2a_gather, dim3((unsigned)gb), dim3(256), 0, s, S.d_uniq, S.d_goff,
                           S.d_res, S.d_slot, S.d_out, S.n_unique, S.d_gather);
        MH_HIP(hipGetLastError());
        MH_HIP(hipMemcpyAsync(&S.gathered[0], S.d_gather, (size_t)g, hipMemcpyDeviceToHost, s));
        MH_HIP(hipStreamSynchronize(s));
    }
    prof_flush(c);
    return 0;
}

}  // namespace mh

using namespace mh;

extern "C" int mh_sam2aln_csv(mh_ctx *ctx, const char *text, int64_t len, int q_cutoff,
                              double max_prop_n, int64_t *n_units)
{
    if (!ctx || (!text && len) || len < 0 || q_cutoff < 0 || q_cutoff > 93) return -3;
    Ctx &c = *ctx_of(ctx);
    MH_HIP(hipSetDevice(c.device));
    if (!c.s2a) c.s2a = new S2AState();
    S2AState &S = *c.s2a;
    S.q_cutoff = q_cutoff;
    S.n_merge = S.n_unique = 0;
    S.res.clear();
    for (auto &o : S.out_cache) std::vector<std::string>().swap(o);
    S.out_valid = 0;
    auto t0 = std::chrono::steady_clock::now();
    int pst = 0;
    try {
        pst = s2a_parse(S, text ? text : "", len);
    } catch (const std::exception &e) {
        set_error("remap csv: out of memory (%s)", e.what());
        pst = -2;
    }
    if (pst) {
        S.u1.clear();
        return pst;
    }
    auto t1 = std::chrono::steady_clock::now();
    if (int st = s2a_run(c, S, max_prop_n)) {
        S.u1.clear();
        return st;
    }
    auto t2 = std::chrono::steady_clock::now();
    S.t_parse = std::chrono::duration<double, std::milli>(t1 - t0).count();
    S.t_device = std::chrono::duration<double, std::milli>(t2 - t1).count();
    if (n_units) *n_units = (int64_t)S.u1.size();
    return 0;
}

extern "C" int mh_sam2aln_file(mh_ctx *ctx, int fd, int q_cutoff, double max_prop_n, int64_t *n_units)
{
    if (!ctx || fd < 0) return -3;
    const char *text = nullptr;
    size_t len = 0;
    if (int st = map_text_file(fd, &text, &len)) return st;
    const int rc = mh_sam2aln_csv(ctx, text, (int64_t)len, q_cutoff, max_prop_n, n_units);
    unmap_text_file(text, len);
    return rc;
}

extern "C" int mh_sam2aln_write(mh_ctx *ctx, int which, int fd, int64_t offset, int64_t *written)
{
    if (!ctx || which < 0 || which > 2 || fd < 0 || offset < 0) return -3;
    Ctx &c = *ctx_of(ctx);
    if (!c.s2a) { set_error("mh_sam2aln_write: no sam2aln results"); return -3; }
    if (!(c.s2a->out_valid & (1 << which))) {
        // not formatted yet (no size query before): formatted and written
        // together, the writes overlapping the formatting
        S2AState &S = *c.s2a;
        auto t0 = std::chrono::steady_clock::now();
        int err = 0;
        try {
            err = s2a_format_write(S, which, fd, offset, written);
        } catch (const std::exception &e) {
            set_error("mh_sam2aln_write: out of memory (%s)", e.what());
            return -2;
        }
        S.t_format[which] = std::chrono::duration<double, std::milli>(
                                std::chrono::steady_clock::now() - t0).count();
        if (err) { set_error("mh_sam2aln_write: write failed (%s)", strerror(err)); return -4; }
        return 0;
    }
    size_t used = 0;
    if (int st = mh_sam2aln_output(ctx, which, nullptr, 0, &used)) return st;
    S2AState &S = *ctx_of(ctx)->s2a;
    int64_t pos = offset;
    for (const std::string &piece : S.out_cache[which]) {
        const char *p = piece.data();
        size_t left = piece.size();
        while (left > 0) {
            const ssize_t w = pwrite(fd, p, left, (off_t)pos);
            if (w <= 0) { set_error("mh_sam2aln_write: write failed (%s)", strerror(errno ? errno : EIO)); return -4; }
            p += w; left -= (size_t)w; pos += w;
        }
    }
    if (written) *written = pos - offset;
    std::vector<std::string>().swap(S.out_cache[which]);
    S.out_valid &= ~(1 << which);
    return 0;
}

extern "C" int mh_sam2aln_output(mh_ctx *ctx, int which, char *buf, size_t cap, size_t *used)
{
    if (!ctx || which < 0 || which > 2 || !used) return -3;
    Ctx &c = *ctx_of(ctx);
    if (!c.s2a) { set_error("mh_sam2aln_output: no sam2aln results"); return -3; }
    S2AState &S = *c.s2a;
    std::vector<std::string> &out = S.out_cache[which];
    if (!(S.out_valid & (1 << which))) {
        auto t0 = std::chrono::steady_clock::now();
        try {
            s2a_format(S, which, out);
        } catch (const std::exception &e) {
            std::vector<std::string>().swap(out);
            set_error("mh_sam2aln_output: out of memory (%s)", e.what());
            return -2;
        }
        S.t_format[which] = std::chrono::duration<double, std::milli>(
                                std::chrono::steady_clock::now() - t0).count();
        S.out_valid |= 1 << which;
    }
    size_t total = 0;
    for (const std::string &p : out) total += p.size();
    *used = total;
    if (!buf) return 0;
    if (cap < total) { set_error("mh_sam2aln_output: buffer too small"); return -2; }
    for (const std::string &p : out) { memcpy(buf, p.data(), p.size()); buf += p.size(); }
    std::vector<std::string>().swap(out);   // handed over: free the cached text
    S.out_valid &= ~(1 << which);
    return 0;
}

extern "C" int mh_sam2aln_timing(mh_ctx *ctx, double *ms5)
{
    if (!ctx || !ms5) return -3;
    Ctx &c = *ctx_of(ctx);
    if (!c.s2a) { set_error("mh_sam2aln_timing: no sam2aln results"); return -3; }
    const S2AState &S = *c.s2a;
    ms5[0] = S.t_parse;
    ms5[1] = S.t_device;
    for (int k = 0; k < 3; ++k) ms5[2 + k] = S.t_format[k];
    return 0;
}

extern "C" int mh_sam2aln_stats(mh_ctx *ctx, int64_t *out4)
{
    if (!ctx || !out4) return -3;
    Ctx &c = *ctx_of(ctx);
    if (!c.s2a) { set_error("mh_sam2aln_stats: no sam2aln results"); return -3; }
    const S2AState &S = *c.s2a;
    int64_t nfail = 0;
    for (int64_t u = 0; u < (int64_t)S.u1.size(); ++u)
        if (S.ucause[u] >= 0 || S.res[4 * S.merge_of_unit[u]] != S2A_OK) ++nfail;
    out4[0] = (int64_t)S.u1.size();
    out4[1] = S.n_merge;
    out4[2] = S.n_unique;
    out4[3] = nfail;
    return 0;
}
