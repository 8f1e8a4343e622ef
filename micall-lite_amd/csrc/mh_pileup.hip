// mh_pileup.hip -- consensus pileup on gfx950: the counting half of
// remap.sam_to_conseqs (micall/core/remap.py:141-306), one wave64 per read
// pair (matchmaker unit):
//   merge_reads    remap.py:86-126    which mates count, the rname check
//   apply_cigar    sam2aln.py:84-153  each mate in reference coordinates
//   merge_pairs    sam2aln.py:156-237 per-position merge, lane-parallel
//   merge_inserts  sam2aln.py:240-273 (lane 0; rare)
//   update_counts  remap.py:271-306   int32 atomics into dense A/C/G/T
//                                     counters, 'N'/'-' flags, sparse events
// The refmap of the reference is order-independent except for its key
// order, which is recovered from first_unit (atomicMin), so results are
// deterministic.  Bit-for-bit specification: oracle/og_pileup.c.
#include <cstring>

#include "mh_internal.h"

namespace mh {

constexpr int PU_INSBUF = 2048;   // merged insertion bytes per unit
constexpr int PU_MAXINS = 2 * MH_MAXOPS;
constexpr int PU_LDS = 160 * 1024 - 64;   // dynamic LDS (the static s_next beside it)
constexpr int PU_XCH = 5;        // 64-position chunks per mate expanded with all loads in flight

struct RowV {
    int present, flag, ref, pos, n_cigar, rev, m;
    const uint32_t *cig;
    int64_t roff;
    uint32_t op0;   // this lane's op of the first 64 (fetch_ops)
};

// This lane's CIGAR op of the first 64, loaded ahead of apply_cigar.
__device__ __forceinline__ void fetch_ops(RowV &v, int lane)
{
    v.op0 = 0;
    if (v.present && lane < v.n_cigar) v.op0 = v.cig[lane];
}

struct PileArgs {
    // source 0: mapped records
    const Rec *rec;
    const uint32_t *pool;
    DevReads R;           // reads of source 0, or rows' reads for source 1
    int paired;
    // source 1: rows
    const int32_t *flag, *ref, *pos, *cig_off, *n_cigar;
    const uint32_t *cigar;
    const int64_t *units;
    int64_t n_units;
    // outputs
    int n_refs;
    int32_t cap;
    int32_t *dense;
    uint8_t *nflag, *dflag;
    unsigned long long *read_counts;
    long long *first_unit;
    int32_t *max_pos;
    int32_t *ev;
    char *ev_pool;
    long long ev_cap, pool_cap;
    unsigned long long *ev_ctr;  // [0] events, [1] pool bytes, [2] overflow, [3] error
    int q_cutoff;
    // LDS layout: every reference's scalars (RefLds), the counter windows of
    // the references that fit (win_map: per reference the window's first
    // word or -1, and its positions wl: a plane of wl A|C<<16 words, then
    // a plane of wl G|T<<16 words), then one staging area per wave
    const int32_t *win_map;
    int win_words;
    int span_cap;                // reference span per mate staged in LDS
    int unit_bytes;              // staging bytes per wave
    char *ins_scratch;           // PU_INS_BYTES per wave of the grid
};

template <int SRC>
__device__ __forceinline__ void load_row(const PileArgs &A, int64_t row, RowV &v)
{
    v.present = 0;
    if (row < 0) return;
    if (SRC == 0) {
        // no branch on the loaded fields, so a prefetch of the next unit's
        // rows does not wait for them here
        const Rec &r = A.rec[row];
        const int sref = r.sam_ref, flag = r.flag;
        v.present = sref >= 0;          // RNAME '*' is not in @SQ (matchmaker)
        v.flag = flag;
        v.ref = sref;
        v.pos = r.sam_pos;
        v.n_cigar = (flag & 4) ? 0 : r.n_cigar;
        v.cig = A.pool + r.cig_off;
        v.rev = (flag & 4) ? 0 : r.rev;
    } else {
        v.present = 1;
        v.flag = A.flag[row];
        v.ref = A.ref[row];
        v.pos = A.pos[row];
        v.n_cigar = A.n_cigar[row];
        v.cig = A.cigar + A.cig_off[row];
        v.rev = 0;
    }
    v.m = A.R.len[row];
    v.roff = A.R.off[row];
}

// The next unit's two rows, prefetched lane-distributed in one VGPR (lanes
// 0-9: row 1, 32-41: row 2; one field per lane) instead of two RowV in
// SGPRs that stay live over the whole unit: k_pileup ran out of SGPRs and
// spilled them to VGPR lanes, paying v_readlane reloads inside its loops.
// Fields: 0 ref, 1 flag, 2 pos, 3 n_cigar, 4 cig_off, 5 rev, 6 m, 7-8 roff,
// 9 row valid.
template <int SRC>
__device__ __forceinline__ int load_rows_packed(const PileArgs &A, int64_t uu, int lane)
{
    const int h = lane >> 5, f = lane & 31;
    if (f > 9) return 0;
    int64_t row;
    if (SRC == 0) row = A.paired ? 2 * uu + h : (h ? -1 : uu);
    else row = A.units[2 * uu + h];
    if (row < 0) return 0;
    if (f == 9) return 1;
    if (f == 6) return A.R.len[row];
    if (f >= 7) return ((const int32_t *)A.R.off)[2 * row + (f - 7)];
    if (SRC == 0) {
        const int32_t *r = (const int32_t *)&A.rec[row];
        const int idx = f == 0 ? 10 : f == 1 ? 5 : f == 2 ? 11 : f == 3 ? 19 : f == 4 ? 20 : 2;
        return r[idx];
    }
    switch (f) {
    case 0: return A.ref[row];
    case 1: return A.flag[row];
    case 2: return A.pos[row];
    case 3: return A.n_cigar[row];
    case 4: return A.cig_off[row];
    default: return 0;
    }
}

template <int SRC>
__device__ __forceinline__ RowV unpack_row(const PileArgs &A, int pk, int h)
{
    auto fld = [&](int f) { return __builtin_amdgcn_readlane(pk, 32 * h + f); };
    RowV v;
    const int valid = fld(9), ref = fld(0), flag = fld(1);
    v.flag = flag;
    v.ref = ref;
    v.pos = fld(2);
    if (SRC == 0) {
        v.present = valid && ref >= 0;   // RNAME '*' is not in @SQ (matchmaker)
        v.n_cigar = (flag & 4) ? 0 : fld(3);
        v.rev = (flag & 4) ? 0 : fld(5);
        v.cig = A.pool + (uint32_t)fld(4);
    } else {
        v.present = valid;
        v.n_cigar = fld(3);
        v.rev = 0;
        v.cig = A.cigar + (uint32_t)fld(4);
    }
    v.m = fld(6);
    v.roff = (int64_t)(((uint64_t)(uint32_t)fld(8) << 32) | (uint32_t)fld(7));
    v.op0 = 0;
    return v;
}

// base code 0..4 -> 'A' 'C' 'G' 'T' 'N' from a register constant (a string
// literal indexed per lane is a global load)
__device__ __forceinline__ char base_char(uint32_t code)
{
    return (char)((0x4E54474341ull >> (8 * code)) & 0xffu);
}

__device__ __forceinline__ void sam_base_at(const DevReads &R, int rev, int m, int64_t roff, int x,
                                            char &c, char &q)
{
    const int b = rev ? m - 1 - x : x;
    const int64_t g = roff + b;
    uint32_t code = ((R.nmask[g >> 5] >> (g & 31)) & 1) ? 4 : (R.seq2[g >> 4] >> (2 * (g & 15))) & 3;
    if (rev && code < 4) code = 3 - code;
    c = base_char(code);
    q = (char)R.qual[g];
}

__device__ __forceinline__ void sam_base(const DevReads &R, const RowV &v, int x, char &c, char &q)
{
    const int b = v.rev ? v.m - 1 - x : x;
    const int64_t g = v.roff + b;
    uint32_t code = ((R.nmask[g >> 5] >> (g & 31)) & 1) ? 4 : (R.seq2[g >> 4] >> (2 * (g & 15))) & 3;
    if (v.rev && code < 4) code = 3 - code;
    c = base_char(code);
    q = (char)R.qual[g];
}

// One wave's LDS staging area (span_cap = SPAN):
//   c[2][SPAN], q[2][SPAN]                 both mates in reference coordinates
//   opref[2][MH_MAXOPS+1], opread[2][...]  reference / read offset of every op
//   n_ins
struct UnitView {
    char *cq;        // c of mate k at cq + 2k*span, q at cq + (2k+1)*span
    int32_t *ops;    // opref of mate k at ops + 2k*(MH_MAXOPS+1), opread after it
    int span;
    int32_t *n_ins;
    __device__ char *c(int k) const { return cq + 2 * k * span; }
    __device__ char *q(int k) const { return cq + (2 * k + 1) * span; }
    __device__ int32_t *opref(int k) const { return ops + 2 * k * (MH_MAXOPS + 1); }
    __device__ int32_t *opread(int k) const { return ops + (2 * k + 1) * (MH_MAXOPS + 1); }
};

__host__ __device__ inline int unit_bytes_for(int span)
{
    return 4 * span + 4 * 4 * (MH_MAXOPS + 1) + 16;
}

__device__ inline UnitView unit_view(unsigned char *base, int span)
{
    UnitView v;
    v.cq = (char *)base;
    v.span = span;
    v.ops = (int32_t *)(base + 4 * span);
    v.n_ins = v.ops + 4 * (MH_MAXOPS + 1);
    return v;
}

// Merged insertions of the unit a wave is on (rare: units with I ops), in a
// per-wave slice of global scratch: key, offset and length of each entry and
// the merged bytes.
constexpr int PU_INS_BYTES = 3 * 4 * PU_MAXINS + PU_INSBUF;
struct InsView {
    int32_t *key, *off, *len;
    char *buf;
};

__device__ inline InsView ins_view(char *base)
{
    InsView v;
    v.key = (int32_t *)base;
    v.off = v.key + PU_MAXINS;
    v.len = v.key + 2 * PU_MAXINS;
    v.buf = (char *)(v.key + 3 * PU_MAXINS);
    return v;
}

struct RefLds {
    unsigned int read_count;
    int max_pos;
    long long first_unit;
};

// Wave-wide scans and reductions on DPP (row shifts, then the two row
// broadcasts): register-to-register, where __shfl goes through the LDS
// crossbar (ds_bpermute) and pays its latency on every step.  A lane with
// no source, or in a row the step does not write, takes the identity.
template <int CTRL, int ROWMASK>
__device__ __forceinline__ int dpp_id(int identity, int v)
{
    return __builtin_amdgcn_update_dpp(identity, v, CTRL, ROWMASK, 0xF, false);
}

template <class Op>
__device__ __forceinline__ int wave_scan_dpp(int v, int identity, Op op)
{
    v = op(v, dpp_id<0x111, 0xF>(identity, v));   // row_shr:1
    v = op(v, dpp_id<0x112, 0xF>(identity, v));   // row_shr:2
    v = op(v, dpp_id<0x114, 0xF>(identity, v));   // row_shr:4
    v = op(v, dpp_id<0x118, 0xF>(identity, v));   // row_shr:8
    v = op(v, dpp_id<0x142, 0xA>(identity, v));   // row_bcast:15 into rows 1, 3
    v = op(v, dpp_id<0x143, 0xC>(identity, v));   // row_bcast:31 into rows 2, 3
    return v;
}

__device__ __forceinline__ int wave_incl_scan(int v, int /*lane*/)
{
    return wave_scan_dpp(v, 0, [](int x, int y) { return x + y; });
}

__device__ __forceinline__ int wave_min_all(int v)
{
    return __builtin_amdgcn_readlane(wave_scan_dpp(v, INT32_MAX, [](int x, int y) { return x < y ? x : y; }), 63);
}

__device__ __forceinline__ int wave_max_all(int v)
{
    return __builtin_amdgcn_readlane(wave_scan_dpp(v, INT32_MIN, [](int x, int y) { return x > y ? x : y; }), 63);
}

// 6 waves per SIMD: at most 80 VGPRs, so 24 waves stay resident per CU
// (pile_geometry); k_pileup<0> keeps 2 VGPRs in scratch (12 B per lane).
// SKIP: some references are not counted (mh_pileup_only); a separate
// instance, so the full pileup pays no per-unit LDS read or SGPR for it
template <int SRC, bool SKIP>
__global__ __launch_bounds__(1024, 6) void k_pileup(PileArgs A)
{
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const int lane = threadIdx.x & 63;
    const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int wpb = blockDim.x >> 6;
    const int NR = A.n_refs;
    RefLds *rl = (RefLds *)smem;                                   // [NR]
    int32_t *wmap = (int32_t *)(smem + sizeof(RefLds) * (size_t)NR);   // [NR][2]
    unsigned int *win = (unsigned int *)(wmap + 2 * NR);           // [win_words]
    UnitView L = unit_view((unsigned char *)(win + A.win_words) + (size_t)wv * A.unit_bytes,
                           A.span_cap);
    const InsView I = ins_view(A.ins_scratch + ((size_t)blockIdx.x * wpb + wv) * PU_INS_BYTES);
    const unsigned char cut = (unsigned char)(A.q_cutoff + 33);
    __shared__ int s_next;   // the block's next unit slot (see unit_of)
    if (threadIdx.x == 0) s_next = wpb;
    for (int x = threadIdx.x; x < A.win_words; x += blockDim.x) win[x] = 0;
    for (int x = threadIdx.x; x < NR; x += blockDim.x) {
        rl[x].read_count = 0;
        rl[x].max_pos = 0;
        rl[x].first_unit = INT64_MAX;
        wmap[2 * x] = A.win_map[2 * x];
        wmap[2 * x + 1] = A.win_map[2 * x + 1];
    }
    __syncthreads();

    // The block's units are the grid-strided set {block * wpb + x + k * wpb *
    // blocks}; its waves take them in order from an LDS counter (slot c ->
    // unit_of(c)), so a wave that drew cheap units takes more and the block
    // ends when its units do, not when its slowest wave's fixed share does.
    // The next unit's rows are loaded while this one is processed.
    const int64_t ustride = (int64_t)gridDim.x * wpb;
    auto unit_of = [&](int64_t c) { return (int64_t)blockIdx.x * wpb + c % wpb + (c / wpb) * ustride; };
    int64_t u = unit_of(wv), un = A.n_units;
    int npk = 0;                  // the next unit's rows, lane-distributed
    uint32_t nop1 = 0, nop2 = 0;  // and this lane's CIGAR op of their first 64
    bool ops_ready = false;       // the CIGAR ops of the next unit were fetched
    if (u < A.n_units) npk = load_rows_packed<SRC>(A, u, lane);
    for (; u < A.n_units; u = un) {
        RowV r1 = unpack_row<SRC>(A, npk, 0), r2 = unpack_row<SRC>(A, npk, 1);
        if (ops_ready) {
            r1.op0 = nop1;
            r2.op0 = nop2;
        } else {
            fetch_ops(r1, lane);
            fetch_ops(r2, lane);
        }
        ops_ready = false;
        {
            int cn = 0;
            if (lane == 0) cn = atomicAdd(&s_next, 1);
            un = unit_of(__builtin_amdgcn_readfirstlane(cn));
        }
        const bool more = un < A.n_units;
        if (more) npk = load_rows_packed<SRC>(A, un, lane);
        if (SRC == 0 && !r1.present && r2.present) { r1 = r2; r2.present = 0; }  // unpaired view
        if (!r1.present) continue;
        if (r2.present && r1.ref != r2.ref) continue;           // remap.py:96-98
        // the mapped mates (merge_reads filters unmapped ones): m0, m1
        const bool u1 = !(r1.flag & 4), u2 = r2.present && !(r2.flag & 4);
        const int nm = (int)u1 + (int)u2;
        if (!u1) r1 = r2;   // mate 0 is the first mapped one (no copies: SGPRs are scarce)
        const RowV &m0 = r1;
        auto mate = [&](int k) -> const RowV & { return k ? r2 : r1; };
        if (nm == 0) continue;                                 // remap.py:111-112
        const int ref = r1.ref;
        if (ref < 0 || ref >= A.n_refs) {
            if (lane == 0) atomicExch(&A.ev_ctr[3], 1ull);
            continue;
        }
        // a reference this pileup does not count (mh_pileup_only)
        if (SKIP && __builtin_amdgcn_readfirstlane(wmap[2 * ref]) == -2) continue;

        // ---- apply_cigar: op offsets by a lane-parallel prefix scan, then
        // expand each mate into reference coordinates lane-parallel ----
        int padA = 0, padB = 0, lenA = 0, lenB = 0, bad = 0, n_iops = 0;
        // per mate: the read offset of its only reference-consuming op when
        // that op is an M (S/M/S reads), else -1; such a mate expands as
        // read offset + t with no op lookup
        int oneA = -1, oneB = -1;
        // lane o: reference end and read offset (-1: deletion) of op o
        // of each mate, for the first 64 ops (the expansion's op lookup)
        int oendA = 0, ordA = 0, oendB = 0, ordB = 0;
        auto pad = [&](int k) { return k ? padB : padA; };
        auto len = [&](int k) { return k ? lenB : lenA; };
        auto one = [&](int k) { return k ? oneB : oneA; };
        #pragma unroll
        for (int k = 0; k < 2; ++k) {
            if (k >= nm) break;
            const RowV mk = mate(k);
            const int nc = mk.n_cigar;
            if (nc > MH_MAXOPS) { bad = 1; break; }
            int rf0 = 0, rd0 = 0, n_refop = 0, first_rd = -1;
            for (int o0 = 0; o0 < nc; o0 += 64) {
                const int o = o0 + lane;
                int dref = 0, dread = 0, isd = 0, isi = 0, badop = 0;
                if (o < nc) {
                    const uint32_t op = o0 == 0 ? mk.op0 : mk.cig[o];
                    const int n = (int)(op >> 4), t = (int)(op & 15);
                    if (t == MH_OP_M) { dref = n; dread = n; }
                    else if (t == MH_OP_D) { dref = n; isd = 1; }
                    else if (t == MH_OP_I) { dread = n; isi = 1; }
                    else if (t == MH_OP_S) dread = n;
                    else badop = 1;
                }
                const int iref = wave_incl_scan(dref, lane), iread = wave_incl_scan(dread, lane);
                if (o < nc) {
                    L.opref(k)[o] = rf0 + iref - dref;
                    L.opread(k)[o] = isd ? -1 : rd0 + iread - dread;   // -1: deletion
                }
                if (o0 == 0) {
                    if (k) { oendB = iref; ordB = isd ? -1 : iread - dread; }
                    else { oendA = iref; ordA = isd ? -1 : iread - dread; }
                }
                bad |= __any(badop);
                n_iops += __popcll(__ballot(isi));
                const uint64_t rops = __builtin_amdgcn_ballot_w64(dref > 0);
                if (rops && n_refop == 0)
                    first_rd = __builtin_amdgcn_readlane(isd ? -1 : rd0 + iread - dread,
                                                         (int)__builtin_ctzll(rops));
                n_refop += __popcll(rops);
                rf0 += __builtin_amdgcn_readlane(iref, 63);
                rd0 += __builtin_amdgcn_readlane(iread, 63);
            }
            if (lane == 0) { L.opref(k)[nc] = rf0; L.opread(k)[nc] = rd0; }
            if (rd0 != mk.m || rf0 > A.span_cap || mk.pos < 1) bad = 1;
            const int onek = n_refop == 1 ? first_rd : -1;
            if (k) { padB = mk.pos - 1; lenB = padB + rf0; oneB = onek; }
            else { padA = mk.pos - 1; lenA = padA + rf0; oneA = onek; }
        }
        if (bad) {
            if (lane == 0) atomicExch(&A.ev_ctr[3], 1ull);
            continue;
        }
        __builtin_amdgcn_wave_barrier();
        const int spanA = lenA - padA, spanB = nm > 1 ? lenB - padB : 0;
        if (spanA <= PU_XCH * 64 && spanB <= PU_XCH * 64) {
            // Both mates at once: every chunk's op lookup (LDS) first, then
            // all base loads in flight together, then the LDS writes; one
            // dependent global round trip per unit instead of one per chunk.
            int bx[2][PU_XCH];   // strand-adjusted read index; -1 deletion, -2 none
#pragma unroll
            for (int k = 0; k < 2; ++k) {
                const RowV mk = mate(k);
                const int span = k ? spanB : spanA;
                // the M/D op covering reference offset t (I/S ops span nothing):
                // the last op whose reference start is <= t, found by a
                // wave-uniform pass over the op ends (lane values, no LDS
                // round trips) when the mate has <= 64 ops
                // dl[ch]: read offset minus reference offset of the op, or
                // DEL_MARK for a deletion
                constexpr int DEL_MARK = -(1 << 30);
                int dl[PU_XCH];
                const int nc = mk.n_cigar;
                if (one(k) < 0 && nc <= 64) {
                    const int oend = k ? oendB : oendA, ord = k ? ordB : ordA;
                    const int rd0 = __builtin_amdgcn_readlane(ord, 0);
#pragma unroll
                    for (int ch = 0; ch < PU_XCH; ++ch) dl[ch] = rd0 >= 0 ? rd0 : DEL_MARK;
                    for (int o = 0; o + 1 < nc; ++o) {
                        const int e = __builtin_amdgcn_readlane(oend, o);
                        const int rdn = __builtin_amdgcn_readlane(ord, o + 1);
                        const int dn = rdn >= 0 ? rdn - e : DEL_MARK;
#pragma unroll
                        for (int ch = 0; ch < PU_XCH; ++ch) dl[ch] = ch * 64 + lane >= e ? dn : dl[ch];
                    }
                }
#pragma unroll
                for (int ch = 0; ch < PU_XCH; ++ch) {
                    const int t = ch * 64 + lane;
                    int x = -2;
                    if (k < nm && t < span) {
                        int rd, r0 = 0;
                        if (one(k) >= 0) {
                            rd = one(k);   // the one M op starts at reference offset 0
                        } else if (nc <= 64) {
                            rd = dl[ch] == DEL_MARK ? -1 : t + dl[ch];
                            r0 = t;
                        } else {
                            int o = 0;
                            while (L.opref(k)[o + 1] <= t) ++o;
                            rd = L.opread(k)[o];
                            r0 = L.opref(k)[o];
                        }
                        x = -1;
                        if (rd >= 0) {
                            x = rd + (t - r0);
                            if (mk.rev) x = mk.m - 1 - x;
                        }
                    }
                    bx[k][ch] = x;
                }
            }
            uint32_t nw[2][PU_XCH], sw[2][PU_XCH], qw[2][PU_XCH];
#pragma unroll
            for (int k = 0; k < 2; ++k) {
                const int64_t roff = mate(k).roff;
#pragma unroll
                for (int ch = 0; ch < PU_XCH; ++ch) {
                    nw[k][ch] = 0; sw[k][ch] = 0; qw[k][ch] = 0;
                    if (bx[k][ch] >= 0) {
                        const int64_t g = roff + bx[k][ch];
                        nw[k][ch] = A.R.nmask[g >> 5];
                        sw[k][ch] = A.R.seq2[g >> 4];
                        qw[k][ch] = A.R.qual[g];
                    }
                }
            }
#pragma unroll
            for (int k = 0; k < 2; ++k) {
                const RowV mk = mate(k);
#pragma unroll
                for (int ch = 0; ch < PU_XCH; ++ch) {
                    const int t = ch * 64 + lane;
                    const int x = bx[k][ch];
                    if (x == -2) continue;
                    char c = '-', q = ' ';
                    if (x >= 0) {
                        const int64_t g = mk.roff + x;
                        uint32_t code = ((nw[k][ch] >> (g & 31)) & 1) ? 4u : (sw[k][ch] >> (2 * (g & 15))) & 3u;
                        if (mk.rev && code < 4) code = 3 - code;
                        c = base_char(code);
                        q = (char)qw[k][ch];
                    }
                    L.c(k)[t] = c;
                    L.q(k)[t] = q;
                }
            }
        } else {
#pragma unroll
            for (int k = 0; k < 2; ++k) {
                if (k >= nm) break;
                const int span = len(k) - pad(k);
                const RowV mk = mate(k);
                for (int t = lane; t < span; t += 64) {
                    // the M/D op covering reference offset t (I/S ops span nothing)
                    int o = 0;
                    while (L.opref(k)[o + 1] <= t) ++o;
                    const int rd = L.opread(k)[o];
                    char c = '-', q = ' ';
                    if (rd >= 0) sam_base(A.R, mk, rd + (t - L.opref(k)[o]), c, q);
                    L.c(k)[t] = c;
                    L.q(k)[t] = q;
                }
            }
        }
        if (more) {   // the next unit's rows have landed: its CIGAR ops land during the merge
            RowV q1 = unpack_row<SRC>(A, npk, 0), q2 = unpack_row<SRC>(A, npk, 1);
            fetch_ops(q1, lane);
            fetch_ops(q2, lane);
            nop1 = q1.op0;
            nop2 = q2.op0;
            ops_ready = true;
        }
        // ---- merge_inserts (only units with I ops): keys left + pad,
        // sam2aln.py:133-135, :240-273.  A wave-uniform walk over the I ops;
        // the inserted bases of each are read, tested and merged
        // lane-parallel (64 per round). ----
        {
            int n = 0, used = 0;
            int keyv = -1;   // lane z < 64: key of entry z
#pragma unroll
            for (int pass = 0; pass < 2; ++pass) {
                if (pass >= nm || !n_iops) break;
                const RowV v = mate(pass);
                for (int o = 0; o < v.n_cigar; ++o) {
                    const uint32_t op = o < 64 ? (uint32_t)__builtin_amdgcn_readlane((int)v.op0, o)
                                               : (uint32_t)__builtin_amdgcn_readfirstlane((int)v.cig[o]);
                    if ((op & 15) != MH_OP_I) continue;
                    const int il = (int)(op >> 4);
                    const int rdo = __builtin_amdgcn_readfirstlane(L.opread(pass)[o]);
                    const int key = rdo + pad(pass);
                    int mn = 255;
                    for (int x0 = 0; x0 < il; x0 += 64) {
                        char tc, tq;
                        if (x0 + lane < il) {
                            sam_base(A.R, v, rdo + x0 + lane, tc, tq);
                            mn = (unsigned char)tq < mn ? (unsigned char)tq : mn;
                        }
                    }
                    mn = wave_min_all(mn);
                    if (!(mn > cut)) continue;
                    if (used + 2 * il + 2 > PU_INSBUF) {
                        if (lane == 0) atomicExch(&A.ev_ctr[3], 1ull);
                        continue;
                    }
                    // an existing entry with the same key (ins1 vs ins2): the last one
                    int at = -1;
                    const uint64_t same = __builtin_amdgcn_ballot_w64(lane < n && keyv == key);
                    if (same) at = 63 - (int)__builtin_clzll(same);
                    for (int z = 64; z < n; ++z)
                        if (__builtin_amdgcn_readfirstlane(I.key[z]) == key) at = z;
                    char *dst = I.buf + used;
                    int outlen;
                    if (pass == 0) {
                        for (int x0 = 0; x0 < il; x0 += 64) {
                            char tc, tq;
                            if (x0 + lane < il) {
                                sam_base(A.R, v, rdo + x0 + lane, tc, tq);
                                dst[x0 + lane] = tc;
                            }
                        }
                        outlen = il;
                    } else {
                        // ins1 at this key (even if it failed quality) merges with ins2
                        int l1 = 0, o1s = 0;
                        const RowV &w = m0;
                        for (int o1 = 0; o1 < w.n_cigar; ++o1) {
                            const uint32_t op1 = o1 < 64 ? (uint32_t)__builtin_amdgcn_readlane((int)w.op0, o1)
                                                         : (uint32_t)__builtin_amdgcn_readfirstlane((int)w.cig[o1]);
                            if ((op1 & 15) != MH_OP_I) continue;
                            const int r1 = __builtin_amdgcn_readfirstlane(L.opread(0)[o1]);
                            if (r1 + padA != key) continue;
                            l1 = (int)(op1 >> 4);
                            if (l1 > PU_INSBUF / 8) l1 = PU_INSBUF / 8;
                            o1s = r1;
                        }
                        const int l2 = il > PU_INSBUF / 8 ? PU_INSBUF / 8 : il;
                        // merge_pairs on the two strings (sam2aln.py:156-237): the
                        // shorter one plays seq1
                        const bool sw = l1 > l2;
                        const int la = sw ? l2 : l1, lb = sw ? l1 : l2;
                        const int oa = sw ? rdo : o1s, ob = sw ? o1s : rdo;
                        const int reva = sw ? v.rev : w.rev, ma = sw ? v.m : w.m;
                        const int revb = sw ? w.rev : v.rev, mb = sw ? w.m : v.m;
                        const int64_t roffa = sw ? v.roff : w.roff, roffb = sw ? w.roff : v.roff;
                        for (int i0 = 0; i0 < lb; i0 += 64) {
                            const int i = i0 + lane;
                            if (i >= lb) continue;
                            char c2, q2c;
                            sam_base_at(A.R, revb, mb, roffb, ob + i, c2, q2c);
                            const unsigned char b = (unsigned char)q2c;
                            char oc;
                            if (i < la) {
                                char c1, q1c;
                                sam_base_at(A.R, reva, ma, roffa, oa + i, c1, q1c);
                                const unsigned char a = (unsigned char)q1c;
                                if (c1 == c2) {
                                    oc = (a > cut || b > cut) ? c1 : 'N';
                                } else {
                                    const int dq = (int)b - (int)a;
                                    if ((dq < 0 ? -dq : dq) >= 5) {
                                        const unsigned char m2 = b > cut ? b : cut, m1 = a > cut ? a : cut;
                                        oc = a > m2 ? c1 : (b > m1 ? c2 : 'N');
                                    } else {
                                        oc = 'N';
                                    }
                                }
                            } else {
                                oc = b > cut ? c2 : 'N';
                            }
                            dst[i] = oc;
                        }
                        outlen = lb;
                    }
                    if (at < 0) at = n++;
                    if (lane == 0) {
                        I.key[at] = key;
                        I.off[at] = used;
                        I.len[at] = outlen;
                    }
                    if (lane == at) keyv = key;
                    used += outlen;
                }
            }
            if (lane == 0) *L.n_ins = n;
        }
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");

        // ---- merge_pairs positions: seq1 = shorter padded read ----
        int a = 0, b = 1;             // mate indices of seq1 / seq2
        int len1, len2, pad1, pad2;
        if (nm == 1) {
            a = -1; b = 0;
            len1 = 0; pad1 = 0;
        } else if (lenA > lenB) {
            a = 1; b = 0;
        }
        if (a >= 0) { len1 = len(a); pad1 = pad(a); }
        len2 = len(b);
        pad2 = pad(b);
        auto ch1 = [&](int i, char &c, char &q) {
            if (i < pad1) { c = '-'; q = '!'; } else { c = L.c(a)[i - pad1]; q = L.q(a)[i - pad1]; }
        };
        auto ch2 = [&](int i, char &c, char &q) {
            if (i < pad2) { c = '-'; q = '!'; } else { c = L.c(b)[i - pad2]; q = L.q(b)[i - pad2]; }
        };
        const int lo = a >= 0 ? (pad1 < pad2 ? pad1 : pad2) : pad2;
        // first index where seq2 is not '-' (is_reverse_started) and where the
        // forward read starts (first i < len1 not both '-')
        int rev_start = 1 << 30, fwd_start = 1 << 30;
        // both padded reads start with a base at their pad (the common case):
        // seq2 starts at pad2 and the forward read at min(pad1, pad2)
        const bool starts_b = len2 > pad2 &&
                              __builtin_amdgcn_readfirstlane((int)(unsigned char)L.c(b)[0]) != '-';
        const bool starts_a = a < 0 || (len1 > pad1 &&
                              __builtin_amdgcn_readfirstlane((int)(unsigned char)L.c(a)[0]) != '-');
        if (starts_b && starts_a) {
            rev_start = pad2;
            if (a >= 0) fwd_start = pad1 < pad2 ? pad1 : pad2;
        }
        for (int i0 = lo; i0 < len2 && !(starts_b && starts_a); i0 += 64) {
            const int i = i0 + lane;
            int rs = 1 << 30, fs = 1 << 30;
            if (i < len2) {
                char c2, q2;
                ch2(i, c2, q2);
                if (c2 != '-') rs = i;
                if (a >= 0 && i < len1) {
                    char c1, q1;
                    ch1(i, c1, q1);
                    if (!(c1 == '-' && c2 == '-')) fs = i;
                }
            }
            rs = wave_min_all(rs);
            fs = wave_min_all(fs);
            rev_start = min(rev_start, rs);
            fwd_start = min(fwd_start, fs);
            if (rev_start < (1 << 30) && (a < 0 || fwd_start < (1 << 30) || i0 + 64 >= len1)) break;
        }
        const bool fwd = a >= 0 && fwd_start < len1;
        // mseq = seq1[:i] + ... when the forward read starts, else only the
        // part past len1 is appended (sam2aln.py:192-199, :220-230)
        const int shift = fwd ? 0 : len1;
        // The first mseq character that is not '-' starts update_counts
        // (remap.py:286-289): the merged base at fwd_start (never '-', a gap's
        // quality ' '/'!' cannot win), else the first index >= len1 (a base or
        // 'n').  From there on every position counts, so the loop starts at
        // fwd_start, or at rev_start skipping the 'n' interval before it.
        const int begin = fwd ? fwd_start : rev_start;

        // ---- update_counts over mseq (remap.py:284-301) ----
        int mxp = 0;
        int err = 0;
        const int n_ins = *L.n_ins;
        // the first merged-insertion keys in registers: a position tests them
        // without a global load (keys are distinct; > 4 is rare)
        int ik0 = -1, ik1 = -1, ik2 = -1, ik3 = -1;
        if (n_ins > 0) ik0 = __builtin_amdgcn_readfirstlane(I.key[0]);
        if (n_ins > 1) ik1 = __builtin_amdgcn_readfirstlane(I.key[1]);
        if (n_ins > 2) ik2 = __builtin_amdgcn_readfirstlane(I.key[2]);
        if (n_ins > 3) ik3 = __builtin_amdgcn_readfirstlane(I.key[3]);
        // this reference's LDS counter window (wo < 0: none), wl positions
        const int wo = __builtin_amdgcn_readfirstlane(wmap[2 * ref]);
        const int wl = __builtin_amdgcn_readfirstlane(wmap[2 * ref + 1]);
        // the merged character of position i (sam2aln merge_pairs, :192-237),
        // 0 past seq2; every LDS read unconditional (clamped index) so the two
        // positions of a round read together
        auto merged = [&](int i) -> char {
            const bool in2 = i < len2, in1 = a >= 0 && i < len1;
            const int j2 = i >= pad2 && in2 ? i - pad2 : 0;
            const int j1 = in1 && i >= pad1 ? i - pad1 : 0;
            const char c2r = L.c(b)[j2], q2r = L.q(b)[j2];
            const char c1r = L.c(a >= 0 ? a : 0)[j1], q1r = L.q(a >= 0 ? a : 0)[j1];
            const char c2 = i < pad2 ? '-' : c2r, q2 = i < pad2 ? '!' : q2r;
            const char c1 = i < pad1 ? '-' : c1r, q1 = i < pad1 ? '!' : q1r;
            // as selects, not branches: the lanes of a round take every case
            const int qa = (unsigned char)q1, qb = (unsigned char)q2, ic = (int)cut;
            const int dq = qb > qa ? qb - qa : qa - qb;
            const int m2 = qb > ic ? qb : ic, m1 = qa > ic ? qa : ic;
            const char mdiff = qa > m2 ? c1 : (qb > m1 ? c2 : 'N');
            const char msame = (qa > ic || qb > ic) ? c1 : 'N';
            const char m_in1 = (c1 == '-' && c2 == '-') ? '-' : (c1 == c2 ? msame : (dq >= 5 ? mdiff : 'N'));
            const char m_out = c2 == '-' ? (i >= rev_start ? '-' : 'n') : (qb > ic ? c2 : 'N');
            const char mc = in1 ? m_in1 : m_out;
            return in2 ? mc : (char)0;
        };
        // update_counts of one merged character
        auto count = [&](int i, char mc) {
            // bitwise, not short-circuit: the tests stay selects, not branches
            const int P = i - shift + 1;
            const bool live = (mc != 0) & (mc != 'n');
            err |= (int)(live & (P > A.cap));
            const bool ok = live & (P <= A.cap);
            mxp = (ok & (P > mxp)) ? P : mxp;
            const int64_t cell = (int64_t)ref * A.cap + (P - 1);
            const bool isN = mc == 'N', isD = mc == '-';
            if (ok & isN) A.nflag[cell] = 1;
            if (ok & isD) A.dflag[cell] = 1;
            bool base = ok & !isN & !isD;
            if (n_ins > 0) {
                int hit = -1;   // keys are distinct and >= 1 (-1: no key)
                hit = P == ik3 ? 3 : hit;
                hit = P == ik2 ? 2 : hit;
                hit = P == ik1 ? 1 : hit;
                hit = P == ik0 ? 0 : hit;
                for (int z = 4; z < n_ins; ++z)
                    if (I.key[z] == P) hit = z;
                if (base && hit >= 0 && I.len[hit] > 0 && I.len[hit] % 3 == 0) {
                    base = false;
                    const int tl = 1 + I.len[hit];
                    const unsigned long long e = atomicAdd(&A.ev_ctr[0], 1ull);
                    const unsigned long long p = atomicAdd(&A.ev_ctr[1], (unsigned long long)tl);
                    if ((long long)e < A.ev_cap && (long long)(p + tl) <= A.pool_cap) {
                        A.ev[4 * e] = ref;
                        A.ev[4 * e + 1] = P;
                        A.ev[4 * e + 2] = (int32_t)p;
                        A.ev[4 * e + 3] = tl;
                        A.ev_pool[p] = mc;
                        for (int x = 0; x < tl - 1; ++x) A.ev_pool[p + 1 + x] = I.buf[I.off[hit] + x];
                    } else {
                        atomicExch(&A.ev_ctr[2], 1ull);
                    }
                }
            }
            if (base) {
                // A C G T (0x41 0x43 0x47 0x54) -> 0 1 2 3 without a branch
                const int code = (((int)mc >> 1) ^ ((int)mc >> 2)) & 3;
                // u16 halves: a block counts < 65536 units (pile_geometry)
                if (wo >= 0 && P <= wl) atomicAdd(&win[wo + (code >> 1) * wl + (P - 1)], 1u << (16 * (code & 1)));
                else atomicAdd(&A.dense[cell * 4 + code], 1);
            }
        };
        for (int i0 = begin; i0 < len2; i0 += 128) {
            const int ia = i0 + lane, ib = ia + 64;
            const char ma = merged(ia), mb = merged(ib);
            count(ia, ma);
            count(ib, mb);
        }
        mxp = wave_max_all(mxp);
        err = wave_max_all(err);
        if (lane == 0) {
            atomicAdd(&rl[ref].read_count, 1u);
            atomicMin(&rl[ref].first_unit, (long long)u);
            if (mxp > 0) atomicMax(&rl[ref].max_pos, mxp);
            if (err) atomicExch(&A.ev_ctr[3], 1ull);
        }
        __builtin_amdgcn_wave_barrier();
    }
    // ---- flush the block's windows (consecutive threads add to consecutive
    // words of dense: cell-major, A/C/G/T minor) and per-reference scalars ----
    __syncthreads();
    for (int r = 0; r < NR; ++r) {
        const int wo = wmap[2 * r], wl = wmap[2 * r + 1];
        if (wo < 0) continue;
        int32_t *dst = A.dense + (int64_t)r * A.cap * 4;
        for (int x = threadIdx.x; x < 4 * wl; x += blockDim.x) {   // x = 4 position + base
            const unsigned int v = (win[wo + ((x & 3) >> 1) * wl + (x >> 2)] >> (16 * (x & 1))) & 0xffffu;
            if (v) atomicAdd(&dst[x], (int)v);
        }
    }
    for (int r = threadIdx.x; r < NR; r += blockDim.x) {
        if (!rl[r].read_count) continue;
        atomicAdd(&A.read_counts[r], (unsigned long long)rl[r].read_count);
        atomicMin(&A.first_unit[r], rl[r].first_unit);
        if (rl[r].max_pos > 0) atomicMax(&A.max_pos[r], rl[r].max_pos);
    }
}

__global__ void k_pile_init(long long *first_unit, int32_t *max_pos, int n)
{
    for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
        first_unit[i] = INT64_MAX;
        max_pos[i] = 0;
    }
}

__global__ void k_pile_fix(long long *first_unit, int n)
{
    for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x)
        if (first_unit[i] == INT64_MAX) first_unit[i] = -1;
}

static int ensure_pile(Ctx &c)
{
    PileState &P = c.pile;
    const int64_t cells = (int64_t)(P.n_refs > 0 ? P.n_refs : 1) * P.cap;
    if (P.alloc_cells < cells) {
        hipFree(P.dense); hipFree(P.nflag); hipFree(P.dflag);
        MH_HIP(hipMalloc(&P.dense, sizeof(int32_t) * 4 * cells));
        MH_HIP(hipMalloc(&P.nflag, cells));
        MH_HIP(hipMalloc(&P.dflag, cells));
        P.alloc_cells = cells;
    }
    if (P.alloc_refs < (P.n_refs > 0 ? P.n_refs : 1)) {
        hipFree(P.read_counts); hipFree(P.first_unit); hipFree(P.max_pos);
        const int nr = P.n_refs > 0 ? P.n_refs : 1;
        MH_HIP(hipMalloc(&P.read_counts, sizeof(int64_t) * nr));
        MH_HIP(hipMalloc(&P.first_unit, sizeof(int64_t) * nr));
        MH_HIP(hipMalloc(&P.max_pos, sizeof(int32_t) * nr));
        P.alloc_refs = nr;
    }
    if (!P.ev_counters) MH_HIP(hipMalloc(&P.ev_counters, sizeof(int64_t) * 4));
    // event records and their token bytes: grown by the retry in run_pileup;
    // a capacity imposed by a test is where every pileup starts
    const int64_t t_ev = c.test_caps.pile_events, t_pool = c.test_caps.pile_event_bytes;
    if (!P.ev || (t_ev > 0 && P.ev_cap != t_ev)) {
        hipFree(P.ev);
        P.ev = nullptr;
        P.ev_cap = t_ev > 0 ? t_ev : 1 << 16;
        MH_HIP(hipMalloc(&P.ev, sizeof(int32_t) * 4 * P.ev_cap));
    }
    if (!P.ev_pool || (t_pool > 0 && P.pool_cap != t_pool)) {
        hipFree(P.ev_pool);
        P.ev_pool = nullptr;
        P.pool_cap = t_pool > 0 ? t_pool : 1 << 20;
        MH_HIP(hipMalloc(&P.ev_pool, P.pool_cap));
    }
    return 0;
}

// Launch shape of k_pileup.  Every reference keeps its scalars (read count,
// first unit, last position) in LDS, and the references the units map to,
// most-hit first, get their A/C/G/T counters for positions 1..len+64 in LDS
// too (an A|C and a G|T plane, one count per u16 half) as long as they fit
// beside 8 waves' staging areas: the memory-side int atomics of the dense
// counters are the kernel's cost otherwise.  The rest holds one staging
// area per wave.
struct PileGeometry {
    int span = 0, unit_bytes = 0, wpb = 1, win_words = 0;
    std::vector<int32_t> win_map;   // per reference: first window word (-1: none), positions
    int64_t blocks = 1;
    size_t lds = 0;
};

// a block's u16 window halves must not wrap: fewer units per block than this
constexpr int64_t PU_UNITS_PER_BLOCK = 60000;

static int pile_geometry(Ctx &c, int source, int64_t n_units, PileGeometry &g)
{
    PileState &P = c.pile;
    const int NR = P.n_refs;
    std::vector<int64_t> hits((size_t)NR, 0);   // units expected per reference
    int span = 0;
    if (source == 0) {
        span = c.reads.max_len + BAND;   // M + D <= read length + band width
        const int n = c.map.n_refs;
        const int64_t *st = map_stats_host(c);
        if (!st) return -1;
        for (int r = 0; r < n && r < NR; ++r) hits[(size_t)r] = st[2 * (size_t)n + r];
    } else {
        span = c.rows.max_span;
        for (int r = 0; r < NR && r < (int)c.rows.ref_rows.size(); ++r) hits[(size_t)r] = c.rows.ref_rows[(size_t)r];
    }
    g.span = ((span > 16 ? span : 16) + 15) & ~15;
    g.unit_bytes = (unit_bytes_for(g.span) + 15) & ~15;
    const size_t base = (sizeof(RefLds) + 2 * sizeof(int32_t)) * (size_t)NR;
    if (base + (size_t)g.unit_bytes > (size_t)PU_LDS) {
        set_error("mh_pileup: reference span %d / %d references do not fit in LDS", span, NR);
        return -3;
    }
    const int64_t room = (int64_t)PU_LDS - (int64_t)base - 8 * (int64_t)g.unit_bytes;
    std::vector<int> order((size_t)NR);
    for (int r = 0; r < NR; ++r) order[(size_t)r] = r;
    std::stable_sort(order.begin(), order.end(), [&](int x, int y) { return hits[(size_t)x] > hits[(size_t)y]; });
    // references outside mh_pileup_only's set: skipped (-2), no window
    const bool some = P.only.size() == (size_t)NR;
    for (int r = 0; r < NR && some; ++r) if (!P.only[(size_t)r]) hits[(size_t)r] = 0;
    g.win_map.assign(2 * (size_t)NR, 0);
    for (int r = 0; r < NR; ++r) g.win_map[2 * (size_t)r] = some && !P.only[(size_t)r] ? -2 : -1;
    int64_t words = 0;
    for (int r : order) {
        if (hits[(size_t)r] <= 0) break;
        int want = P.ref_lens[(size_t)r] + 64;
        if (want > P.cap) want = P.cap;
        if (want < 1 || 4 * (words + 2 * (int64_t)want) > room) continue;
        g.win_map[2 * (size_t)r] = (int32_t)words;
        g.win_map[2 * (size_t)r + 1] = want;
        words += 2 * (int64_t)want;
    }
    g.win_words = (int)words;
    // The block shape that keeps the most waves resident per CU: k_pileup is
    // a chain of dependent loads per unit and runs as fast as the waves in
    // flight; its 80 VGPRs allow 24 per CU, which one block of 16 waves
    // leaves at 16 (2 blocks of 12 waves: 8.0 -> 6.5 ms per C2 step).  LDS
    // per block is the windows plus the waves' staging areas.
    const int64_t lds0 = (int64_t)base + 4 * words;
    const auto key = std::make_tuple(source, lds0, g.unit_bytes);
    auto hit = P.shapes.find(key);
    if (hit == P.shapes.end()) {
        if (!c.n_cu) MH_HIP(hipDeviceGetAttribute(&c.n_cu, hipDeviceAttributeMultiprocessorCount, c.device));
        // the skipping instances have the same resources (the occupancy
        // query of the full ones stands for them)
        const void *kern = source == 0 ? (const void *)k_pileup<0, false> : (const void *)k_pileup<1, false>;
        MH_HIP(hipFuncSetAttribute(kern, hipFuncAttributeMaxDynamicSharedMemorySize, PU_LDS));
        int best_w = 0, best_wpb = 1, best_nb = 1;
        for (int wpb = 16; wpb >= 1; --wpb) {
            const int64_t lds = lds0 + (int64_t)wpb * g.unit_bytes;
            if (lds > PU_LDS) continue;
            int nb = 0;
            MH_HIP(hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, kern, 64 * wpb, (size_t)lds));
            if (nb * wpb > best_w) { best_w = nb * wpb; best_wpb = wpb; best_nb = nb; }
        }
        hit = P.shapes.emplace(key, std::make_pair(best_wpb, best_nb > 0 ? best_nb : 1)).first;
    }
    g.wpb = hit->second.first;
    g.lds = (size_t)lds0 + (size_t)g.wpb * g.unit_bytes;
    g.blocks = (n_units + g.wpb - 1) / g.wpb;
    // windows: one resident wave of blocks (each flushes its windows once);
    // without windows more blocks than fit, grid-strided
    const int64_t n_cu = c.n_cu > 0 ? c.n_cu : 256;
    const int64_t max_blocks = words > 0 ? n_cu * hit->second.second : n_cu * 8;
    if (g.blocks > max_blocks) g.blocks = max_blocks;
    if (words > 0 && g.blocks < (n_units + PU_UNITS_PER_BLOCK - 1) / PU_UNITS_PER_BLOCK)
        g.blocks = (n_units + PU_UNITS_PER_BLOCK - 1) / PU_UNITS_PER_BLOCK;
    if (g.blocks < 1) g.blocks = 1;
    return 0;
}

int run_pileup(Ctx &c, int source, int q_cutoff)
{
    PileState &P = c.pile;
    ++P.gen;
    int64_t n_units;
    const DevReads *R;
    if (source == 0) {
        if (!c.map.valid) { set_error("mh_pileup: no mapping results"); return -3; }
        R = &c.reads;
        n_units = c.reads.paired ? c.reads.n / 2 : c.reads.n;
    } else {
        R = &c.rows.reads;
        n_units = c.rows.n_units;
    }
    if (int st = ensure_pile(c)) return st;
    hipStream_t s = c.stream;
    PileGeometry geo;
    if (int st = pile_geometry(c, source, n_units, geo)) return st;
    {
        const int64_t need = geo.blocks * geo.wpb * (int64_t)PU_INS_BYTES;
        if (P.ins_scratch_bytes < need) {
            hipFree(P.ins_scratch);
            P.ins_scratch = nullptr;
            MH_HIP(hipMalloc(&P.ins_scratch, need));
            P.ins_scratch_bytes = need;
        }
    }
    if (P.win_map_cap < 2 * P.n_refs || !P.win_map) {
        hipFree(P.win_map);
        P.win_map = nullptr;
        P.win_map_cap = 2 * (P.n_refs > 16 ? P.n_refs : 16);
        MH_HIP(hipMalloc(&P.win_map, sizeof(int32_t) * P.win_map_cap));
    }
    if (P.n_refs > 0)
        MH_HIP(hipMemcpyAsync(P.win_map, geo.win_map.data(), sizeof(int32_t) * 2 * P.n_refs,
                              hipMemcpyHostToDevice, s));
    const int64_t cells = (int64_t)P.n_refs * P.cap;
    for (int attempt = 0; attempt < 3; ++attempt) {
        MH_HIP(hipMemsetAsync(P.dense, 0, sizeof(int32_t) * 4 * (cells > 0 ? cells : 1), s));
        MH_HIP(hipMemsetAsync(P.nflag, 0, cells > 0 ? cells : 1, s));
        MH_HIP(hipMemsetAsync(P.dflag, 0, cells > 0 ? cells : 1, s));
        MH_HIP(hipMemsetAsync(P.read_counts, 0, sizeof(int64_t) * (P.n_refs > 0 ? P.n_refs : 1), s));
        MH_HIP(hipMemsetAsync(P.ev_counters, 0, sizeof(int64_t) * 4, s));
        hipLaunchKernelGGL(k_pile_init, dim3(8), dim3(256), 0, s, (long long *)P.first_unit,
                           P.max_pos, P.n_refs);
        PileArgs A{};
        A.rec = c.map.rec;
        A.pool = c.map.pool;
        A.R = *R;
        A.paired = source == 0 ? c.reads.paired : 0;
        A.flag = c.rows.flag; A.ref = c.rows.ref; A.pos = c.rows.pos; A.cig_off = c.rows.cig_off;
        A.n_cigar = c.rows.n_cigar; A.cigar = c.rows.cigar; A.units = c.rows.units;
        A.n_units = n_units;
        A.n_refs = P.n_refs;
        A.cap = P.cap;
        A.dense = P.dense; A.nflag = P.nflag; A.dflag = P.dflag;
        A.read_counts = (unsigned long long *)P.read_counts;
        A.first_unit = (long long *)P.first_unit;
        A.max_pos = P.max_pos;
        A.ev = P.ev; A.ev_pool = P.ev_pool; A.ev_cap = P.ev_cap; A.pool_cap = P.pool_cap;
        A.ev_ctr = (unsigned long long *)P.ev_counters;
        A.q_cutoff = q_cutoff;
        A.win_map = P.win_map;
        A.win_words = geo.win_words;
        A.span_cap = geo.span;
        A.unit_bytes = geo.unit_bytes;
        A.ins_scratch = P.ins_scratch;
        if (n_units > 0) {
            const int pk = prof_begin(c, "k_pileup");
            const bool skip = P.only.size() == (size_t)P.n_refs &&
                              std::find(P.only.begin(), P.only.end(), (uint8_t)0) != P.only.end();
            const void *kern = source == 0 ? (skip ? (const void *)k_pileup<0, true> : (const void *)k_pileup<0, false>)
                                           : (skip ? (const void *)k_pileup<1, true> : (const void *)k_pileup<1, false>);
            MH_HIP(hipFuncSetAttribute(kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)geo.lds));
            void *kargs[] = {&A};
            MH_HIP(hipLaunchKernel(kern, dim3((unsigned)geo.blocks), dim3(64 * geo.wpb), kargs, geo.lds, s));
            prof_end(c, pk);
            MH_HIP(hipGetLastError());
        }
        hipLaunchKernelGGL(k_pile_fix, dim3(8), dim3(256), 0, s, (long long *)P.first_unit, P.n_refs);
        int64_t ctr[4];
        MH_HIP(hipMemcpyAsync(ctr, P.ev_counters, sizeof(ctr), hipMemcpyDeviceToHost, s));
        MH_HIP(hipStreamSynchronize(s));
        if (ctr[3]) { set_error("mh_pileup: malformed alignment row (CIGAR/position)"); return -3; }
        if (!ctr[2]) return 0;
        // events or token bytes past their buffers: grow both to what the
        // launch asked for (the counters count every claim) and run it again
        ++c.retries[RETRY_PILE_EVENTS];
        hipFree(P.ev); hipFree(P.ev_pool);
        P.ev = nullptr; P.ev_pool = nullptr;
        P.ev_cap = ctr[0] * 2 + 1024;
        P.pool_cap = ctr[1] * 2 + 4096;
        MH_HIP(hipMalloc(&P.ev, sizeof(int32_t) * 4 * P.ev_cap));
        MH_HIP(hipMalloc(&P.ev_pool, P.pool_cap));
    }
    set_error("mh_pileup: event buffer overflow");
    return -2;
}

// ---- token events aggregated on the device -----------------------------------
// Every merged pair with an insertion token at a counted position left one
// event (ref, pos, tok_off, tok_len) and its bytes in the pool.  The host
// needs the distinct (ref, pos, token) keys with their counts (remap.py's
// per-position Counter of tokens).  One thread per event hashes its key and
// claims or joins a slot of an open-addressing table (the first event to claim
// a slot represents the key; joining compares the bytes with it); the used
// slots are listed, and a second pass gathers the representatives' metadata and
// bytes.  Only the distinct keys cross PCIe; the order is fixed on the host by
// sorting them, so the result does not depend on which event claimed a slot.
__device__ __forceinline__ uint64_t token_hash(int32_t ref, int32_t pos, const char *b, int32_t len)
{
    uint64_t h = 1469598103934665603ull;
    for (int32_t x = 0; x < len; ++x) h = (h ^ (unsigned char)b[x]) * 1099511628211ull;
    h ^= ((uint64_t)(uint32_t)ref << 32) | (uint32_t)pos;
    h ^= h >> 33; h *= 0xff51afd7ed558ccdull; h ^= h >> 33;
    return h;
}

__device__ __forceinline__ bool same_event(const int32_t *ev, const char *pool, int64_t u, int32_t r,
                                           int32_t ps, int32_t of, int32_t ln)
{
    bool same = ev[4 * u] == r && ev[4 * u + 1] == ps && ev[4 * u + 3] == ln;
    for (int32_t x = 0; same && x < ln; ++x) same = pool[ev[4 * u + 2] + x] == pool[of + x];
    return same;
}

// pass 1: every event finds (or claims) the slot of its key; eslot[e] = slot.
// Most events repeat a few keys (one insertion at one position, seen by many
// reads), and a claim on the global table is a same-address CAS that the
// device serialises.  Each block therefore first groups its events in an LDS
// table (the first event of a key in the block leads it); only the leaders go
// to the global table, and the other events copy their leader's slot.
constexpr int TOK_LDS_SLOTS = 4096;
constexpr int TOK_LDS_PROBES = 32;
__global__ __launch_bounds__(1024) void k_tok_insert(const int32_t *ev, const char *pool, int64_t ne,
                                                     int32_t *slot, int32_t *used, int32_t *eslot,
                                                     int64_t mask)
{
    __shared__ int32_t lrep[TOK_LDS_SLOTS];    // leader event + 1 (0: free)
    __shared__ int32_t lglob[TOK_LDS_SLOTS];   // the leader's global slot
    for (int x = threadIdx.x; x < TOK_LDS_SLOTS; x += blockDim.x) lrep[x] = 0;
    __syncthreads();
    const int64_t per = (ne + gridDim.x - 1) / gridDim.x;
    const int64_t a = (int64_t)blockIdx.x * per, b = a + per < ne ? a + per : ne;
    for (int64_t e0 = a; e0 < b; e0 += blockDim.x) {   // block-uniform rounds
        const int64_t e = e0 + threadIdx.x;
        const bool live = e < b;
        int32_t r = 0, ps = 0, of = 0, ln = 0;
        uint64_t h = 0;
        int li = -1;          // LDS entry of this event's key (-1: table full)
        bool lead = false;
        if (live) {
            r = ev[4 * e]; ps = ev[4 * e + 1]; of = ev[4 * e + 2]; ln = ev[4 * e + 3];
            h = token_hash(r, ps, pool + of, ln);
            int x = (int)((h >> 40) & (TOK_LDS_SLOTS - 1));
            for (int p = 0; p < TOK_LDS_PROBES; ++p, x = (x + 1) & (TOK_LDS_SLOTS - 1)) {
                int32_t s = lrep[x];
                if (s == 0) {
                    s = atomicCAS(&lrep[x], 0, (int32_t)(e + 1));
                    if (s == 0) { li = x; lead = true; break; }
                }
                if (same_event(ev, pool, s - 1, r, ps, of, ln)) { li = x; break; }
            }
        }
        __syncthreads();
        if (live && (lead || li < 0)) {   // global find-or-claim, once per key per block
            int64_t i = (int64_t)(h & (uint64_t)mask);
            for (;;) {
                int32_t s = slot[i];
                if (s == 0) {
                    s = atomicCAS(&slot[i], 0, (int32_t)(e + 1));
                    if (s == 0) {   // claimed: this event represents the key
                        used[1 + atomicAdd(&used[0], 1)] = (int32_t)i;
                        break;
                    }
                }
                if (same_event(ev, pool, s - 1, r, ps, of, ln)) break;
                i = (i + 1) & mask;
            }
            eslot[e] = (int32_t)i;
            if (lead) lglob[li] = (int32_t)i;
        }
        __syncthreads();
        if (live && !lead && li >= 0) eslot[e] = lglob[li];
    }
}

// key number of every used slot (slot -> d)
__global__ void k_tok_number(const int32_t *used, int32_t *slotid)
{
    const int nd = used[0];
    for (int d = blockIdx.x * blockDim.x + threadIdx.x; d < nd; d += gridDim.x * blockDim.x)
        slotid[used[1 + d]] = d;
}

// pass 2: counts per key.  A few blocks, each over a contiguous range of
// events, count in LDS and add their totals once per key: a popular key gets
// one global atomic per block instead of one per event.
constexpr int TOK_LDS_KEYS = 8192;
__global__ __launch_bounds__(1024) void k_tok_count(const int32_t *eslot, int64_t ne,
                                                    const int32_t *slotid, const int32_t *used,
                                                    uint32_t *cnt)
{
    __shared__ uint32_t hist[TOK_LDS_KEYS];
    const int nd = used[0];
    const bool lds = nd <= TOK_LDS_KEYS;
    if (lds)
        for (int d = threadIdx.x; d < nd; d += blockDim.x) hist[d] = 0;
    __syncthreads();
    const int64_t per = (ne + gridDim.x - 1) / gridDim.x;
    const int64_t a = (int64_t)blockIdx.x * per, b = a + per < ne ? a + per : ne;
    for (int64_t e = a + threadIdx.x; e < b; e += blockDim.x) {
        const int d = slotid[eslot[e]];
        if (lds) atomicAdd(&hist[d], 1u);
        else atomicAdd(&cnt[d], 1u);
    }
    __syncthreads();
    if (lds)
        for (int d = threadIdx.x; d < nd; d += blockDim.x)
            if (hist[d]) atomicAdd(&cnt[d], hist[d]);
}

// distinct key d: meta[5d..5d+4] = (ref, pos, offset in bytes, len, count);
// offsets are a prefix over the keys' lengths (one wave, serial chunks)
__global__ void k_tok_gather(const int32_t *ev, const char *pool, const int32_t *slot,
                             const uint32_t *cnt, const int32_t *used, int32_t *meta,
                             char *bytes, int64_t bytes_cap, int32_t *overflow)
{
    const int lane = threadIdx.x;
    const int nd = used[0];
    int base = 0;
    for (int d0 = 0; d0 < nd; d0 += 64) {
        const int d = d0 + lane;
        int32_t ln = 0, u = 0, i = 0;
        if (d < nd) {
            i = used[1 + d];
            u = slot[i] - 1;
            ln = ev[4 * u + 3];
        }
        const int incl = wave_incl_scan(ln, lane);
        const int off = base + incl - ln;
        if (d < nd) {
            meta[5 * d] = ev[4 * u];
            meta[5 * d + 1] = ev[4 * u + 1];
            meta[5 * d + 2] = off;
            meta[5 * d + 3] = ln;
            meta[5 * d + 4] = (int32_t)cnt[d];
            if (off + ln <= bytes_cap) {
                for (int32_t x = 0; x < ln; ++x) bytes[off + x] = pool[ev[4 * u + 2] + x];
            } else {
                *overflow = 1;
            }
        }
        base += __builtin_amdgcn_readlane(incl, 63);
    }
}

int run_token_aggregate(Ctx &c, int64_t ne, int64_t pool_used, std::vector<int32_t> &meta,
                        std::string &bytes)
{
    PileState &P = c.pile;
    hipStream_t s = c.stream;
    meta.clear();
    bytes.clear();
    if (ne <= 0) return 0;
    int64_t cap = 1024;
    while (cap < 2 * ne) cap <<= 1;
    if (P.tok_cap < cap) {
        hipFree(P.tok_slot); hipFree(P.tok_cnt); hipFree(P.tok_used);
        P.tok_slot = nullptr; P.tok_cnt = nullptr; P.tok_used = nullptr; P.tok_cap = 0;
        // slot (cap), slot -> key number (cap), per-event slot (<= cap / 2)
        MH_HIP(hipMalloc(&P.tok_slot, sizeof(int32_t) * 2 * cap + sizeof(int32_t) * (cap / 2 + 1)));
        MH_HIP(hipMalloc(&P.tok_cnt, sizeof(uint32_t) * cap));
        MH_HIP(hipMalloc(&P.tok_used, sizeof(int32_t) * (cap + 1)));
        P.tok_cap = cap;
    }
    // room for every event to be a distinct key, and the overflow flag after it
    if (P.tok_meta_cap < ne) {
        hipFree(P.tok_meta);
        P.tok_meta = nullptr;
        P.tok_meta_cap = 0;
        MH_HIP(hipMalloc(&P.tok_meta, sizeof(int32_t) * (5 * (size_t)ne + 1)));
        P.tok_meta_cap = ne;
    }
    int32_t *ovf = P.tok_meta + 5 * (size_t)P.tok_meta_cap;
    // the distinct keys' bytes are a subset of the events' pool: sized by it,
    // the gather cannot overflow (a test may impose less, to run the retry)
    const int64_t want = c.test_caps.token_bytes > 0 ? c.test_caps.token_bytes
                                                     : std::max<int64_t>(pool_used, 64);
    if (P.tok_bytes_cap < want || (c.test_caps.token_bytes > 0 && P.tok_bytes_cap != want)) {
        hipFree(P.tok_bytes);
        P.tok_bytes = nullptr;
        P.tok_bytes_cap = 0;
        MH_HIP(hipMalloc(&P.tok_bytes, (size_t)want));
        P.tok_bytes_cap = want;
    }
    int32_t *slotid = P.tok_slot + cap, *eslot = P.tok_slot + 2 * cap;
    MH_HIP(hipMemsetAsync(P.tok_slot, 0, sizeof(int32_t) * cap, s));
    MH_HIP(hipMemsetAsync(P.tok_cnt, 0, sizeof(uint32_t) * cap, s));
    MH_HIP(hipMemsetAsync(P.tok_used, 0, sizeof(int32_t), s));
    int64_t blocks = (ne + 1023) / 1024;
    if (blocks > 256) blocks = 256;
    hipLaunchKernelGGL(k_tok_insert, dim3((unsigned)blocks), dim3(1024), 0, s, P.ev, P.ev_pool, ne,
                       P.tok_slot, P.tok_used, eslot, cap - 1);
    hipLaunchKernelGGL(k_tok_number, dim3(64), dim3(256), 0, s, P.tok_used, slotid);
    int64_t cblocks = (ne + 4095) / 4096;
    if (cblocks > 256) cblocks = 256;
    hipLaunchKernelGGL(k_tok_count, dim3((unsigned)cblocks), dim3(1024), 0, s, eslot, ne, slotid,
                       P.tok_used, P.tok_cnt);
    MH_HIP(hipGetLastError());
    // one round trip in the common case: the key count, the overflow flag, the
    // first keys and the first bytes, through pinned memory
    const int64_t K = std::min<int64_t>(ne, 4096), B = std::min<int64_t>(P.tok_bytes_cap, 64 << 10);
    const size_t pin_need = 16 + 20 * (size_t)K + (size_t)B;
    if (P.tok_pin_cap < pin_need) {
        if (P.tok_pin) hipHostFree(P.tok_pin);
        P.tok_pin = nullptr;
        P.tok_pin_cap = 0;
        MH_HIP(hipHostMalloc((void **)&P.tok_pin, pin_need, hipHostMallocDefault));
        P.tok_pin_cap = pin_need;
    }
    for (int attempt = 0; attempt < 2; ++attempt) {
        MH_HIP(hipMemsetAsync(ovf, 0, sizeof(int32_t), s));
        hipLaunchKernelGGL(k_tok_gather, dim3(1), dim3(64), 0, s, P.ev, P.ev_pool, P.tok_slot,
                           P.tok_cnt, P.tok_used, P.tok_meta, P.tok_bytes, P.tok_bytes_cap, ovf);
        MH_HIP(hipGetLastError());
        MH_HIP(hipMemcpyAsync(P.tok_pin, P.tok_used, sizeof(int32_t), hipMemcpyDeviceToHost, s));
        MH_HIP(hipMemcpyAsync(P.tok_pin + 4, ovf, sizeof(int32_t), hipMemcpyDeviceToHost, s));
        MH_HIP(hipMemcpyAsync(P.tok_pin + 16, P.tok_meta, 20 * (size_t)K, hipMemcpyDeviceToHost, s));
        MH_HIP(hipMemcpyAsync(P.tok_pin + 16 + 20 * (size_t)K, P.tok_bytes, (size_t)B, hipMemcpyDeviceToHost, s));
        MH_HIP(hipStreamSynchronize(s));
        int32_t nd = 0, of = 0;
        std::memcpy(&nd, P.tok_pin, 4);
        std::memcpy(&of, P.tok_pin + 4, 4);
        if (nd <= 0) return 0;
        meta.resize(5 * (size_t)nd);
        std::memcpy(meta.data(), P.tok_pin + 16, 20 * (size_t)std::min<int64_t>(nd, K));
        if (nd > K)   // more keys than the first round brought
            MH_HIP(copy_sync(c, meta.data() + 5 * (size_t)K, P.tok_meta + 5 * (size_t)K,
                             20 * (size_t)(nd - K), hipMemcpyDeviceToHost));
        const int64_t total = (int64_t)meta[5 * (size_t)(nd - 1) + 2] + meta[5 * (size_t)(nd - 1) + 3];
        if (!of) {
            bytes.resize((size_t)total);
            if (total > 0) std::memcpy(&bytes[0], P.tok_pin + 16 + 20 * (size_t)K, (size_t)std::min(total, B));
            if (total > B)
                MH_HIP(copy_sync(c, &bytes[(size_t)B], P.tok_bytes + B, (size_t)(total - B), hipMemcpyDeviceToHost));
            return 0;
        }
        // longer tokens than the room a test imposed: room for all of them
        ++c.retries[RETRY_TOKEN_BYTES];
        hipFree(P.tok_bytes);
        P.tok_bytes = nullptr;
        P.tok_bytes_cap = 0;
        MH_HIP(hipMalloc(&P.tok_bytes, (size_t)total));
        P.tok_bytes_cap = total;
    }
    set_error("mh_pileup_events: token gather overflow");
    return -2;
}

// ---- multi-GPU exchange layout ---------------------------------------------
// Multi-GPU exchange of the references selected on every rank (those with
// data anywhere): blockIdx.y = position in sel.  Buffers:
//   sum   int32: dense rows of the selected refs, then read_counts of all refs
//   mx    int32: max_pos of all refs, then -(first_unit + unit_base)
//   flags uint8: nflag rows, then dflag rows of the selected refs (MAX = OR)
__global__ void k_pile_export(const int32_t *dense, const uint8_t *nflag, const uint8_t *dflag,
                              const int64_t *read_counts, const int64_t *first_unit,
                              const int32_t *max_pos, int32_t cap, int n_refs, const int32_t *sel,
                              int n_sel, int64_t unit_base, int32_t *sum, int32_t *mx,
                              uint8_t *flags)
{
    const int sidx = blockIdx.y;
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    const int64_t t0 = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (sidx < n_sel) {
        const int64_t src = (int64_t)sel[sidx] * cap, dst = (int64_t)sidx * cap;
        for (int64_t i = t0; i < 4 * (int64_t)cap; i += stride) sum[4 * dst + i] = dense[4 * src + i];
        for (int64_t i = t0; i < cap; i += stride) {
            flags[dst + i] = nflag[src + i];
            flags[(int64_t)n_sel * cap + dst + i] = dflag[src + i];
        }
    }
    if (sidx == 0) {
        for (int64_t i = t0; i < n_refs; i += stride) {
            sum[4 * (int64_t)n_sel * cap + i] = (int32_t)read_counts[i];
            mx[i] = max_pos[i];
            mx[n_refs + i] = first_unit[i] < 0 ? INT32_MIN : (int32_t)(-(first_unit[i] + unit_base));
        }
    }
}

__global__ void k_pile_import(int32_t *dense, uint8_t *nflag, uint8_t *dflag, int64_t *read_counts,
                              int64_t *first_unit, int32_t *max_pos, int32_t cap, int n_refs,
                              const int32_t *sel, int n_sel, const int32_t *sum, const int32_t *mx,
                              const uint8_t *flags)
{
    const int sidx = blockIdx.y;
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    const int64_t t0 = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (sidx < n_sel) {
        const int64_t dst = (int64_t)sel[sidx] * cap, src = (int64_t)sidx * cap;
        for (int64_t i = t0; i < 4 * (int64_t)cap; i += stride) dense[4 * dst + i] = sum[4 * src + i];
        for (int64_t i = t0; i < cap; i += stride) {
            nflag[dst + i] = flags[src + i] ? 1 : 0;
            dflag[dst + i] = flags[(int64_t)n_sel * cap + src + i] ? 1 : 0;
        }
    }
    if (sidx == 0) {
        for (int64_t i = t0; i < n_refs; i += stride) {
            read_counts[i] = sum[4 * (int64_t)n_sel * cap + i];
            max_pos[i] = mx[i];
            const int32_t f = mx[n_refs + i];
            first_unit[i] = f == INT32_MIN ? -1 : -(int64_t)f;
        }
    }
}

}  // namespace mh

using namespace mh;

extern "C" int mh_pileup_exchange_bytes(mh_ctx *ctx, int n_sel, int64_t *sum_bytes,
                                        int64_t *max_bytes, int64_t *flag_bytes)
{
    if (!ctx || n_sel < 0) return -3;
    Ctx &c = *reinterpret_cast<Ctx *>(ctx);
    const int64_t cells = (int64_t)n_sel * c.pile.cap;
    if (sum_bytes) *sum_bytes = sizeof(int32_t) * (4 * cells + c.pile.n_refs);
    if (max_bytes) *max_bytes = sizeof(int32_t) * 2 * c.pile.n_refs;
    if (flag_bytes) *flag_bytes = 2 * cells;
    return 0;
}

static int upload_sel(Ctx &c, int n_sel, const int32_t *sel, int32_t **dsel)
{
    PileState &P = c.pile;
    for (int i = 0; i < n_sel; ++i)
        if (sel[i] < 0 || sel[i] >= P.n_refs) { set_error("pileup exchange: ref %d out of range", sel[i]); return -3; }
    if (P.sel_cap < n_sel || !P.sel) {
        hipFree(P.sel);
        P.sel = nullptr;
        P.sel_cap = n_sel > 64 ? n_sel : 64;
        MH_HIP(hipMalloc(&P.sel, sizeof(int32_t) * P.sel_cap));
    }
    if (n_sel) MH_HIP(copy_sync(c, P.sel, sel, sizeof(int32_t) * n_sel, hipMemcpyHostToDevice));
    *dsel = P.sel;
    return 0;
}

extern "C" int mh_pileup_export(mh_ctx *ctx, int n_sel, const int32_t *sel, int64_t unit_base,
                                void *dev_sum, void *dev_max, void *dev_flags)
{
    if (!ctx || !dev_sum || !dev_max || (n_sel > 0 && (!sel || !dev_flags))) return -3;
    Ctx &c = *reinterpret_cast<Ctx *>(ctx);
    PileState &P = c.pile;
    if (!P.dense) { set_error("no pileup to export"); return -3; }
    MH_HIP(hipSetDevice(c.device));
    int32_t *dsel = nullptr;
    if (int st = upload_sel(c, n_sel, sel, &dsel)) return st;
    hipLaunchKernelGGL(k_pile_export, dim3(64, n_sel > 0 ? n_sel : 1), dim3(256), 0, c.stream,
                       P.dense, P.nflag, P.dflag, P.read_counts, P.first_unit, P.max_pos, P.cap,
                       P.n_refs, n_sel > 0 ? dsel : nullptr, n_sel, unit_base, (int32_t *)dev_sum,
                       (int32_t *)dev_max, (uint8_t *)dev_flags);
    MH_HIP(hipGetLastError());
    MH_HIP(hipStreamSynchronize(c.stream));
    return 0;
}

extern "C" int mh_pileup_import(mh_ctx *ctx, int n_sel, const int32_t *sel, const void *dev_sum,
                                const void *dev_max, const void *dev_flags)
{
    if (!ctx || !dev_sum || !dev_max || (n_sel > 0 && (!sel || !dev_flags))) return -3;
    Ctx &c = *reinterpret_cast<Ctx *>(ctx);
    PileState &P = c.pile;
    if (!P.dense) { set_error("no pileup to import into"); return -3; }
    MH_HIP(hipSetDevice(c.device));
    P.land_ok = false;   // the scalars change
    int32_t *dsel = nullptr;
    if (int st = upload_sel(c, n_sel, sel, &dsel)) return st;
    hipLaunchKernelGGL(k_pile_import, dim3(64, n_sel > 0 ? n_sel : 1), dim3(256), 0, c.stream,
                       P.dense, P.nflag, P.dflag, P.read_counts, P.first_unit, P.max_pos, P.cap,
                       P.n_refs, n_sel > 0 ? dsel : nullptr, n_sel, (const int32_t *)dev_sum,
                       (const int32_t *)dev_max, (const uint8_t *)dev_flags);
    MH_HIP(hipGetLastError());
    MH_HIP(hipStreamSynchronize(c.stream));
    return 0;
}

// ---------------------------------------------------------------------------
// Multi-GPU exchange of the raw insertion-token events (ref, pos, tok_off,
// tok_len) + their byte pool: each rank exports its events into a caller
// device buffer, the caller all-gathers the buffers (RCCL), and every rank
// imports the concatenation (rank order).  The token aggregation of
// mh_pileup_events then runs over every rank's events.  Nothing of the
// exchange goes through the host.
// ---------------------------------------------------------------------------
namespace mh {

__global__ void k_ev_rebase(int32_t *ev, int64_t first, int64_t n, int32_t pool_base)
{
    for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < n;
         e += (int64_t)gridDim.x * blockDim.x)
        ev[4 * (first + e) + 2] += pool_base;
}

}  // namespace mh

extern "C" int mh_pileup_event_bytes(mh_ctx *ctx, int64_t *n_events, int64_t *pool_bytes)
{
    if (!ctx) return -3;
    Ctx &c = *reinterpret_cast<Ctx *>(ctx);
    PileState &P = c.pile;
    int64_t ctr[4] = {0, 0, 0, 0};
    MH_HIP(hipSetDevice(c.device));
    if (P.ev_counters) MH_HIP(copy_sync(c, ctr, P.ev_counters, sizeof(ctr), hipMemcpyDeviceToHost));
    if (n_events) *n_events = ctr[0];
    if (pool_bytes) *pool_bytes = ctr[1];
    return 0;
}

extern "C" int mh_pileup_events_export(mh_ctx *ctx, void *dev_events, void *dev_pool)
{
    if (!ctx) return -3;
    Ctx &c = *reinterpret_cast<Ctx *>(ctx);
    PileState &P = c.pile;
    int64_t n = 0, bytes = 0;
    if (int st = mh_pileup_event_bytes(ctx, &n, &bytes)) return st;
    if ((n > 0 && !dev_events) || (bytes > 0 && !dev_pool)) return -3;
    if (n > 0) MH_HIP(hipMemcpyAsync(dev_events, P.ev, sizeof(int32_t) * 4 * n,
                                     hipMemcpyDeviceToDevice, c.stream));
    if (bytes > 0) MH_HIP(hipMemcpyAsync(dev_pool, P.ev_pool, bytes, hipMemcpyDeviceToDevice, c.stream));
    MH_HIP(hipStreamSynchronize(c.stream));
    return 0;
}

extern "C" int mh_pileup_events_import(mh_ctx *ctx, int parts, const int64_t *n_events,
                                       const int64_t *pool_bytes, const void *dev_events,
                                       int64_t events_stride, const void *dev_pool,
                                       int64_t pool_stride)
{
    if (!ctx || parts < 0 || (parts > 0 && (!n_events || !pool_bytes))) return -3;
    Ctx &c = *reinterpret_cast<Ctx *>(ctx);
    PileState &P = c.pile;
    int64_t tot_n = 0, tot_b = 0;
    for (int p = 0; p < parts; ++p) {
        if (n_events[p] < 0 || pool_bytes[p] < 0 || 4 * n_events[p] > events_stride ||
            pool_bytes[p] > pool_stride) { set_error("mh_pileup_events_import: bad part %d", p); return -3; }
        tot_n += n_events[p];
        tot_b += pool_bytes[p];
    }
    if ((tot_n > 0 && !dev_events) || (tot_b > 0 && !dev_pool)) return -3;
    if (tot_b >= INT32_MAX) { set_error("mh_pileup_events_import: pool too large"); return -2; }
    MH_HIP(hipSetDevice(c.device));
    if (P.ev_cap < tot_n || !P.ev) {
        hipFree(P.ev);
        P.ev_cap = tot_n * 2 + 1024;
        MH_HIP(hipMalloc(&P.ev, sizeof(int32_t) * 4 * P.ev_cap));
    }
    if (P.pool_cap < tot_b || !P.ev_pool) {
        hipFree(P.ev_pool);
        P.pool_cap = tot_b * 2 + 4096;
        MH_HIP(hipMalloc(&P.ev_pool, P.pool_cap));
    }
    if (!P.ev_counters) MH_HIP(hipMalloc(&P.ev_counters, sizeof(int64_t) * 4));
    int64_t at_n = 0, at_b = 0;
    for (int p = 0; p < parts; ++p) {
        const int32_t *src_e = (const int32_t *)dev_events + (size_t)p * events_stride;
        const char *src_b = (const char *)dev_pool + (size_t)p * pool_stride;
        if (n_events[p] > 0) {
            MH_HIP(hipMemcpyAsync(P.ev + 4 * at_n, src_e, sizeof(int32_t) * 4 * n_events[p],
                                  hipMemcpyDeviceToDevice, c.stream));
            if (at_b > 0) {
                int64_t blocks = (n_events[p] + 255) / 256;
                if (blocks > 4096) blocks = 4096;
                hipLaunchKernelGGL(k_ev_rebase, dim3((unsigned)blocks), dim3(256), 0, c.stream,
                                   P.ev, at_n, n_events[p], (int32_t)at_b);
                MH_HIP(hipGetLastError());
            }
        }
        if (pool_bytes[p] > 0)
            MH_HIP(hipMemcpyAsync(P.ev_pool + at_b, src_b, pool_bytes[p], hipMemcpyDeviceToDevice,
                                  c.stream));
        at_n += n_events[p];
        at_b += pool_bytes[p];
    }
    const int64_t ctr[4] = {tot_n, tot_b, 0, 0};
    MH_HIP(hipMemcpyAsync(P.ev_counters, ctr, sizeof(ctr), hipMemcpyHostToDevice, c.stream));
    MH_HIP(hipStreamSynchronize(c.stream));
    ++P.gen;   // the aggregated tokens are recomputed from the new events
    P.land_ok = false;   // ev_counters change
    return 0;
}
