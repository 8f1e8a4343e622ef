// mh_a2c.hip -- the per-read half of aln2counts (micall/core/aln2counts.py)
// on gfx950, over the rows of aligned.csv (sam2aln's distinct merged reads
// with their counts) resident in HBM.
//
//   k_a2c_count   SequenceReport._count_reads (:115-172) with
//                 SeedAmino.count_aminos / SeedNucleotide.count_nucleotides
//                 (:595-606, :636-645).  Work unit: a chunk of <= 1024 rows of
//                 one bin; a bin is 21 consecutive codons of one (refname,
//                 qcut) group.  A wave takes a row, lane 21 f + c codon c of
//                 the bin in reading frame f (63 lanes: the three frames read
//                 the same bytes in one load instruction, so every row is
//                 fetched once per bin, not once per frame): the three
//                 characters of the frame- and
//                 offset-padded read ('-' outside it, :155-157), the amino
//                 acid from the codon table, then LDS counters per (codon,
//                 amino acid) and per (codon, position, base): a count and
//                 the first row that touched it.  The first row is the
//                 Counter insertion order that most_common() breaks ties by
//                 (:624, :668).  One global atomic per touched counter
//                 flushes the chunk.
//   k_a2c_ins_*   the read loop of InsertionWriter.write (:786-795): per
//                 (insert range, row) the framed slice [3 left, 3 right) of
//                 the read, rejected when it starts in the padding, holds '-'
//                 or 'n' or no whole codon, and translated; equal amino-acid
//                 strings of one range are grouped in an open-addressing
//                 table (count, first row), every member is compared with
//                 its group's first row (a collision is an error, never a
//                 merge) and the distinct strings are gathered for the host.
// Host half (below the kernels): aligned.csv as csv.DictReader reads it,
// consecutive (refname, qcut) groups (itertools.groupby, :884-887), the
// codon extent of every frame, the bin lists.
// Bit-for-bit specification: oracle/og_aln2counts.py.
#include <algorithm>
#include <charconv>
#include <chrono>
#include <cstring>
#include <deque>
#include <map>
#include <functional>
#include <string>
#include <thread>
#include <unordered_map>
#include <vector>

#include "mh_gunzip.h"
#include "mh_internal.h"
#include "mh_sam2aln.h"
#include "mh_text.h"

namespace mh {

constexpr int A2C_W = 21;                       // codons per bin (x 3 frames = 63 lanes)
constexpr int A2C_LANES = 3 * A2C_W;
constexpr int A2C_CHUNK = 1024;                 // rows per workgroup
constexpr int A2C_NAA = 21;                     // AMINO_ALPHABET
constexpr int A2C_STRIDE = A2C_NAA + 18;        // per codon: 21 amino acids, 3 x 6 bases
constexpr int A2C_CELLS = A2C_LANES * A2C_STRIDE;   // counters per bin (3 frames)
constexpr int A2C_SLOTS = 4;
constexpr uint32_t A2C_NONE = 0xffffffffu;
constexpr int64_t A2C_MAX_SPAN = 1 << 28;
// Read characters: A C G T N - are classes 0-5; 'n' (the gap between the
// mates: no base, an 'N' to translate, :642-645) is 6; anything else is 7.
enum { A2C_DASH = 5, A2C_GAP = 6, A2C_BAD = 7 };
static const char A2C_CODES[] = "ACDEFGHIKLMNPQRSTVWY*?-";   // amino-acid codes 0..22
__constant__ char c_a2c_codes[24] = "ACDEFGHIKLMNPQRSTVWY*?-";

struct A2CRow {
    int64_t soff;      // first seq byte in the uploaded text
    int32_t len;       // seq length
    int32_t off;       // offset column
    uint32_t cnt;      // count column
    uint32_t local;    // row index within its group
};

struct A2CChunk {
    int32_t bin, codon0;
    int64_t beg, end;  // slice of bin_rows
};

struct A2CEntry {
    int32_t range;
    uint32_t first;
    int32_t n_codons;
    int32_t lo;        // slice start in the first row
    unsigned long long count;
};

struct A2CState {
    // host
    int64_t n_rows = 0, n_bins = 0;
    std::vector<A2CRow> rows;
    std::vector<int64_t> g_first;             // n_groups + 1
    std::vector<std::string> g_ref, g_qcut;
    std::vector<int32_t> g_ncod;              // 3 per group
    std::vector<int64_t> g_bin0;              // n_groups + 1
    std::vector<uint32_t> h_cnt, h_first;     // [bin][frame * 21 + codon][39]
    int8_t code[512];
    uint8_t cls[256];
    std::string pool;                         // row text when it is not the caller's CSV
    // device
    uint8_t *d_text = nullptr, *d_cls = nullptr;
    int8_t *d_code = nullptr;
    A2CRow *d_rows = nullptr;
    int32_t *d_bin_rows = nullptr;
    A2CChunk *d_chunks = nullptr;
    uint32_t *d_cnt = nullptr, *d_first = nullptr;
    // insertion strings of the last mh_a2c_inserts, in (range, first row) order
    std::vector<A2CEntry> entries;
    std::string aminos;                       // one line per entry
    std::string ins_rows;                     // mh_a2c_insert_rows text (size query, then copy)
    std::unordered_map<const void *, size_t> dcap;   // bytes behind each device pointer (grow-only)
    double t_parse = 0, t_count = 0, t_ins = 0;
    // a part of aligned.csv held between mh_a2c_part_open and _count (mapped)
    const char *part_text = nullptr;          // (null for an empty file)
    size_t part_len = 0;
    bool part_open = false;                   // mh_a2c_part_open done, not counted yet
    int64_t part_b0 = 0, part_b1 = 0;         // the part's bytes of the text
    std::vector<int64_t> part_first;          // local groups' first rows (+ end)
};

// ---------------------------------------------------------------------------
// device
// ---------------------------------------------------------------------------
struct A2CCountArgs {
    const uint8_t *text;
    const A2CRow *rows;
    const int32_t *bin_rows;
    const A2CChunk *chunks;
    const int8_t *code;   // 512: codon of classes (c0, c1, c2) at 64 c0 + 8 c1 + c2
    const uint8_t *cls;   // 256
    uint32_t *cnt, *first;
};

__global__ __launch_bounds__(256) void k_a2c_count(A2CCountArgs A)
{
    __shared__ uint32_t s_cnt[A2C_CELLS], s_first[A2C_CELLS];
    __shared__ int8_t s_code[512];
    __shared__ uint8_t s_cls[256];
    const A2CChunk ch = A.chunks[blockIdx.x];
    for (int i = threadIdx.x; i < A2C_CELLS; i += 256) {
        s_cnt[i] = 0;
        s_first[i] = A2C_NONE;
    }
    s_code[threadIdx.x] = A.code[threadIdx.x];
    s_code[threadIdx.x + 256] = A.code[threadIdx.x + 256];
    s_cls[threadIdx.x] = A.cls[threadIdx.x];
    __syncthreads();
    const int lane = threadIdx.x & 63;
    const int f = lane / A2C_W;                  // this lane's frame and codon
    const int j = ch.codon0 + lane - A2C_W * f;
    // lane stride 39 words: odd, so the lanes of a wave hit distinct banks
    uint32_t *cc = s_cnt + lane * A2C_STRIDE, *cf = s_first + lane * A2C_STRIDE;
    for (int64_t i = ch.beg + (threadIdx.x >> 6); i < ch.end; i += 4) {
        if (lane >= A2C_LANES) continue;
        const A2CRow R = A.rows[A.bin_rows[i]];
        // codons offset // 3 .. ceil((frame + offset + len) / 3) - 1 (:155-160)
        if (j < R.off / 3 || j >= (f + R.off + R.len + 2) / 3) continue;
        const int q0 = 3 * j - f - R.off;
        const uint8_t *s = A.text + R.soff;
        int c[3];
#pragma unroll
        for (int t = 0; t < 3; ++t) {
            const int q = q0 + t;
            c[t] = (q >= 0 && q < R.len) ? s_cls[s[q]] : A2C_DASH;
        }
        const int a = s_code[64 * c[0] + 8 * c[1] + c[2]];
        if (a < A2C_NAA) {
            atomicAdd(&cc[a], R.cnt);
            atomicMin(&cf[a], R.local);
        }
#pragma unroll
        for (int t = 0; t < 3; ++t)
            if (c[t] < A2C_GAP) {
                const int k = A2C_NAA + 6 * t + c[t];
                atomicAdd(&cc[k], R.cnt);
                atomicMin(&cf[k], R.local);
            }
    }
    __syncthreads();
    const size_t base = (size_t)ch.bin * A2C_CELLS;
    for (int i = threadIdx.x; i < A2C_CELLS; i += 256) {
        const uint32_t fr = s_first[i];
        if (fr == A2C_NONE) continue;
        if (s_cnt[i]) atomicAdd(&A.cnt[base + i], s_cnt[i]);
        atomicMin(&A.first[base + i], fr);
    }
}

struct A2CInsArgs {
    const uint8_t *text;
    const A2CRow *rows;      // the rows of one group
    uint32_t row0;           // rows[0].local: a first-row number minus row0 indexes rows
                             // (a rank's part of a group starts at the ranks before's rows)
    const int8_t *code;
    const uint8_t *cls;
    const int32_t *left, *right;
    int64_t n_rows, n_pairs;
    int frame;
    uint64_t *h;             // per (range, row): 0 = no insertion string
    uint64_t *tkey;
    unsigned long long *tcnt;
    uint32_t *tfirst;
    int32_t *trange;
    uint64_t mask;
    A2CEntry *entries;
    unsigned long long *ctr; // [0] strings, [1] collisions, [2] entries
};

// The framed slice of one read for one range (:787-791): read indices
// [lo, lo + 3 n) of its whole codons, or false when the slice starts in the
// '-' padding, is empty, holds '-' or 'n', or translates to nothing.
__device__ bool a2c_slice(const A2CInsArgs &A, const A2CRow &R, int rg, int &lo, int &n)
{
    const int64_t s = 3LL * A.left[rg] - A.frame - R.off;
    int64_t e = 3LL * A.right[rg] - A.frame - R.off;
    if (e > R.len) e = R.len;
    if (s < 0 || e - s < 3) return false;
    const uint8_t *p = A.text + R.soff;
    for (int64_t q = s; q < e; ++q) {
        const uint8_t c = A.cls[p[q]];
        if (c == A2C_DASH || c == A2C_GAP) return false;
    }
    lo = (int)s;
    n = (int)((e - s) / 3);
    return true;
}

__device__ __forceinline__ int a2c_codon(const A2CInsArgs &A, const uint8_t *p, int q)
{
    return A.code[64 * A.cls[p[q]] + 8 * A.cls[p[q + 1]] + A.cls[p[q + 2]]];
}

__device__ __forceinline__ uint64_t a2c_mix(uint64_t z)
{
    z += 0x9e3779b97f4a7c15ull;
    z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
    z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
    return z ^ (z >> 31);
}

__device__ __forceinline__ int64_t a2c_find(const A2CInsArgs &A, uint64_t h)
{
    uint64_t s = (h >> 7) & A.mask;
    while (A.tkey[s] != h) s = (s + 1) & A.mask;
    return (int64_t)s;
}

__global__ __launch_bounds__(256) void k_a2c_ins_hash(A2CInsArgs A)
{
    const int64_t p = (int64_t)blockIdx.x * 256 + threadIdx.x;
    bool ok = false;
    if (p < A.n_pairs) {
        const int rg = (int)(p / A.n_rows);
        const A2CRow R = A.rows[p % A.n_rows];
        int lo, n;
        uint64_t h = 0;
        if (a2c_slice(A, R, rg, lo, n)) {
            const uint8_t *s = A.text + R.soff;
            h = a2c_mix(0x243f6a8885a308d3ull + (uint64_t)rg);
            for (int k = 0; k < n; ++k) h = a2c_mix(h ^ (uint64_t)(a2c_codon(A, s, lo + 3 * k) + 1));
            h = a2c_mix(h ^ ((uint64_t)n << 32)) | 1ull;
            ok = true;
        }
        A.h[p] = h;
    }
    const unsigned long long b = __ballot(ok);
    if ((threadIdx.x & 63) == 0 && b) atomicAdd(&A.ctr[0], (unsigned long long)__popcll(b));
}

__global__ __launch_bounds__(256) void k_a2c_ins_count(A2CInsArgs A)
{
    const int64_t p = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (p >= A.n_pairs) return;
    const uint64_t h = A.h[p];
    if (!h) return;
    const A2CRow R = A.rows[p % A.n_rows];
    uint64_t s = (h >> 7) & A.mask;
    for (;;) {
        const unsigned long long old =
            atomicCAS((unsigned long long *)&A.tkey[s], 0ull, (unsigned long long)h);
        if (old == 0ull || old == h) {
            if (old == 0ull) A.trange[s] = (int32_t)(p / A.n_rows);
            atomicAdd(&A.tcnt[s], (unsigned long long)R.cnt);
            atomicMin(&A.tfirst[s], R.local);
            return;
        }
        s = (s + 1) & A.mask;
    }
}

__global__ __launch_bounds__(256) void k_a2c_ins_verify(A2CInsArgs A)
{
    const int64_t p = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (p >= A.n_pairs) return;
    const uint64_t h = A.h[p];
    if (!h) return;
    const int rg = (int)(p / A.n_rows);
    const int64_t s = a2c_find(A, h);
    const A2CRow R = A.rows[p % A.n_rows], F = A.rows[A.tfirst[s] - A.row0];
    int lo = 0, n = 0, flo = 0, fn = 0;
    bool same = A.trange[s] == rg && a2c_slice(A, R, rg, lo, n) && a2c_slice(A, F, rg, flo, fn) &&
                n == fn;
    const uint8_t *pr = A.text + R.soff, *pf = A.text + F.soff;
    for (int k = 0; same && k < n; ++k)
        same = a2c_codon(A, pr, lo + 3 * k) == a2c_codon(A, pf, flo + 3 * k);
    if (!same) atomicAdd(&A.ctr[1], 1ull);
}

__global__ __launch_bounds__(256) void k_a2c_ins_compact(A2CInsArgs A)
{
    const uint64_t s = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    if (s > A.mask || !A.tkey[s]) return;
    A2CEntry e;
    e.range = A.trange[s];
    e.first = A.tfirst[s];
    e.count = A.tcnt[s];
    int lo = 0, n = 0;
    a2c_slice(A, A.rows[e.first - A.row0], e.range, lo, n);
    e.lo = lo;
    e.n_codons = n;
    A.entries[atomicAdd(&A.ctr[2], 1ull)] = e;
}

// amino-acid strings of the (sorted) entries, each followed by '\n'
__global__ __launch_bounds__(256) void k_a2c_ins_gather(A2CInsArgs A, const A2CEntry *ent,
                                                        const int64_t *eoff, int64_t n_ent,
                                                        char *out)
{
    const int64_t k = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (k >= n_ent) return;
    const A2CEntry e = ent[k];
    const uint8_t *s = A.text + A.rows[e.first - A.row0].soff;
    char *o = out + eoff[k];
    for (int c = 0; c < e.n_codons; ++c) o[c] = c_a2c_codes[a2c_codon(A, s, e.lo + 3 * c)];
    o[e.n_codons] = '\n';
}

// ---------------------------------------------------------------------------
// host
// ---------------------------------------------------------------------------
static void a2c_free_device(A2CState &S)
{
    hipFree(S.d_text); hipFree(S.d_cls); hipFree(S.d_code); hipFree(S.d_rows);
    hipFree(S.d_bin_rows); hipFree(S.d_chunks); hipFree(S.d_cnt); hipFree(S.d_first);
    S.d_text = S.d_cls = nullptr;
    S.d_code = nullptr;
    S.d_rows = nullptr;
    S.d_bin_rows = nullptr;
    S.d_chunks = nullptr;
    S.d_cnt = S.d_first = nullptr;
    S.dcap.clear();
}

static void a2c_parallel_for(int nt, const std::function<void(int)> &fn)
{
    if (nt <= 1) { fn(0); return; }
    std::vector<std::thread> th;
    for (int t = 1; t < nt; ++t) th.emplace_back(fn, t);
    fn(0);
    for (auto &x : th) x.join();
}

// byte classes and the codon table from the caller's translations of the 216
// codons over A C G T N - (micall_amd/translation.py codon_chars)
static int a2c_tables(A2CState &S, const char *codon_chars)
{
    if (!codon_chars || strlen(codon_chars) != 216) {
        set_error("aln2counts: codon_chars must hold 216 translations");
        return -3;
    }
    memset(S.cls, A2C_BAD, sizeof(S.cls));
    const char *alpha = "ACGTN-";
    for (int k = 0; k < 6; ++k) S.cls[(uint8_t)alpha[k]] = (uint8_t)k;
    S.cls[(uint8_t)'n'] = A2C_GAP;
    for (int c0 = 0; c0 < 8; ++c0)
        for (int c1 = 0; c1 < 8; ++c1)
            for (int c2 = 0; c2 < 8; ++c2) {
                // count_aminos upper-cases the codon: 'n' translates as 'N'
                const int m0 = c0 == A2C_GAP ? 4 : c0, m1 = c1 == A2C_GAP ? 4 : c1,
                          m2 = c2 == A2C_GAP ? 4 : c2;
                int8_t v = 22;
                if (m0 < 6 && m1 < 6 && m2 < 6) {
                    const char ch = codon_chars[36 * m0 + 6 * m1 + m2];
                    const char *hit = ch ? strchr(A2C_CODES, ch) : nullptr;
                    if (!hit) {
                        set_error("aln2counts: codon translation '%c' is not an amino-acid code", ch);
                        return -3;
                    }
                    v = (int8_t)(hit - A2C_CODES);
                }
                S.code[64 * c0 + 8 * c1 + c2] = v;
            }
    return 0;
}

// Python int() on a CSV field (surrounding whitespace, one sign)
static bool a2c_int(const char *a, const char *b, int64_t &v)
{
    while (a < b && (*a == ' ' || *a == '\t' || *a == '\r' || *a == '\n' || *a == '\f' || *a == '\v')) ++a;
    while (b > a && (b[-1] == ' ' || b[-1] == '\t' || b[-1] == '\r' || b[-1] == '\n' ||
                     b[-1] == '\f' || b[-1] == '\v')) --b;
    bool neg = false;
    if (a < b && (*a == '+' || *a == '-')) { neg = *a == '-'; ++a; }
    if (a == b) return false;
    long long x = 0;
    auto r = std::from_chars(a, b, x);
    if (r.ec != std::errc() || r.ptr != b) return false;
    v = neg ? -x : x;
    return true;
}

struct A2CKey {
    const char *p;
    int32_t n;
};

struct A2CPart {
    const char *beg, *end;
    std::vector<A2CRow> rows;
    std::vector<A2CKey> kref, kqcut;
    std::deque<std::string> pool;      // unquoted keys and seqs (quoted input only)
    int64_t err_row = -1;
    std::string err;
};

enum { COL_REF, COL_QCUT, COL_COUNT, COL_OFFSET, COL_SEQ, N_COLS };

// One data row into P (fields as [begin, end) views); false on an error.
static bool a2c_row(A2CPart &P, const char *const *fb, const char *const *fe, const int *col,
                    const char *base, const uint8_t *cls)
{
    int64_t cnt = 0, off = 0;
    if (!a2c_int(fb[col[COL_COUNT]], fe[col[COL_COUNT]], cnt)) {
        P.err = "invalid literal for int() with base 10 in column count";
        return false;
    }
    if (!a2c_int(fb[col[COL_OFFSET]], fe[col[COL_OFFSET]], off)) {
        P.err = "invalid literal for int() with base 10 in column offset";
        return false;
    }
    if (cnt < 0 || cnt > (int64_t)UINT32_MAX) { P.err = "count outside 0 .. 2**32-1"; return false; }
    if (off < 0 || off > A2C_MAX_SPAN) { P.err = "offset outside 0 .. 2**28"; return false; }
    const char *sb = fb[col[COL_SEQ]], *se = fe[col[COL_SEQ]];
    if (se - sb > A2C_MAX_SPAN) { P.err = "seq longer than 2**28"; return false; }
    for (const char *c = sb; c < se; ++c)
        if (cls[(uint8_t)*c] == A2C_BAD) {
            P.err = std::string("character '") + *c + "' in seq is not one of A C G T N - n";
            return false;
        }
    A2CRow R;
    R.soff = sb - base;
    R.len = (int32_t)(se - sb);
    R.off = (int32_t)off;
    R.cnt = (uint32_t)cnt;
    R.local = 0;
    P.rows.push_back(R);
    P.kref.push_back({fb[col[COL_REF]], (int32_t)(fe[col[COL_REF]] - fb[col[COL_REF]])});
    P.kqcut.push_back({fb[col[COL_QCUT]], (int32_t)(fe[col[COL_QCUT]] - fb[col[COL_QCUT]])});
    return true;
}

// unquoted text: every field is a view into the text
static void a2c_parse_part(A2CPart &P, const int *col, int need, const char *base,
                           const uint8_t *cls)
{
    std::vector<const char *> fb(need), fe(need);
    const char *p = P.beg;
    int64_t row = 0;
    while (p < P.end) {
        int nf = 0;
        const char *s = p;
        for (;;) {
            const char *q = s;
            while (q < P.end && *q != ',' && *q != '\n' && *q != '\r') ++q;
            if (nf < need) { fb[nf] = s; fe[nf] = q; }
            ++nf;
            if (q < P.end && *q == ',') { s = q + 1; continue; }
            if (q < P.end && *q == '\r') ++q;
            if (q < P.end && *q == '\n') ++q;
            p = q;
            break;
        }
        if (nf == 1 && fb[0] == fe[0]) continue;             // blank line: DictReader skips it
        if (nf < need) { P.err_row = row; P.err = "row has fewer fields than the header"; return; }
        if (!a2c_row(P, fb.data(), fe.data(), col, base, cls)) { P.err_row = row; return; }
        ++row;
    }
}

// quoted text (rare): fields unescaped into P.pool; seqs are copied too, so
// the rows point into the state's pool instead of the caller's text
static void a2c_parse_quoted(A2CPart &P, const int *col, int need, const uint8_t *cls,
                             std::string &seqpool)
{
    std::vector<std::string> f;
    std::vector<const char *> fb(need), fe(need);
    const char *p = P.beg;
    int64_t row = 0;
    std::vector<size_t> seq_at;
    while (p < P.end) {
        csv_record(p, P.end, f);
        if (f.size() == 1 && f[0].empty()) continue;
        if ((int)f.size() < need) { P.err_row = row; P.err = "row has fewer fields than the header"; return; }
        for (int k = 0; k < need; ++k) {
            P.pool.push_back(f[k]);
            fb[k] = P.pool.back().data();
            fe[k] = fb[k] + P.pool.back().size();
        }
        const std::string &sq = f[col[COL_SEQ]];
        seq_at.push_back(seqpool.size());
        seqpool.append(sq);
        if (!a2c_row(P, fb.data(), fe.data(), col, fb[col[COL_SEQ]], cls)) { P.err_row = row; return; }
        P.rows.back().soff = (int64_t)seq_at.back();
        ++row;
    }
}

// Per-group codon extents, bins, bin row lists and chunks.
// preset: g_ncod and every row's `local` were set by the caller (a part of
// a sharded job: the job's codon extents and row numbers within the group)
static int a2c_layout(A2CState &S, std::vector<int32_t> &bin_rows, std::vector<A2CChunk> &chunks,
                      bool preset = false)
{
    const int64_t ng = (int64_t)S.g_first.size() - 1;
    if (!preset) S.g_ncod.assign(3 * ng, 0);
    S.g_bin0.assign(ng + 1, 0);
    if (S.n_rows >= INT32_MAX) { set_error("aln2counts: more than 2**31 rows"); return -3; }
    for (int64_t g = 0; g < ng; ++g) {
        int32_t *nc = &S.g_ncod[3 * g];
        if (preset) {
            const int top = std::max(nc[0], std::max(nc[1], nc[2]));
            S.g_bin0[g + 1] = S.g_bin0[g] + (top + A2C_W - 1) / A2C_W;
            continue;
        }
        uint64_t total = 0;
        for (int64_t r = S.g_first[g]; r < S.g_first[g + 1]; ++r) {
            A2CRow &R = S.rows[r];
            R.local = (uint32_t)(r - S.g_first[g]);
            total += R.cnt;
            const int lo = R.off / 3;
            for (int f = 0; f < 3; ++f) {
                const int hi = (f + R.off + R.len + 2) / 3;
                if (hi > lo && hi > nc[f]) nc[f] = hi;
            }
        }
        if (total > UINT32_MAX) {
            set_error("aln2counts: the counts of group %lld add up to more than 2**32-1", (long long)g);
            return -3;
        }
        const int top = std::max(nc[0], std::max(nc[1], nc[2]));
        S.g_bin0[g + 1] = S.g_bin0[g] + (top + A2C_W - 1) / A2C_W;
    }
    S.n_bins = S.g_bin0[ng];
    std::vector<int64_t> start(S.n_bins + 1, 0);
    for (int64_t g = 0; g < ng; ++g)
        for (int64_t r = S.g_first[g]; r < S.g_first[g + 1]; ++r) {
            const A2CRow &R = S.rows[r];
            const int64_t b0 = S.g_bin0[g] + (R.off / 3) / A2C_W;
            const int64_t b1 = S.g_bin0[g] + ((2 + R.off + R.len + 2) / 3 - 1) / A2C_W;
            for (int64_t b = b0; b <= b1; ++b) ++start[b + 1];
        }
    for (int64_t b = 0; b < S.n_bins; ++b) start[b + 1] += start[b];
    bin_rows.assign(start[S.n_bins], 0);
    std::vector<int64_t> cur(start.begin(), start.end() - 1);
    for (int64_t g = 0; g < ng; ++g)
        for (int64_t r = S.g_first[g]; r < S.g_first[g + 1]; ++r) {
            const A2CRow &R = S.rows[r];
            const int64_t b0 = S.g_bin0[g] + (R.off / 3) / A2C_W;
            const int64_t b1 = S.g_bin0[g] + ((2 + R.off + R.len + 2) / 3 - 1) / A2C_W;
            for (int64_t b = b0; b <= b1; ++b) bin_rows[cur[b]++] = (int32_t)r;
        }
    chunks.clear();
    for (int64_t g = 0; g < ng; ++g)
        for (int64_t b = S.g_bin0[g]; b < S.g_bin0[g + 1]; ++b)
            for (int64_t i = start[b]; i < start[b + 1]; i += A2C_CHUNK)
                chunks.push_back({(int32_t)b, (int32_t)((b - S.g_bin0[g]) * A2C_W), i,
                                  std::min<int64_t>(i + A2C_CHUNK, start[b + 1])});
    return 0;
}

template <class T>
static int a2c_reserve(A2CState &S, T *&p, size_t bytes)
{
    // kept between calls, reallocated only to grow (hipFree waits for the device)
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
static int a2c_upload(A2CState &S, T *&dst, const T *src, size_t n, hipStream_t s)
{
    if (int st = a2c_reserve(S, dst, sizeof(T) * n)) return st;
    if (n) MH_HIP(hipMemcpyAsync(dst, src, sizeof(T) * n, hipMemcpyHostToDevice, s));
    return 0;
}

// upload the rows, count every group on the device, fetch the counters
static int a2c_count(Ctx &c, A2CState &S, const char *text, int64_t text_len, bool preset = false)
{
    std::vector<int32_t> bin_rows;
    std::vector<A2CChunk> chunks;
    if (int st = a2c_layout(S, bin_rows, chunks, preset)) return st;
    hipStream_t s = c.stream;
    if (int st = a2c_upload(S, S.d_text, (const uint8_t *)text, (size_t)text_len, s)) return st;
    if (int st = a2c_upload(S, S.d_rows, S.rows.data(), S.rows.size(), s)) return st;
    if (int st = a2c_upload(S, S.d_bin_rows, bin_rows.data(), bin_rows.size(), s)) return st;
    if (int st = a2c_upload(S, S.d_chunks, chunks.data(), chunks.size(), s)) return st;
    if (int st = a2c_upload(S, S.d_code, S.code, 512, s)) return st;
    if (int st = a2c_upload(S, S.d_cls, S.cls, 256, s)) return st;
    const size_t cells = (size_t)S.n_bins * A2C_CELLS;
    if (int st = a2c_reserve(S, S.d_cnt, sizeof(uint32_t) * cells)) return st;
    if (int st = a2c_reserve(S, S.d_first, sizeof(uint32_t) * cells)) return st;
    if (cells) {
        MH_HIP(hipMemsetAsync(S.d_cnt, 0, sizeof(uint32_t) * cells, s));
        MH_HIP(hipMemsetAsync(S.d_first, 0xff, sizeof(uint32_t) * cells, s));
    }
    if (!chunks.empty()) {
        A2CCountArgs a{S.d_text, S.d_rows, S.d_bin_rows, S.d_chunks, S.d_code, S.d_cls,
                       S.d_cnt, S.d_first};
        const int p0 = prof_begin(c, "k_a2c_count");
        hipLaunchKernelGGL(k_a2c_count, dim3((unsigned)chunks.size()), dim3(256), 0, s, a);
        prof_end(c, p0);
        MH_HIP(hipGetLastError());
    }
    S.h_cnt.resize(cells);
    S.h_first.resize(cells);
    if (cells) {
        MH_HIP(hipMemcpyAsync(S.h_cnt.data(), S.d_cnt, sizeof(uint32_t) * cells,
                              hipMemcpyDeviceToHost, s));
        MH_HIP(hipMemcpyAsync(S.h_first.data(), S.d_first, sizeof(uint32_t) * cells,
                              hipMemcpyDeviceToHost, s));
    }
    MH_HIP(hipStreamSynchronize(s));
    prof_flush(c);
    return 0;
}

static int a2c_parse_csv(A2CState &S, const char *text, int64_t len, bool &use_pool,
                         int64_t body_lo = -1, int64_t body_hi = -1)
{
    const char *p = text, *end = text + len;
    std::vector<std::string> head;
    S.rows.clear();
    S.g_first.assign(1, 0);
    S.g_ref.clear();
    S.g_qcut.clear();
    S.pool.clear();
    use_pool = false;
    if (!csv_record(p, end, head)) return 0;             // empty file: no rows
    if (body_lo >= 0) {      // one part of the body: the records of [body_lo, body_hi)
        p = text + std::max<int64_t>(body_lo, p - text);
        end = text + std::max<int64_t>(body_hi, p - text);
    }
    static const char *const want[N_COLS] = {"refname", "qcut", "count", "offset", "seq"};
    int col[N_COLS];
    int need = 0;
    for (int k = 0; k < N_COLS; ++k) {
        col[k] = -1;
        for (size_t z = 0; z < head.size(); ++z)
            if (head[z] == want[k]) col[k] = (int)z;     // DictReader: the last duplicate wins
        need = std::max(need, col[k] + 1);
    }
    const int64_t body = end - p;
    const bool quoted = memchr(p, '"', (size_t)body) != nullptr;
    for (int k = 0; k < N_COLS; ++k)
        if (col[k] < 0) {
            // DictReader only fails when a row is read: row['refname'] -> KeyError
            const char *q = p;
            while (q < end && (*q == '\n' || *q == '\r')) ++q;
            if (q == end) return 0;
            set_error("aligned csv: KeyError: '%s'", want[k]);
            return -3;
        }
    int nt = quoted ? 1 : s2a_threads();
    if (body < (int64_t)nt * (1 << 20)) nt = (int)std::max<int64_t>(1, body >> 20);
    std::vector<A2CPart> parts(nt);
    for (int t = 0; t < nt; ++t) {
        const char *c0 = p + body * t / nt;
        if (t) {
            while (c0 < end && *c0 != '\n') ++c0;
            if (c0 < end) ++c0;
        }
        parts[t].beg = c0;
    }
    for (int t = 0; t < nt; ++t) {
        parts[t].end = t + 1 < nt ? parts[t + 1].beg : end;
        if (parts[t].end < parts[t].beg) parts[t].end = parts[t].beg;
    }
    if (quoted) {
        use_pool = true;
        a2c_parse_quoted(parts[0], col, need, S.cls, S.pool);
    } else {
        a2c_parallel_for(nt, [&](int t) { a2c_parse_part(parts[t], col, need, text, S.cls); });
    }
    int64_t base = 0;
    for (auto &P : parts) {
        if (P.err_row >= 0) {
            set_error("aligned csv row %lld: %s", (long long)(base + P.err_row + 1), P.err.c_str());
            return -3;
        }
        base += (int64_t)P.rows.size();
    }
    S.n_rows = base;
    S.rows.resize(base);
    int64_t o = 0;
    A2CKey pr{nullptr, -1}, pq{nullptr, -1};
    for (auto &P : parts) {
        memcpy(S.rows.data() + o, P.rows.data(), sizeof(A2CRow) * P.rows.size());
        for (size_t i = 0; i < P.rows.size(); ++i) {
            const A2CKey &kr = P.kref[i], &kq = P.kqcut[i];
            const bool same = kr.n == pr.n && kq.n == pq.n && !memcmp(kr.p, pr.p, kr.n) &&
                              !memcmp(kq.p, pq.p, kq.n);
            if (!same) {
                if (o + (int64_t)i > 0) S.g_first.push_back(o + (int64_t)i);
                S.g_ref.emplace_back(kr.p, kr.n);
                S.g_qcut.emplace_back(kq.p, kq.n);
                pr = kr;
                pq = kq;
            }
        }
        o += (int64_t)P.rows.size();
    }
    if (S.n_rows) S.g_first.push_back(S.n_rows);
    // the key views of the last part may point into its pool: the group
    // names were copied above, so the parts can go
    return 0;
}

static A2CState *a2c_state(Ctx &c, int slot)
{
    if (!c.a2c) c.a2c = new A2CState *[A2C_SLOTS]();
    if (!c.a2c[slot]) c.a2c[slot] = new A2CState();
    return c.a2c[slot];
}

void a2c_free(Ctx &c)
{
    if (!c.a2c) return;
    for (int k = 0; k < A2C_SLOTS; ++k)
        if (c.a2c[k]) {
            if (c.a2c[k]->part_text) unmap_text_file(c.a2c[k]->part_text, c.a2c[k]->part_len);
            a2c_free_device(*c.a2c[k]);
            delete c.a2c[k];
        }
    delete[] c.a2c;
    c.a2c = nullptr;
}

static void a2c_clear_inserts(A2CState &S)
{
    S.entries.clear();
    S.aminos.clear();
}

}  // namespace mh

using namespace mh;

static double ms_since(std::chrono::steady_clock::time_point t0)
{
    return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
}

extern "C" int mh_a2c_load_csv(mh_ctx *ctx, int slot, const char *text, int64_t len,
                               const char *codon_chars, int64_t *n_groups)
{
    if (!ctx || slot < 0 || slot >= A2C_SLOTS || (!text && len) || len < 0) return -3;
    Ctx &c = *ctx_of(ctx);
    MH_HIP(hipSetDevice(c.device));
    A2CState &S = *a2c_state(c, slot);
    a2c_clear_inserts(S);
    if (S.part_text) {       // a part left open by a sharded load that fell back
        unmap_text_file(S.part_text, S.part_len);
        S.part_text = nullptr;
        S.part_open = false;
    }
    auto t0 = std::chrono::steady_clock::now();
    if (int st = a2c_tables(S, codon_chars)) return st;
    bool use_pool = false;
    if (int st = a2c_parse_csv(S, text ? text : "", len, use_pool)) {
        S.rows.clear();
        S.g_first.assign(1, 0);
        return st;
    }
    S.t_parse = ms_since(t0);
    auto t1 = std::chrono::steady_clock::now();
    const int st = use_pool ? a2c_count(c, S, S.pool.data(), (int64_t)S.pool.size())
                            : a2c_count(c, S, text ? text : "", len);
    if (st) {
        S.rows.clear();
        S.g_first.assign(1, 0);
        return st;
    }
    S.t_count = ms_since(t1);
    if (n_groups) *n_groups = (int64_t)S.g_first.size() - 1;
    return 0;
}

extern "C" int mh_a2c_load_file(mh_ctx *ctx, int slot, int fd, const char *codon_chars, int64_t *n_groups)
{
    if (!ctx || fd < 0) return -3;
    const char *text = nullptr;
    size_t len = 0;
    if (int st = map_text_file(fd, &text, &len)) return st;
    const int rc = mh_a2c_load_csv(ctx, slot, text, (int64_t)len, codon_chars, n_groups);
    unmap_text_file(text, len);
    return rc;
}

extern "C" int mh_a2c_load_rows(mh_ctx *ctx, int slot, int64_t n_rows, const char *pool,
                                int64_t pool_len, const int64_t *seq_off, const int32_t *seq_len,
                                const int64_t *offset, const int64_t *count, int64_t n_groups,
                                const int64_t *group_first, const char *codon_chars)
{
    if (!ctx || slot < 0 || slot >= A2C_SLOTS || n_rows < 0 || pool_len < 0 || n_groups < 0 ||
        (n_rows && (!pool || !seq_off || !seq_len || !offset || !count)) || !group_first)
        return -3;
    Ctx &c = *ctx_of(ctx);
    MH_HIP(hipSetDevice(c.device));
    A2CState &S = *a2c_state(c, slot);
    a2c_clear_inserts(S);
    auto t0 = std::chrono::steady_clock::now();
    if (int st = a2c_tables(S, codon_chars)) return st;
    if (group_first[0] != 0 || group_first[n_groups] != n_rows) {
        set_error("mh_a2c_load_rows: group_first must run from 0 to n_rows");
        return -3;
    }
    S.rows.assign(n_rows, A2CRow{});
    for (int64_t r = 0; r < n_rows; ++r) {
        if (seq_off[r] < 0 || seq_len[r] < 0 || seq_off[r] + seq_len[r] > pool_len ||
            seq_len[r] > A2C_MAX_SPAN) {
            set_error("mh_a2c_load_rows: row %lld: seq outside the pool", (long long)r);
            return -3;
        }
        if (count[r] < 0 || count[r] > (int64_t)UINT32_MAX) {
            set_error("mh_a2c_load_rows: row %lld: count outside 0 .. 2**32-1", (long long)r);
            return -3;
        }
        if (offset[r] < 0 || offset[r] > A2C_MAX_SPAN) {
            set_error("mh_a2c_load_rows: row %lld: offset outside 0 .. 2**28", (long long)r);
            return -3;
        }
        for (int32_t k = 0; k < seq_len[r]; ++k) {
            const char ch = pool[seq_off[r] + k];
            if (S.cls[(uint8_t)ch] == A2C_BAD) {
                set_error("mh_a2c_load_rows: row %lld: character '%c' is not one of A C G T N - n",
                          (long long)r, ch);
                return -3;
            }
        }
        S.rows[r] = A2CRow{seq_off[r], seq_len[r], (int32_t)offset[r], (uint32_t)count[r], 0};
    }
    S.n_rows = n_rows;
    S.g_first.assign(group_first, group_first + n_groups + 1);
    for (int64_t g = 0; g < n_groups; ++g)
        if (group_first[g + 1] < group_first[g]) {
            set_error("mh_a2c_load_rows: group_first must not decrease");
            return -3;
        }
    S.g_ref.assign(n_groups, std::string());
    S.g_qcut.assign(n_groups, std::string());
    S.t_parse = ms_since(t0);
    auto t1 = std::chrono::steady_clock::now();
    if (int st = a2c_count(c, S, pool ? pool : "", pool_len)) {
        S.rows.clear();
        S.g_first.assign(1, 0);
        return st;
    }
    S.t_count = ms_since(t1);
    return 0;
}

extern "C" int mh_a2c_group(mh_ctx *ctx, int slot, int64_t g, int64_t *info5, char *names,
                            size_t cap, size_t *used)
{
    if (!ctx || slot < 0 || slot >= A2C_SLOTS || !info5) return -3;
    Ctx &c = *ctx_of(ctx);
    A2CState &S = *a2c_state(c, slot);
    const int64_t ng = (int64_t)S.g_first.size() - 1;
    if (g < 0 || g >= ng) { set_error("mh_a2c_group: no group %lld", (long long)g); return -3; }
    info5[0] = S.g_first[g];
    info5[1] = S.g_first[g + 1] - S.g_first[g];
    for (int f = 0; f < 3; ++f) info5[2 + f] = S.g_ncod[3 * g + f];
    const std::string &r = S.g_ref[g], &q = S.g_qcut[g];
    const size_t need = r.size() + 1 + q.size();
    if (used) *used = need;
    if (names) {
        if (cap < need) { set_error("mh_a2c_group: buffer too small"); return -2; }
        memcpy(names, r.data(), r.size());
        names[r.size()] = '\0';
        memcpy(names + r.size() + 1, q.data(), q.size());
    }
    return 0;
}

extern "C" int mh_a2c_counts(mh_ctx *ctx, int slot, int64_t g, int frame, uint32_t *aa_count,
                             uint32_t *aa_first, uint32_t *nuc_count, uint32_t *nuc_first)
{
    if (!ctx || slot < 0 || slot >= A2C_SLOTS || frame < 0 || frame > 2) return -3;
    Ctx &c = *ctx_of(ctx);
    A2CState &S = *a2c_state(c, slot);
    const int64_t ng = (int64_t)S.g_first.size() - 1;
    if (g < 0 || g >= ng) { set_error("mh_a2c_counts: no group %lld", (long long)g); return -3; }
    const int n = S.g_ncod[3 * g + frame];
    if (n && (!aa_count || !aa_first || !nuc_count || !nuc_first)) return -3;
    for (int j = 0; j < n; ++j) {
        const size_t at = (size_t)(S.g_bin0[g] + j / A2C_W) * A2C_CELLS +
                          (size_t)(A2C_W * frame + j % A2C_W) * A2C_STRIDE;
        memcpy(aa_count + (size_t)j * A2C_NAA, &S.h_cnt[at], 4 * A2C_NAA);
        memcpy(aa_first + (size_t)j * A2C_NAA, &S.h_first[at], 4 * A2C_NAA);
        memcpy(nuc_count + (size_t)j * 18, &S.h_cnt[at + A2C_NAA], 4 * 18);
        memcpy(nuc_first + (size_t)j * 18, &S.h_first[at + A2C_NAA], 4 * 18);
    }
    return 0;
}

extern "C" int mh_a2c_inserts(mh_ctx *ctx, int slot, int64_t g, int frame, int n_ranges,
                              const int32_t *left, const int32_t *right, int64_t *n_entries)
{
    if (!ctx || slot < 0 || slot >= A2C_SLOTS || frame < 0 || frame > 2 || n_ranges < 0 ||
        (n_ranges && (!left || !right)))
        return -3;
    Ctx &c = *ctx_of(ctx);
    MH_HIP(hipSetDevice(c.device));
    A2CState &S = *a2c_state(c, slot);
    a2c_clear_inserts(S);
    if (n_entries) *n_entries = 0;
    const int64_t ng = (int64_t)S.g_first.size() - 1;
    if (g < 0 || g >= ng) { set_error("mh_a2c_inserts: no group %lld", (long long)g); return -3; }
    for (int k = 0; k < n_ranges; ++k)
        if (left[k] < 0 || right[k] < left[k] || right[k] > (1 << 27)) {
            set_error("mh_a2c_inserts: bad range %d..%d", left[k], right[k]);
            return -3;
        }
    const int64_t nr = S.g_first[g + 1] - S.g_first[g], np = nr * n_ranges;
    if (np == 0) return 0;
    auto t0 = std::chrono::steady_clock::now();
    hipStream_t s = c.stream;
    int32_t *d_lr = nullptr;
    uint64_t *d_h = nullptr, *d_tkey = nullptr;
    unsigned long long *d_tcnt = nullptr, *d_ctr = nullptr;
    uint32_t *d_tfirst = nullptr;
    int32_t *d_trange = nullptr;
    A2CEntry *d_ent = nullptr, *d_sorted = nullptr;
    int64_t *d_eoff = nullptr;
    char *d_out = nullptr;
    int rc = 0;
    auto fail = [&](hipError_t e, const char *what) {
        rc = hip_fail(e, what);
        return rc;
    };
    A2CInsArgs a{};
    uint64_t tsize = 1024;
    unsigned long long ctr[3] = {0, 0, 0};
    std::vector<int32_t> lr(2 * (size_t)n_ranges);
    std::vector<A2CEntry> ent;
    std::vector<int64_t> eoff;
    hipError_t e = hipMalloc(&d_lr, sizeof(int32_t) * lr.size());
    for (int k = 0; k < n_ranges; ++k) { lr[k] = left[k]; lr[n_ranges + k] = right[k]; }
    if (e == hipSuccess) e = hipMemcpyAsync(d_lr, lr.data(), sizeof(int32_t) * lr.size(), hipMemcpyHostToDevice, s);
    if (e == hipSuccess) e = hipMalloc(&d_h, sizeof(uint64_t) * np);
    if (e == hipSuccess) e = hipMalloc(&d_ctr, sizeof(unsigned long long) * 3);
    if (e == hipSuccess) e = hipMemsetAsync(d_ctr, 0, sizeof(unsigned long long) * 3, s);
    if (e != hipSuccess) { fail(e, "mh_a2c_inserts alloc"); goto done; }
    a.text = S.d_text;
    a.rows = S.d_rows + S.g_first[g];
    a.row0 = S.rows[(size_t)S.g_first[g]].local;
    a.code = S.d_code;
    a.cls = S.d_cls;
    a.left = d_lr;
    a.right = d_lr + n_ranges;
    a.n_rows = nr;
    a.n_pairs = np;
    a.frame = frame;
    a.h = d_h;
    a.ctr = d_ctr;
    {
        const int p0 = prof_begin(c, "k_a2c_ins");
        hipLaunchKernelGGL(k_a2c_ins_hash, dim3((unsigned)((np + 255) / 256)), dim3(256), 0, s, a);
        prof_end(c, p0);
    }
    e = hipGetLastError();
    if (e == hipSuccess) e = hipMemcpyAsync(ctr, d_ctr, sizeof(ctr), hipMemcpyDeviceToHost, s);
    if (e == hipSuccess) e = hipStreamSynchronize(s);
    if (e != hipSuccess) { fail(e, "k_a2c_ins_hash"); goto done; }
    if (ctr[0] == 0) goto done;
    while (tsize < 2 * ctr[0]) tsize <<= 1;
    e = hipMalloc(&d_tkey, sizeof(uint64_t) * tsize);
    if (e == hipSuccess) e = hipMalloc(&d_tcnt, sizeof(unsigned long long) * tsize);
    if (e == hipSuccess) e = hipMalloc(&d_tfirst, sizeof(uint32_t) * tsize);
    if (e == hipSuccess) e = hipMalloc(&d_trange, sizeof(int32_t) * tsize);
    if (e == hipSuccess) e = hipMalloc(&d_ent, sizeof(A2CEntry) * ctr[0]);
    if (e == hipSuccess) e = hipMemsetAsync(d_tkey, 0, sizeof(uint64_t) * tsize, s);
    if (e == hipSuccess) e = hipMemsetAsync(d_tcnt, 0, sizeof(unsigned long long) * tsize, s);
    if (e == hipSuccess) e = hipMemsetAsync(d_tfirst, 0xff, sizeof(uint32_t) * tsize, s);
    if (e != hipSuccess) { fail(e, "mh_a2c_inserts table"); goto done; }
    a.tkey = d_tkey;
    a.tcnt = d_tcnt;
    a.tfirst = d_tfirst;
    a.trange = d_trange;
    a.mask = tsize - 1;
    a.entries = d_ent;
    {
        const int p0 = prof_begin(c, "k_a2c_ins");
        hipLaunchKernelGGL(k_a2c_ins_count, dim3((unsigned)((np + 255) / 256)), dim3(256), 0, s, a);
        hipLaunchKernelGGL(k_a2c_ins_verify, dim3((unsigned)((np + 255) / 256)), dim3(256), 0, s, a);
        hipLaunchKernelGGL(k_a2c_ins_compact, dim3((unsigned)((tsize + 255) / 256)), dim3(256), 0, s, a);
        prof_end(c, p0);
    }
    e = hipGetLastError();
    if (e == hipSuccess) e = hipMemcpyAsync(ctr, d_ctr, sizeof(ctr), hipMemcpyDeviceToHost, s);
    if (e == hipSuccess) e = hipStreamSynchronize(s);
    if (e != hipSuccess) { fail(e, "k_a2c_ins"); goto done; }
    if (ctr[1]) {
        set_error("aln2counts: insertion-string hash collision (distinct strings share a key)");
        rc = -4;
        goto done;
    }
    ent.resize(ctr[2]);
    e = copy_sync(c, ent.data(), d_ent, sizeof(A2CEntry) * ent.size(), hipMemcpyDeviceToHost);
    if (e != hipSuccess) { fail(e, "mh_a2c_inserts fetch"); goto done; }
    // InsertionWriter order: ranges in order, then Counter insertion order
    std::sort(ent.begin(), ent.end(), [](const A2CEntry &x, const A2CEntry &y) {
        return x.range != y.range ? x.range < y.range : x.first < y.first;
    });
    eoff.resize(ent.size() + 1);
    eoff[0] = 0;
    for (size_t k = 0; k < ent.size(); ++k) eoff[k + 1] = eoff[k] + ent[k].n_codons + 1;
    S.aminos.assign((size_t)eoff.back(), '\0');
    e = hipMalloc(&d_sorted, sizeof(A2CEntry) * ent.size());
    if (e == hipSuccess) e = hipMalloc(&d_eoff, sizeof(int64_t) * eoff.size());
    if (e == hipSuccess) e = hipMalloc(&d_out, (size_t)eoff.back());
    if (e == hipSuccess) e = hipMemcpyAsync(d_sorted, ent.data(), sizeof(A2CEntry) * ent.size(), hipMemcpyHostToDevice, s);
    if (e == hipSuccess) e = hipMemcpyAsync(d_eoff, eoff.data(), sizeof(int64_t) * eoff.size(), hipMemcpyHostToDevice, s);
    if (e != hipSuccess) { fail(e, "mh_a2c_inserts gather"); goto done; }
    hipLaunchKernelGGL(k_a2c_ins_gather, dim3((unsigned)((ent.size() + 255) / 256)), dim3(256), 0, s,
                       a, d_sorted, d_eoff, (int64_t)ent.size(), d_out);
    e = hipGetLastError();
    if (e == hipSuccess) e = hipMemcpyAsync(&S.aminos[0], d_out, (size_t)eoff.back(), hipMemcpyDeviceToHost, s);
    if (e == hipSuccess) e = hipStreamSynchronize(s);
    if (e != hipSuccess) { fail(e, "k_a2c_ins_gather"); goto done; }
    S.entries = std::move(ent);
    if (n_entries) *n_entries = (int64_t)S.entries.size();
done:
    hipFree(d_lr); hipFree(d_h); hipFree(d_ctr); hipFree(d_tkey); hipFree(d_tcnt);
    hipFree(d_tfirst); hipFree(d_trange); hipFree(d_ent); hipFree(d_sorted); hipFree(d_eoff);
    hipFree(d_out);
    prof_flush(c);
    S.t_ins += ms_since(t0);
    if (rc) a2c_clear_inserts(S);
    return rc;
}

extern "C" int mh_a2c_insert_entries(mh_ctx *ctx, int slot, int32_t *range, int64_t *count,
                                     uint32_t *first, char *aminos, size_t cap, size_t *used)
{
    if (!ctx || slot < 0 || slot >= A2C_SLOTS) return -3;
    Ctx &c = *ctx_of(ctx);
    A2CState &S = *a2c_state(c, slot);
    for (size_t k = 0; k < S.entries.size(); ++k) {
        if (range) range[k] = S.entries[k].range;
        if (count) count[k] = (int64_t)S.entries[k].count;
        if (first) first[k] = S.entries[k].first;
    }
    if (used) *used = S.aminos.size();
    if (aminos) {
        if (cap < S.aminos.size()) { set_error("mh_a2c_insert_entries: buffer too small"); return -2; }
        memcpy(aminos, S.aminos.data(), S.aminos.size());
    }
    return 0;
}

extern "C" int mh_a2c_insert_rows(mh_ctx *ctx, int slot, const char *lead, int n_ranges,
                                  const int32_t *left, const int32_t *target, const char *eol,
                                  char *buf, size_t cap, size_t *used)
{
    if (!ctx || slot < 0 || slot >= A2C_SLOTS || !lead || !eol || !used || n_ranges < 0 ||
        (n_ranges && (!left || !target)))
        return -3;
    Ctx &c = *ctx_of(ctx);
    A2CState &S = *a2c_state(c, slot);
    if (!buf) {
        // InsertionWriter.write's rows: lead, left codon + 1, the amino-acid
        // string, its count, the coordinate position (blank when none)
        std::string &o = S.ins_rows;
        o.clear();
        const size_t ll = strlen(lead), el = strlen(eol);
        o.reserve(S.entries.size() * (ll + el + 24) + S.aminos.size());
        const char *am = S.aminos.data(), *am_end = am + S.aminos.size();
        char num[24];
        auto put = [&](long long v) {
            auto r = std::to_chars(num, num + sizeof num, v);
            o.append(num, (size_t)(r.ptr - num));
        };
        for (size_t k = 0; k < S.entries.size(); ++k) {
            const char *nl = (const char *)memchr(am, '\n', (size_t)(am_end - am));
            if (!nl) { set_error("mh_a2c_insert_rows: entry strings out of step"); return -3; }
            const int r = S.entries[k].range;
            if (r < 0 || r >= n_ranges) { set_error("mh_a2c_insert_rows: range %d out of %d", r, n_ranges); return -3; }
            o.append(lead, ll);
            put((long long)left[r] + 1);
            o.push_back(',');
            o.append(am, (size_t)(nl - am));
            o.push_back(',');
            put((long long)S.entries[k].count);
            o.push_back(',');
            if (target[r] != INT32_MIN) put(target[r]);
            o.append(eol, el);
            am = nl + 1;
        }
        *used = o.size();
        return 0;
    }
    *used = S.ins_rows.size();
    if (cap < S.ins_rows.size()) { set_error("mh_a2c_insert_rows: buffer too small"); return -2; }
    memcpy(buf, S.ins_rows.data(), S.ins_rows.size());
    std::string().swap(S.ins_rows);
    return 0;
}

extern "C" int mh_a2c_timing(mh_ctx *ctx, int slot, double *ms3)
{
    if (!ctx || slot < 0 || slot >= A2C_SLOTS || !ms3) return -3;
    Ctx &c = *ctx_of(ctx);
    A2CState &S = *a2c_state(c, slot);
    ms3[0] = S.t_parse;
    ms3[1] = S.t_count;
    ms3[2] = S.t_ins;
    S.t_ins = 0;
    return 0;
}

// ---------------------------------------------------------------------------
// aln2counts split over the ranks of a job.  The reference counts every row
// of aligned.csv into per-(refname, qcut) Counters (aln2counts.py:115-172),
// in file order; the counts are sums and the first row a Counter saw is a
// minimum, so rank r counts the rows in its share of the file's bytes and
// the caller adds the ranks' counters up (and takes the minimum of their
// first rows): mh_a2c_part_open parses the share, mh_a2c_part_groups reports
// its runs of (refname, qcut), mh_a2c_part_count lays out the job's groups
// (codon extents, row numbers within a group from the ranks before) and
// counts, mh_a2c_part_counters hands the counters out and takes the sums
// back.  The insertion strings of InsertionWriter.write (:786-795) are the
// same kind of reduction: mh_a2c_insert_export / mh_a2c_insert_merge.
// ---------------------------------------------------------------------------
static int64_t a2c_line_start(const char *t, int64_t lo, int64_t hi, int64_t x)
{
    if (x <= lo) return lo;
    if (x >= hi) return hi;
    if (t[x - 1] == '\n') return x;
    const char *q = (const char *)memchr(t + x, '\n', (size_t)(hi - x));
    return q ? (q - t) + 1 : hi;
}

extern "C" int mh_a2c_part_open(mh_ctx *ctx, int slot, int fd, int part, int parts,
                                const char *codon_chars, int64_t *info3)
{
    if (!ctx || slot < 0 || slot >= A2C_SLOTS || fd < 0 || parts < 1 || part < 0 || part >= parts ||
        !info3)
        return -3;
    Ctx &c = *ctx_of(ctx);
    MH_HIP(hipSetDevice(c.device));
    A2CState &S = *a2c_state(c, slot);
    a2c_clear_inserts(S);
    if (S.part_text) { unmap_text_file(S.part_text, S.part_len); S.part_text = nullptr; }
    S.part_open = false;
    if (int st = a2c_tables(S, codon_chars)) return st;
    const char *text = nullptr;
    size_t len = 0;
    if (int st = map_text_file(fd, &text, &len)) return st;   // 1: '\r' in it
    auto t0 = std::chrono::steady_clock::now();
    const char *p = text, *end = text + len;
    std::vector<std::string> head;
    int64_t lo = 0, hi = (int64_t)len;
    if (csv_record(p, end, head)) lo = p - text;
    const int64_t b0 = a2c_line_start(text, lo, hi, lo + (hi - lo) * part / parts);
    const int64_t b1 = a2c_line_start(text, lo, hi, lo + (hi - lo) * (part + 1) / parts);
    // a quoted field (a refname with a comma) is parsed on one thread into a
    // pool; the split is kept to unquoted files
    if (memchr(text + b0, '"', (size_t)(b1 - b0))) { unmap_text_file(text, len); return 1; }
    bool use_pool = false;
    int st = 0;
    try {
        st = a2c_parse_csv(S, text, (int64_t)len, use_pool, b0, b1);
    } catch (const std::exception &e) {
        set_error("aligned csv: out of memory (%s)", e.what());
        st = -2;
    }
    if (st || use_pool) {
        unmap_text_file(text, len);
        S.rows.clear();
        S.g_first.assign(1, 0);
        return st ? st : 1;
    }
    S.part_text = text;
    S.part_len = len;
    S.part_open = true;
    S.part_b0 = b0;
    S.part_b1 = b1;
    S.part_first = S.g_first;
    S.t_parse = ms_since(t0);
    info3[0] = S.n_rows;
    info3[1] = (int64_t)S.g_first.size() - 1;
    info3[2] = b1 - b0;
    return 0;
}

extern "C" int mh_a2c_part_groups(mh_ctx *ctx, int slot, char *keys, size_t cap, size_t *used,
                                  int64_t *rows, int32_t *ncod3, int64_t *total)
{
    if (!ctx || slot < 0 || slot >= A2C_SLOTS || !used) return -3;
    Ctx &c = *ctx_of(ctx);
    A2CState &S = *a2c_state(c, slot);
    const int64_t ng = (int64_t)S.part_first.size() - 1;
    size_t need = 0;
    for (int64_t g = 0; g < ng; ++g) need += S.g_ref[g].size() + S.g_qcut[g].size() + 2;
    *used = need;
    if (!keys) return 0;
    if (cap < need || !rows || !ncod3 || !total) { set_error("mh_a2c_part_groups: buffer too small"); return -2; }
    for (int64_t g = 0; g < ng; ++g) {
        memcpy(keys, S.g_ref[g].data(), S.g_ref[g].size());
        keys += S.g_ref[g].size();
        *keys++ = '\x1f';
        memcpy(keys, S.g_qcut[g].data(), S.g_qcut[g].size());
        keys += S.g_qcut[g].size();
        *keys++ = '\n';
        int32_t nc[3] = {0, 0, 0};
        uint64_t tot = 0;
        for (int64_t r = S.part_first[g]; r < S.part_first[g + 1]; ++r) {
            const A2CRow &R = S.rows[r];
            tot += R.cnt;
            const int l = R.off / 3;
            for (int f = 0; f < 3; ++f) {
                const int h = (f + R.off + R.len + 2) / 3;
                if (h > l && h > nc[f]) nc[f] = h;
            }
        }
        rows[g] = S.part_first[g + 1] - S.part_first[g];
        for (int f = 0; f < 3; ++f) ncod3[3 * g + f] = nc[f];
        total[g] = (int64_t)tot;
    }
    return 0;
}

extern "C" int mh_a2c_part_count(mh_ctx *ctx, int slot, int64_t n_groups, const char *keys,
                                 const int64_t *gid, const int32_t *ncod3, const int64_t *row_base,
                                 int64_t *cells)
{
    if (!ctx || slot < 0 || slot >= A2C_SLOTS || n_groups < 0 || (n_groups && (!keys || !ncod3)) ||
        !cells)
        return -3;
    Ctx &c = *ctx_of(ctx);
    MH_HIP(hipSetDevice(c.device));
    A2CState &S = *a2c_state(c, slot);
    if (!S.part_open) { set_error("mh_a2c_part_count: no part open"); return -3; }
    const int64_t nl = (int64_t)S.part_first.size() - 1;
    if (nl && (!gid || !row_base)) return -3;
    for (int64_t k = 0; k < nl; ++k)
        if (gid[k] < 0 || gid[k] >= n_groups || (k && gid[k] <= gid[k - 1])) {
            set_error("mh_a2c_part_count: group ids out of order");
            return -3;
        }
    // the job's groups, this part's rows in them (global row numbers within
    // a group for the first-row counters)
    std::vector<std::string> ref, qcut;
    const char *p = keys;
    for (int64_t g = 0; g < n_groups; ++g) {
        const char *us = strchr(p, '\x1f'), *nlp = us ? strchr(us, '\n') : nullptr;
        if (!us || !nlp) { set_error("mh_a2c_part_count: malformed group keys"); return -3; }
        ref.emplace_back(p, (size_t)(us - p));
        qcut.emplace_back(us + 1, (size_t)(nlp - us - 1));
        p = nlp + 1;
    }
    std::vector<int64_t> first((size_t)n_groups + 1, 0);
    {
        int64_t k = 0, at = 0;
        for (int64_t g = 0; g < n_groups; ++g) {
            first[(size_t)g] = at;
            if (k < nl && gid[k] == g) {
                for (int64_t r = S.part_first[k]; r < S.part_first[k + 1]; ++r)
                    S.rows[r].local = (uint32_t)(row_base[k] + (r - S.part_first[k]));
                at = S.part_first[k + 1];
                ++k;
            }
        }
        first[(size_t)n_groups] = at;
    }
    S.g_first.swap(first);
    S.g_ref.swap(ref);
    S.g_qcut.swap(qcut);
    S.g_ncod.assign(ncod3, ncod3 + 3 * n_groups);
    auto t1 = std::chrono::steady_clock::now();
    int st = 0;
    try {
        // only the part's bytes go to the device: row offsets from b0
        for (A2CRow &R : S.rows) R.soff -= S.part_b0;
        st = a2c_count(c, S, S.part_text + S.part_b0, S.part_b1 - S.part_b0, true);
    } catch (const std::exception &e) {
        set_error("aln2counts: out of memory (%s)", e.what());
        st = -2;
    }
    unmap_text_file(S.part_text, S.part_len);
    S.part_text = nullptr;
    S.part_len = 0;
    S.part_open = false;
    if (st) {
        S.rows.clear();
        S.g_first.assign(1, 0);
        return st;
    }
    S.t_count = ms_since(t1);
    *cells = (int64_t)S.h_cnt.size();
    return 0;
}

extern "C" int mh_a2c_part_counters(mh_ctx *ctx, int slot, int set, uint32_t *cnt, uint32_t *first)
{
    if (!ctx || slot < 0 || slot >= A2C_SLOTS || !cnt || !first) return -3;
    Ctx &c = *ctx_of(ctx);
    A2CState &S = *a2c_state(c, slot);
    const size_t n = S.h_cnt.size();
    if (set) {
        memcpy(S.h_cnt.data(), cnt, 4 * n);
        memcpy(S.h_first.data(), first, 4 * n);
    } else {
        memcpy(cnt, S.h_cnt.data(), 4 * n);
        memcpy(first, S.h_first.data(), 4 * n);
    }
    return 0;
}

// insertion entries on the wire: range, first row, codons, string length,
// count, then the string, padded to 8
struct A2CWireEntry {
    int32_t range;
    uint32_t first;
    int32_t n_codons;
    int32_t slen;
    unsigned long long count;
};

extern "C" int mh_a2c_insert_export(mh_ctx *ctx, int slot, uint8_t *buf, size_t cap, size_t *used)
{
    if (!ctx || slot < 0 || slot >= A2C_SLOTS || !used) return -3;
    Ctx &c = *ctx_of(ctx);
    A2CState &S = *a2c_state(c, slot);
    size_t need = 0;
    const char *am = S.aminos.data(), *am_end = am + S.aminos.size();
    std::vector<std::pair<const char *, size_t>> str;
    for (size_t k = 0; k < S.entries.size(); ++k) {
        const char *nl = (const char *)memchr(am, '\n', (size_t)(am_end - am));
        if (!nl) { set_error("mh_a2c_insert_export: entry strings out of step"); return -3; }
        str.emplace_back(am, (size_t)(nl - am));
        need += sizeof(A2CWireEntry) + ((str.back().second + 7) & ~(size_t)7);
        am = nl + 1;
    }
    *used = need;
    if (!buf) return 0;
    if (cap < need) { set_error("mh_a2c_insert_export: buffer too small"); return -2; }
    memset(buf, 0, need);
    for (size_t k = 0; k < S.entries.size(); ++k) {
        const A2CEntry &e = S.entries[k];
        A2CWireEntry w{e.range, e.first, e.n_codons, (int32_t)str[k].second, e.count};
        memcpy(buf, &w, sizeof w);
        memcpy(buf + sizeof w, str[k].first, str[k].second);
        buf += sizeof w + ((str[k].second + 7) & ~(size_t)7);
    }
    return 0;
}

// every rank's entries of one insertion call: equal (range, string) added
// up, the first row the least, in (range, first row) order
extern "C" int mh_a2c_insert_merge(mh_ctx *ctx, int slot, const uint8_t *buf, int64_t len,
                                   int64_t *n_entries)
{
    if (!ctx || slot < 0 || slot >= A2C_SLOTS || (!buf && len) || len < 0) return -3;
    Ctx &c = *ctx_of(ctx);
    A2CState &S = *a2c_state(c, slot);
    std::map<std::pair<int32_t, std::string>, A2CEntry> merged;
    int64_t at = 0;
    while (at < len) {
        if (len - at < (int64_t)sizeof(A2CWireEntry)) { set_error("mh_a2c_insert_merge: malformed"); return -3; }
        A2CWireEntry w;
        memcpy(&w, buf + at, sizeof w);
        const int64_t sz = (int64_t)(sizeof w + (((size_t)w.slen + 7) & ~(size_t)7));
        if (w.slen < 0 || len - at < sz) { set_error("mh_a2c_insert_merge: malformed"); return -3; }
        std::string key((const char *)buf + at + sizeof w, (size_t)w.slen);
        auto it = merged.find({w.range, key});
        if (it == merged.end()) {
            merged.emplace(std::make_pair(w.range, std::move(key)), A2CEntry{w.range, w.first, w.n_codons, 0, w.count});
        } else {
            it->second.count += w.count;
            it->second.first = std::min(it->second.first, w.first);
        }
        at += sz;
    }
    std::vector<std::pair<const std::string *, A2CEntry>> v;
    for (auto &kv : merged) v.push_back({&kv.first.second, kv.second});
    std::sort(v.begin(), v.end(), [](const auto &x, const auto &y) {
        return x.second.range != y.second.range ? x.second.range < y.second.range
                                                : x.second.first < y.second.first;
    });
    S.entries.clear();
    S.aminos.clear();
    for (auto &x : v) {
        S.entries.push_back(x.second);
        S.aminos += *x.first;
        S.aminos.push_back('\n');
    }
    if (n_entries) *n_entries = (int64_t)S.entries.size();
    return 0;
}
