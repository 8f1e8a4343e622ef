// mh_internal.h -- device-side data layout shared by the HIP translation
// units of libmicall_hip.so (gfx950 only).  See DESIGN.md "Data layout".
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <string.h>

#include <map>
#include <mutex>
#include <string>
#include <string_view>
#include <tuple>
#include <vector>

#include "micall_hip.h"
#include "mh_gunzip.h"

namespace mh {

// Mapper constants (the specification lives in oracle/og_mapper.c, which the
// kernels reproduce bit for bit).
constexpr int BAND = 64;            // bound on the diagonals a DP band spans (2 * MAXHALF + 1 <= 64)
constexpr int MAXCAND = 4;          // extension candidates per mate
constexpr int MAXHITS_SEED = 64;    // seeds with more exact hits are skipped
constexpr int MAXHITS_MATE = 512;   // hit budget per mate, in seed order
constexpr int CLUSTER_GAP = 8;      // diagonal gap that splits clusters
constexpr int MAXSEEDS = 32;        // seeds per strand
constexpr int MAXLEN = 1024;        // longest read accepted
constexpr int GBAR = 4;             // --gbar 4
constexpr int NPEN = 1;             // --np 1
constexpr int NEG = -(1 << 29);     // minus infinity of the DP
constexpr int32_t I32MIN = INT32_MIN;
constexpr int MAXHALF = 15;         // bowtie2's maxhalf: DP band = center +- min(15, max gaps)

// the mapping parameters the per-length tables depend on
inline int64_t len_tab_key(const mh_params &p)
{
    return (int64_t)p.mode | (int64_t)(p.rdg_open & 0xff) << 8 | (int64_t)(p.rdg_ext & 0xff) << 16 |
           (int64_t)(p.rfg_open & 0xff) << 24 | (int64_t)(p.rfg_ext & 0xff) << 32;
}

// Reads resident in HBM: each read starts on a 32-base boundary.
//   seq2 : 2-bit codes, 16 bases per u32, base b at bits 2*(b%16)
//   nmask: 1 bit per base (ambiguous -> code 0 in seq2 and bit set here)
//   qual : Phred+33 bytes
struct DevReads {
    int64_t n = 0;
    int paired = 0;
    int max_len = 0;
    int64_t total_bases = 0;  // padded
    uint32_t *seq2 = nullptr;
    uint32_t *nmask = nullptr;
    uint8_t *qual = nullptr;
    int64_t *off = nullptr;   // padded base offset (multiple of 32)
    int32_t *len = nullptr;
};

// Reference set + exact-seed hash index (replaces the .bt2 files).
struct DevIndex {
    int n_refs = 0;
    int seedlen = 0;
    int64_t total = 0;
    uint8_t *codes = nullptr;      // 0..3, 4 = ambiguous; refs back to back
    uint32_t *code2 = nullptr;     // the same packed: 16 bases per word (0 where ambiguous)
    uint32_t *ncode = nullptr;     // 1 bit per base: ambiguous
    uint32_t *cplane = nullptr;    // bit planes, 32 bases per word: [2k] low code bits, [2k+1] high
    int64_t *ref_off = nullptr;
    int32_t *ref_len = nullptr;
    // open addressing: one 16-B entry per slot, (key low, key high, start,
    // count) with key EMPTY = ~0, so a probe that finds its key has the hits'
    // range in the same load (one dependent round trip less per seed)
    uint4 *hent = nullptr;
    uint64_t hmask = 0;
    int2 *hits = nullptr;          // (ref, pos) sorted per key
    uint64_t sig = 0;              // content signature (cache key)
    // every array above lives in one device allocation, uploaded with one
    // copy (a small index is rebuilt in place every remap pass)
    void *blob = nullptr;
    int64_t cap_blob = 0;
};

constexpr uint64_t HEMPTY = ~0ull;

__host__ __device__ inline uint64_t hash_key(uint64_t k)
{
    k ^= k >> 33;
    k *= 0xff51afd7ed558ccdull;
    k ^= k >> 33;
    k *= 0xc4ceb9fe1a85ec53ull;
    k ^= k >> 33;
    return k;
}

struct Cand {
    int32_t strand, ref, center, support;
};

// Result of one banded extension (one candidate of one read), as k_dp
// builds it in registers.
struct Slot {
    int32_t valid, strand, ref, pos, end, score, xm, xo, xg, nm, n_cigar, cig_off;
    int32_t maxm;   // longest M run of the CIGAR (remap.py:500-506 filter), from the traceback
};

// In HBM a slot is split in two arrays: the 16-B key that pairing, mate
// rescue and the best-candidate choice compare (a read's MAXCAND keys are
// one 64-B line), and the 16-B statistics only the chosen candidate's
// record copies.  Memory requests are 128-B lines
// (profiles/r06/diag/fetch_calib.json), so the statistics are packed to put
// a pair's two reads (2 x MAXCAND x 16 B) in one line: k_pair reads one line
// of them per pair, not two.  NM = XM + XG is not stored.
struct alignas(16) SlotKey {
    int32_t rs;      // ref << 1 | strand; -1 when the extension found no alignment
    int32_t pos, end, score;
};
struct alignas(16) SlotInfo {
    int32_t cig_off;
    uint32_t xm_xo;   // xm | xo << 16 (both below 2^16: reads <= MAXLEN, ops <= MH_MAXOPS)
    uint32_t xg_nc;   // xg | n_cigar << 16
    int32_t maxm;
};
static_assert(sizeof(SlotInfo) == 16, "a read's MAXCAND statistics fill half a 128-B line");

// Final per-read SAM record (mh_aln without the inline CIGAR).
struct Rec {
    int32_t ref, pos, rev, score, secbest, flag, mapq, rnext, pnext, tlen;
    int32_t sam_ref, sam_pos, xm, xo, xg, nm, ys, yt, yf, n_cigar;
    int32_t cig_off, maxm;   // cigar offset in the pool; longest M run
};

// slot id (read * MAXCAND + candidate) -> its index in the candidate-major
// slot planes of stride `plane`
__host__ __device__ inline int64_t slot_at(int32_t sid, int64_t plane)
{
    const uint32_t u = (uint32_t)sid;
    return (int64_t)(u % MAXCAND) * plane + (int64_t)(u / MAXCAND);
}

struct MapState {
    int64_t n_reads = 0;
    int n_refs = 0;
    mh_params par{};
    Cand *cand = nullptr;        // MAXCAND planes of cap_reads, like the slots
    int32_t *n_cand = nullptr;   // n_reads
    int32_t *yf = nullptr;       // n_reads
    int32_t *work = nullptr;     // slot ids to extend
    int32_t *rwork = nullptr;    // slot ids of mate-rescue candidates (one per pair at most)
    // the extension slots, candidate-major: slot id r * MAXCAND + c lives at
    // c * cap_reads + r (slot_at), so a pass where most reads have one
    // candidate reads one plane of keys and statistics, not every line
    SlotKey *skey = nullptr;     // MAXCAND planes of cap_reads
    SlotInfo *sinfo = nullptr;   // MAXCAND planes of cap_reads
    uint32_t *pool = nullptr;    // CIGAR ops of all slots
    int64_t pool_cap = 0;
    unsigned long long *pool_used = nullptr;  // words claimed (demand; may exceed pool_cap)
    Rec *rec = nullptr;          // n_reads
    int32_t *counters = nullptr; // [work_n, unused, pool_overflow, fast, rescue_n, queue, rescue queue, pad]
    int64_t *ref_stats = nullptr;// per ref: lines, filtered, mapped, first_row, first_mapped; + unmapped, star
    int64_t cap_reads = 0;
    int cap_refs = 0;
    int64_t last_work = 0;       // extensions (k_dp work items) of the last pass
    int64_t last_cigar = 0;      // CIGAR ops written by the last pass
    int64_t last_fast = 0;       // extensions resolved by the ungapped fast path
    int64_t last_rescue = 0;     // mate-rescue extensions
    bool valid = false;
    // host copy of ref_stats (5 * n_refs + 3), filled on first use after a
    // mapping pass: mh_map_counts and the pileup's window choice share it
    std::vector<int64_t> stats_host;
    // pinned landing area of ref_stats, copied at the end of each pass (mh_map
    // synchronises anyway), so mh_map_counts needs no round trip of its own
    int64_t *stats_pin = nullptr;
    size_t stats_pin_cap = 0;
    bool stats_pin_ready = false;
    // k_dp launch shapes already sized: (kernel, LDS bytes) -> blocks per CU
    // that fit (the occupancy query is a host call worth skipping per launch)
    std::map<std::pair<const void *, int>, int> dp_occ;
    bool stats_host_valid = false;
};

// External SAM rows for the pileup (prelim.csv read back).
struct RowState {
    int64_t n_rows = 0, n_units = 0;
    int32_t *flag = nullptr, *ref = nullptr, *pos = nullptr, *cig_off = nullptr,
            *n_cigar = nullptr;
    uint32_t *cigar = nullptr;
    int64_t *units = nullptr;
    DevReads reads;
    int hot_ref = -1;      // reference of most mapped rows
    std::vector<int64_t> ref_rows;   // mapped rows per reference (pileup LDS windows)
    int max_span = 0;      // longest reference span (M + D) of a mapped row
};

struct PileState {
    int n_refs = 0;
    int32_t cap = 0;
    int32_t *dense = nullptr;       // n_refs * cap * 4
    uint8_t *nflag = nullptr;       // n_refs * cap
    uint8_t *dflag = nullptr;
    int64_t *read_counts = nullptr; // n_refs
    int64_t *first_unit = nullptr;  // n_refs
    int32_t *max_pos = nullptr;     // n_refs
    int32_t *ev = nullptr;          // events: 4 int32 (ref, pos, tok_off, tok_len)
    char *ev_pool = nullptr;
    int64_t ev_cap = 0, pool_cap = 0;
    int64_t *ev_counters = nullptr; // [n_events, pool_used, overflow, error]
    int64_t alloc_cells = 0;
    int alloc_refs = 0;
    int64_t gen = 0;                // bumped by every mh_pileup / mh_pileup_import
    // pinned landing of the per-reference scalars (read_counts, first_unit,
    // max_pos) and ev_counters, copied behind mh_pileup's kernels so the
    // fetches after it need no round trip; cleared by anything that changes them
    char *land = nullptr;
    size_t land_cap = 0;
    bool land_ok = false;
    std::vector<int32_t> ref_lens;  // host copy (sizes the LDS window)
    // references this pileup counts (mh_pileup_only; empty: all): the units
    // of any other are skipped and its counters stay zero
    std::vector<uint8_t> only;
    int32_t *sel = nullptr;         // references of a multi-GPU exchange
    int sel_cap = 0;
    int32_t *win_map = nullptr;     // k_pileup: per reference (LDS window word offset, -1 none, -2 skipped; positions)
    int win_map_cap = 0;
    char *ins_scratch = nullptr;    // per-wave merged-insertion scratch of k_pileup
    int64_t ins_scratch_bytes = 0;
    // k_pileup block shapes already sized by the occupancy query: key (source,
    // LDS bytes before the staging areas, staging bytes per wave) -> waves
    // per block, resident blocks per CU
    std::map<std::tuple<int, int64_t, int>, std::pair<int, int>> shapes;
    // device aggregation of the token events (mh_pileup_events): an
    // open-addressing table of representative event + count per distinct
    // (ref, pos, token), and the list of used slots
    int32_t *tok_slot = nullptr;    // event index + 1, 0 empty
    uint32_t *tok_cnt = nullptr;
    int32_t *tok_used = nullptr;    // [0] = number of distinct keys, then their slots
    int64_t tok_cap = 0;            // slots (power of two)
    int32_t *tok_meta = nullptr;    // gather: per distinct key (ref, pos, off, len, count)
    char *tok_bytes = nullptr;
    int64_t tok_meta_cap = 0, tok_bytes_cap = 0;
    char *tok_pin = nullptr;        // pinned staging of the gather's first round trip
    size_t tok_pin_cap = 0;
};

// ---- kernels' host-side launchers (defined in the .hip files) ----------
hipError_t launch_pack_reads(DevReads &r, const uint8_t *d_seq, const uint8_t *d_qual,
                             const int64_t *d_src_off, hipStream_t s);
int run_map(struct Ctx &c, const mh_params &par);
int run_probe_ext(struct Ctx &c, const mh_params &par, int n, const int32_t *items, int32_t *out);
// the per-reference tallies of the last mapping pass on the host (one copy
// per pass); nullptr on a copy error
const int64_t *map_stats_host(struct Ctx &c);
int run_pileup(struct Ctx &c, int source, int q_cutoff);
// distinct (ref, pos, token) keys of the last pileup's events with their
// counts, aggregated on the device; tokens concatenated in `bytes` at `off`
int run_token_aggregate(struct Ctx &c, int64_t n_events, int64_t pool_used,
                        std::vector<int32_t> &meta, std::string &bytes);
int run_gotoh(struct Ctx &c, const char *s1, const char *s2, int gop, int gep, int is_global,
              const char *alphabet, const int *matrix, char *out1, char *out2, int cap,
              int *score);
int run_gotoh_batch(struct Ctx &c, int count, const char *const *s1, const char *const *s2,
                    int gop, int gep, int is_global, const char *alphabet, const int *matrix,
                    char *const *out1, char *const *out2, const int *cap, int *score,
                    int *status);
int run_gotoh_distance_batch(struct Ctx &c, int count, const char *const *s1, const char *const *s2,
                             const char *const *text, int gop, int gep, int is_global,
                             const char *alphabet, const int *matrix, int *dist, int *score,
                             int *status);

// Read names (QNAMEs) in one byte pool: name r is bytes off[r] .. off[r + 1]
// (one allocation for millions of names instead of one string each).
struct NameTable {
    TextBuf pool;   // not zero-filled when sized (the names are copied in by many threads)
    std::vector<int64_t> off{0};
    size_t size() const { return off.size() - 1; }
    std::string_view operator[](size_t r) const
    {
        return std::string_view(pool.data() + off[r], (size_t)(off[r + 1] - off[r]));
    }
    void clear() { pool.clear(); off.assign(1, 0); }
    void assign(const char *const *names, int64_t n)
    {
        clear();
        off.resize((size_t)n + 1);
        for (int64_t r = 0; r < n; ++r) off[r + 1] = off[r] + (int64_t)strlen(names[r]);
        pool.resize((size_t)off[n]);
        for (int64_t r = 0; r < n; ++r) memcpy(&pool[off[r]], names[r], (size_t)(off[r + 1] - off[r]));
    }
    void swap(NameTable &o) { pool.swap(o.pool); off.swap(o.off); }
};

struct ProfEntry {
    double ms = 0.0;
    int64_t launches = 0;
};

struct ProfPending {
    const char *name;
    hipEvent_t a, b;
};

struct S2AState;      // mh_sam2aln.h
struct CensorState;   // mh_censor.hip
struct A2CState;      // mh_a2c.hip

// Capacities a test can impose on the grow-and-retry buffers
// (mh_test_set_capacities); 0 keeps the library's own sizing.  Each call that
// sizes one of these buffers starts it at the imposed capacity, so every pass
// that needs more goes through the retry.
struct TestCaps {
    int64_t cigar_pool_words = 0;   // MapState::pool
    int64_t pile_events = 0;        // PileState::ev
    int64_t pile_event_bytes = 0;   // PileState::ev_pool
    int64_t token_bytes = 0;        // PileState::tok_bytes
    int64_t gotoh_wait_ticks = 0;   // k_gotoh's first-attempt wait limit (0: the default)
};

// retries taken by the grow-and-retry paths (mh_retry_counts)
enum { RETRY_CIGAR_POOL = 0, RETRY_PILE_EVENTS = 1, RETRY_TOKEN_BYTES = 2, RETRY_GOTOH_WAIT = 3,
       RETRY_KINDS = 4 };

struct Ctx {
    int device = 0;
    TestCaps test_caps;
    int64_t retries[RETRY_KINDS] = {0, 0, 0, 0};
    int n_cu = 0;                    // compute units of the device (launch sizing)
    // per-kernel timing with HIP events on `stream` (mh_profile)
    bool prof = false;
    std::map<std::string, ProfEntry> prof_acc;
    std::vector<ProfPending> prof_pending;
    hipStream_t stream = nullptr;
    DevReads reads;
    NameTable names;                 // QNAMEs for SAM text
    std::vector<std::string> host_seq, host_qual; // kept only when names are
    DevIndex index;
    MapState map;
    RowState rows;
    PileState pile;
    // per-length tables (host-computed, uploaded): seed interval, min score,
    // n ceil, DP band half-width
    int32_t *len_tab = nullptr;      // [4][MAXLEN + 1]
    S2AState *s2a = nullptr;         // sam2aln rows and results (mh_sam2aln_csv)
    CensorState *censor = nullptr;   // censored FASTQ of the last mh_censor_fastq
    A2CState **a2c = nullptr;        // aln2counts row tables (mh_a2c_*), one per slot
    int64_t len_tab_key = -1;        // len_tab_key() of the parameters the tables hold
    // every parameter set's tables seen so far (a prelim pass and a remap
    // pass alternate end-to-end and local; the band column's gap counts take
    // a few hundred microseconds of host time to rebuild): key -> device copy
    std::map<int64_t, int32_t *> len_tabs;
    // k_gotoh's device scratch (traceback planes etc.), grown on demand and
    // kept up to 1 GiB: a hipMalloc / hipFree pair per call cost more than
    // the kernel.  The mutex serialises callers of one context (ctypes
    // releases the GIL).
    char *gotoh_buf = nullptr;
    size_t gotoh_cap = 0;
    std::mutex gotoh_mutex;
};

void set_error(const char *fmt, ...);
Ctx *ctx_of(mh_ctx *ctx);          // the context behind a C-ABI handle
void s2a_free(Ctx &c);
void censor_free(Ctx &c);
void a2c_free(Ctx &c);
// bracket one kernel launch on c.stream when profiling is on
int prof_begin(Ctx &c, const char *name);
void prof_end(Ctx &c, int slot);
void prof_flush(Ctx &c);   // after a stream sync: fold pending events
int hip_fail(hipError_t e, const char *what);
// a blocking copy ordered on c.stream: the stream is non-blocking, so a plain
// hipMemcpy (legacy null stream) is not ordered after its kernels
hipError_t copy_sync(Ctx &c, void *dst, const void *src, size_t bytes, hipMemcpyKind kind);

}  // namespace mh

#define MH_HIP(call)                                                  \
    do {                                                              \
        hipError_t e_ = (call);                                       \
        if (e_ != hipSuccess) return ::mh::hip_fail(e_, #call);       \
    } while (0)
