// mh_api.cpp -- host side of libmicall_hip.so: the extern "C" entry points of
// include/micall_hip.h, context and device-memory management, the seed index
// build (bowtie2-build's job), FASTQ ingest and SAM/CSV text emission.
#include <errno.h>
#include <fcntl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>
#include <zlib.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cmath>
#include <cstdarg>
#include <cstdio>
#include <cstring>
#include <memory>
#include <new>
#include <string>
#include <condition_variable>
#include <deque>
#include <exception>
#include <mutex>
#include <functional>
#include <string_view>
#include <thread>
#include <unordered_map>
#include <vector>

#include "mh_fastq.h"
#include "mh_gunzip.h"
#include "mh_internal.h"
#include "mh_text.h"

#include <map>
#include <tuple>

namespace mh {

static thread_local char g_err[1024];

void set_error(const char *fmt, ...)
{
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(g_err, sizeof(g_err), fmt, ap);
    va_end(ap);
}

static std::string last_error_text() { return std::string(g_err); }

int hip_fail(hipError_t e, const char *what)
{
    set_error("HIP error %d (%s) in %s", (int)e, hipGetErrorString(e), what);
    return -4;
}

hipError_t copy_sync(Ctx &c, void *dst, const void *src, size_t bytes, hipMemcpyKind kind)
{
    hipError_t e = hipMemcpyAsync(dst, src, bytes, kind, c.stream);
    return e == hipSuccess ? hipStreamSynchronize(c.stream) : e;
}

int prof_begin(Ctx &c, const char *name)
{
    if (!c.prof) return -1;
    ProfPending p{name, nullptr, nullptr};
    if (hipEventCreate(&p.a) != hipSuccess || hipEventCreate(&p.b) != hipSuccess) return -1;
    hipEventRecord(p.a, c.stream);
    c.prof_pending.push_back(p);
    return (int)c.prof_pending.size() - 1;
}

void prof_end(Ctx &c, int slot)
{
    if (slot < 0 || slot >= (int)c.prof_pending.size()) return;
    hipEventRecord(c.prof_pending[slot].b, c.stream);
}

void prof_flush(Ctx &c)
{
    for (auto &p : c.prof_pending) {
        float ms = 0.f;
        if (hipEventSynchronize(p.b) == hipSuccess && hipEventElapsedTime(&ms, p.a, p.b) == hipSuccess) {
            ProfEntry &e = c.prof_acc[p.name];
            e.ms += ms;
            e.launches += 1;
        }
        hipEventDestroy(p.a);
        hipEventDestroy(p.b);
    }
    c.prof_pending.clear();
}

// ---- per-length tables, same formulas as oracle/og_mapper.c --------------
static int seed_interval(int mode, int len)
{
    const double f = mode == MH_LOCAL ? 0.75 : 1.15;
    int iv = (int)(1.0 + f * std::sqrt((double)len) + 0.5);
    return iv < 1 ? 1 : iv;
}

static int min_score(int mode, int len)
{
    if (mode == MH_LOCAL) {
        double v = 20.0 + 8.0 * std::log((double)(len > 0 ? len : 1));
        long s = (long)v;
        return (int)(s < 0 ? 0 : s);
    }
    long s = (long)(-0.6 + -0.6 * (double)len);
    return (int)(s > 0 ? 0 : s);
}

static int n_ceil(int len) { return (int)(0.0 + 0.15 * (double)len); }

// gaps of one kind an alignment can hold and still reach minsc from the
// perfect score (bowtie2 Scoring::maxReadGaps / maxRefGaps)
static int max_gaps(int perfect, int minsc, int oe, int ex)
{
    int sc = perfect, num = 0;
    while (sc >= minsc) {
        sc -= num == 0 ? oe : ex;
        ++num;
    }
    return num - 1;
}

// DP band half-width: max(read gaps, ref gaps) capped at maxhalf
// (DynProgFramer::frameSeedExtensionRect; oracle og_band_half)
static int band_half(const mh_params &p, int len)
{
    const int perfect = p.mode == MH_LOCAL ? 2 * len : 0;
    const int minsc = min_score(p.mode, len);
    const int gd = max_gaps(perfect, minsc, p.rdg_open + p.rdg_ext, p.rdg_ext);
    const int gi = max_gaps(perfect, minsc, p.rfg_open + p.rfg_ext, p.rfg_ext);
    int h = gd > gi ? gd : gi;
    if (h > MAXHALF) h = MAXHALF;
    return h < 0 ? 0 : h;
}

static int prepare_len_tab(Ctx &c, const mh_params &par)
{
    const int64_t key = len_tab_key(par);
    if (c.len_tab && c.len_tab_key == key) return 0;
    const auto hit = c.len_tabs.find(key);
    if (hit != c.len_tabs.end()) {
        c.len_tab = hit->second;
        c.len_tab_key = key;
        return 0;
    }
    std::vector<int32_t> t(4 * (MAXLEN + 1));
    for (int l = 0; l <= MAXLEN; ++l) {
        t[l] = seed_interval(par.mode, l);
        t[(MAXLEN + 1) + l] = min_score(par.mode, l);
        t[2 * (MAXLEN + 1) + l] = n_ceil(l);
        t[3 * (MAXLEN + 1) + l] = band_half(par, l);
    }
    int32_t *d = nullptr;
    MH_HIP(hipMalloc(&d, sizeof(int32_t) * t.size()));
    c.len_tabs[key] = d;
    MH_HIP(copy_sync(c, d, t.data(), sizeof(int32_t) * t.size(), hipMemcpyHostToDevice));
    c.len_tab = d;
    c.len_tab_key = key;
    return 0;
}

// ---- host copies of the reads (SAM SEQ/QUAL text) ------------------------
// Host bytes that are not zero-filled on allocation (the ingest writes
// every byte it keeps; a std::vector's value-initialisation of a GB buffer
// is a serial memset the ingest does not need).
struct Bytes {
    std::unique_ptr<char[], BigDeleter> p{nullptr, BigDeleter{}};
    size_t n = 0;
    void alloc(size_t k)
    {
        p = std::unique_ptr<char[], BigDeleter>(big_alloc(k > 0 ? k : 1), BigDeleter{k > 0 ? k : 1});
        n = k;
    }
    void assign(const uint8_t *a, const uint8_t *b) { alloc((size_t)(b - a)); if (b > a) std::memcpy(p.get(), a, n); }
    uint8_t *data() { return (uint8_t *)p.get(); }
    const uint8_t *data() const { return (const uint8_t *)p.get(); }
    size_t size() const { return n; }
};

// the reads as text on the host (SEQ / QUAL of the SAM rows)
struct HostReads {
    Bytes seq, qual;
    std::vector<int64_t> off;
    std::vector<int32_t> len;
};

struct CtxEx : Ctx {
    HostReads host;
    // index cache: large (fixed seed-set) indexes are kept by content signature
    std::vector<DevIndex> cache;
    // the reference bytes of each cache entry (every sequence and its NUL, in
    // order): a signature hit is used only when they compare equal
    std::vector<std::string> cache_text;
    std::vector<Rec> rec_cache;
    std::vector<int32_t> csv_rows_info;   // per prelim.csv row: name id, flag, max M run, ref
    std::vector<int32_t> csv_present;     // compact ref id -> index into the @SQ list
    std::vector<std::string> csv_unknown; // names outside @SQ, by -1 - name id
    int64_t fastq_lines1 = -1;            // newlines in FASTQ 1 (LineCounter, externals.py:206)
    DevIndex small;                       // reusable buffers of the non-cached (consensus) index
    // insertion tokens of the last pileup, aggregated: (ref, pos, token) -> count
    int64_t tok_gen = -1;
    std::vector<int32_t> tok_ref, tok_pos, tok_off, tok_len;
    std::vector<int64_t> tok_count;
    std::string tok_pool;
    // pinned staging for the pileup fetches: several copies on the stream,
    // one synchronisation (pageable hipMemcpy synchronises every copy)
    void *pin = nullptr;
    size_t pin_cap = 0;
    // mh_format_rows: the text of a size query, kept for the copy after it
    int64_t map_gen = 0;                  // bumped by every mh_map
    uint64_t fmt_key = 0;
    bool fmt_valid = false;
    std::vector<TextBuf> fmt_chunks;
    // host wall time per phase of the file-to-file path (mh_phase_times)
    double phase_ms[MH_PHASES] = {};
    // mh_format_segments: the formatted chunks and the byte offset of every
    // segment bound in their concatenation, kept for mh_write_segments
    std::vector<TextBuf> seg_chunks;
    std::vector<int64_t> seg_at;
    // device buffers of the reads (both DevReads) and the upload staging,
    // kept between loads and grown only: bytes behind each pointer
    std::unordered_map<const void *, size_t> rcap;
    uint8_t *stage_seq = nullptr, *stage_qual = nullptr;
    int64_t *stage_off = nullptr;
};

// p sized to at least `need` bytes: kept when it already is, else freed and
// allocated again (cap: CtxEx::rcap)
template <class T>
static hipError_t grow_dev(CtxEx &c, T *&p, size_t need)
{
    if (need == 0) need = 1;
    if (p) {
        auto it = c.rcap.find((const void *)p);
        if (it != c.rcap.end() && it->second >= need) return hipSuccess;
        if (it != c.rcap.end()) c.rcap.erase(it);
        hipFree(p);
        p = nullptr;
    }
    void *q = nullptr;
    const hipError_t e = hipMalloc(&q, need);
    if (e != hipSuccess) return e;
    p = (T *)q;
    c.rcap[(const void *)q] = need;
    return hipSuccess;
}

static void free_index(DevIndex &ix)
{
    hipFree(ix.blob);
    ix = DevIndex{};
}

static void free_reads(DevReads &r)
{
    hipFree(r.seq2); hipFree(r.nmask); hipFree(r.qual); hipFree(r.off); hipFree(r.len);
    r = DevReads{};
}

static uint8_t code_of(char ch)
{
    switch (ch) {
    case 'A': case 'a': return 0;
    case 'C': case 'c': return 1;
    case 'G': case 'g': return 2;
    case 'T': case 't': return 3;
    default: return 4;
    }
}

// Cache key of a reference set: every sequence's length and bytes, 8 bytes
// per multiply-xorshift step (the byte-wise FNV this replaces spent ~0.5 ms
// per prelim pass on the 590 kb of seeds just to find the cached index)
static inline uint64_t mix64(uint64_t h, uint64_t w)
{
    h = (h ^ w) * 0x9E3779B97F4A7C15ull;
    return h ^ (h >> 29);
}

static uint64_t signature(int n, const char *const *seqs, int seedlen)
{
    uint64_t h = 1469598103934665603ull ^ (uint64_t)seedlen;
    for (int r = 0; r < n; ++r) {
        const size_t len = std::strlen(seqs[r]);
        h = mix64(h, (uint64_t)len);
        // four independent chains over 32-byte steps (the 74 seeds are
        // 0.74 MB, hashed on every prelim pass), folded in order
        uint64_t q[4] = {h, h ^ 1, h ^ 2, h ^ 3};
        size_t i = 0;
        for (; i + 32 <= len; i += 32)
            for (int k = 0; k < 4; ++k) {
                uint64_t w;
                std::memcpy(&w, seqs[r] + i + 8 * k, 8);
                q[k] = mix64(q[k], w);
            }
        h = mix64(mix64(mix64(mix64(h, q[0]), q[1]), q[2]), q[3]);
        for (; i + 8 <= len; i += 8) {
            uint64_t w;
            std::memcpy(&w, seqs[r] + i, 8);
            h = mix64(h, w);
        }
        uint64_t tail = 0;
        std::memcpy(&tail, seqs[r] + i, len - i);
        h = mix64(h, tail ^ 0xffull << 56);
    }
    return mix64(h, (uint64_t)n);
}

static void par_for(int nt, const std::function<void(int)> &fn);
int s2a_threads();   // mh_s2a_host.cpp: host worker count

static int build_index(DevIndex &ix, int n_refs, const char *const *seqs, int seedlen)
{
    // MH_INDEX_TRACE=1: phase times to stderr
    static const bool trace = getenv("MH_INDEX_TRACE") && *getenv("MH_INDEX_TRACE") == '1';
    const auto tb = std::chrono::steady_clock::now();
    auto mark = [&](const char *what) {
        if (trace)
            fprintf(stderr, "index %s %.2f ms\n", what,
                    std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - tb).count());
    };
    struct E { uint64_t key; int32_t ref, pos; };
    std::vector<int64_t> ref_off(n_refs);
    std::vector<int32_t> ref_len(n_refs);
    int64_t total_len = 0;
    for (int r = 0; r < n_refs; ++r) {
        ref_len[r] = (int)std::strlen(seqs[r]);
        ref_off[r] = total_len;
        total_len += ref_len[r];
    }
    std::vector<uint8_t> codes((size_t)total_len);
    // every reference's seeds by its own thread (references are independent),
    // then concatenated in reference order
    const int nt = std::max(1, std::min<int>(s2a_threads(), n_refs));
    std::vector<std::vector<E>> per(n_refs);
    mark("pre");
    std::vector<double> t_start((size_t)nt, 0.0);
    {
        std::atomic<int> next(0);
        par_for(nt, [&](int t) {
            t_start[(size_t)t] = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - tb).count();
            for (int r; (r = next.fetch_add(1)) < n_refs;) {
                const int L = ref_len[r];
                uint8_t *cr = codes.data() + ref_off[r];
                std::vector<E> &v = per[r];
                v.reserve(L > seedlen ? (size_t)(L - seedlen + 1) : 0);
                uint64_t key = 0;
                int last_n = -1;
                for (int p = 0; p < L; ++p) {
                    const uint8_t c = code_of(seqs[r][p]);
                    cr[p] = c;
                    if (c > 3) last_n = p;
                    // little-endian 2-bit packing: base x of the window at bits 2x+1:2x
                    key = (key >> 2) | ((uint64_t)(c & 3) << (2 * (seedlen - 1)));
                    if (p >= seedlen - 1 && last_n <= p - seedlen) v.push_back({key, r, p - seedlen + 1});
                }
            }
        });
    }
    if (trace) {
        double mx = 0;
        for (double x : t_start) mx = std::max(mx, x);
        fprintf(stderr, "index thread starts: last at %.2f ms\n", mx);
    }
    mark("seeds");
    std::vector<E> ent;
    {
        size_t n = 0;
        for (auto &v : per) n += v.size();
        ent.reserve(n);
        for (auto &v : per) { ent.insert(ent.end(), v.begin(), v.end()); std::vector<E>().swap(v); }
    }
    // (key, ref, pos) order, a total order (no two entries share ref and
    // pos), so an unstable sort gives it (std::stable_sort's buffer cost
    // ~0.1 ms per consensus index of a few thousand entries)
    auto less = [](const E &a, const E &b) {
        return a.key != b.key ? a.key < b.key : a.ref != b.ref ? a.ref < b.ref : a.pos < b.pos;
    };
    {   // sorted in parallel chunks, then merged pairwise
        const int ns = ent.size() < 65536 ? 1 : s2a_threads();
        std::vector<size_t> b((size_t)ns + 1);
        for (int t = 0; t <= ns; ++t) b[(size_t)t] = ent.size() * (size_t)t / (size_t)ns;
        par_for(ns, [&](int t) { std::sort(ent.begin() + b[(size_t)t], ent.begin() + b[(size_t)t + 1], less); });
        for (int w = 1; w < ns; w *= 2) {
            std::vector<std::pair<int, int>> jobs;
            for (int t = 0; t + w < ns; t += 2 * w) jobs.push_back({t, std::min(t + 2 * w, ns)});
            par_for((int)jobs.size(), [&](int j) {
                const int a = jobs[(size_t)j].first, m = a + w, z = jobs[(size_t)j].second;
                std::inplace_merge(ent.begin() + b[(size_t)a], ent.begin() + b[(size_t)m], ent.begin() + b[(size_t)z], less);
            });
        }
    }
    mark("sort");
    size_t nkeys = 0;
    for (size_t i = 0; i < ent.size(); ++i) if (i == 0 || ent[i].key != ent[i - 1].key) ++nkeys;
    uint64_t cap = 1024;
    while (cap < 2 * nkeys) cap <<= 1;
    // one 16-B entry per slot: key (two words, EMPTY = ~0), start, count
    std::vector<uint4> hent(cap, make_uint4(~0u, ~0u, 0u, 0u));
    std::vector<int2> hits(ent.size() ? ent.size() : 1);
    for (size_t i = 0; i < ent.size();) {
        size_t j = i + 1;
        while (j < ent.size() && ent[j].key == ent[i].key) ++j;
        uint64_t h = hash_key(ent[i].key) & (cap - 1);
        while (((uint64_t)hent[h].x | ((uint64_t)hent[h].y << 32)) != HEMPTY) h = (h + 1) & (cap - 1);
        hent[h] = make_uint4((uint32_t)ent[i].key, (uint32_t)(ent[i].key >> 32), (uint32_t)i, (uint32_t)(j - i));
        i = j;
    }
    for (size_t i = 0; i < ent.size(); ++i) hits[i] = make_int2(ent[i].ref, ent[i].pos);
    mark("hash");
    ix.n_refs = n_refs;
    ix.seedlen = seedlen;
    ix.total = (int64_t)codes.size();
    ix.hmask = cap - 1;
    codes.resize(codes.size() + 64, 4);
    // packed copies for word-wise window reads (k_rescue), with the padding
    std::vector<uint32_t> code2((codes.size() + 15) / 16 + 2, 0), ncode((codes.size() + 31) / 32 + 2, 0);
    for (size_t j = 0; j < codes.size(); ++j) {
        if (codes[j] > 3) ncode[j >> 5] |= 1u << (j & 31);
        else code2[j >> 4] |= (uint32_t)codes[j] << (2 * (j & 15));
    }
    std::vector<uint32_t> cplane(2 * ((codes.size() + 31) / 32 + 2), 0);
    for (size_t j = 0; j < codes.size(); ++j) {
        const uint32_t c = codes[j] > 3 ? 0u : codes[j];
        cplane[2 * (j >> 5)] |= (c & 1u) << (j & 31);
        cplane[2 * (j >> 5) + 1] |= (c >> 1) << (j & 31);
    }
    // one blob: codes, ref_off, ref_len, hent, hits, code2, ncode, cplane
    // (256-B aligned parts), staged on the host and uploaded with one copy
    auto al = [](size_t x) { return (x + 255) & ~(size_t)255; };
    constexpr int NP = 8;
    const size_t sz[NP] = {codes.size(), sizeof(int64_t) * (size_t)n_refs, sizeof(int32_t) * (size_t)n_refs,
                           sizeof(uint4) * cap, sizeof(int2) * hits.size(), sizeof(uint32_t) * code2.size(),
                           sizeof(uint32_t) * ncode.size(), sizeof(uint32_t) * cplane.size()};
    const void *src[NP] = {codes.data(), ref_off.data(), ref_len.data(), hent.data(), hits.data(),
                           code2.data(), ncode.data(), cplane.data()};
    size_t at[NP], total = 0;
    for (int x = 0; x < NP; ++x) { at[x] = total; total += al(sz[x]); }
    if ((int64_t)total > ix.cap_blob) {   // (re)allocate only when it does not fit
        hipFree(ix.blob);
        ix.blob = nullptr;
        ix.cap_blob = 0;
        MH_HIP(hipMalloc(&ix.blob, total));
        ix.cap_blob = (int64_t)total;
    }
    mark("planes+alloc");
    std::vector<uint8_t> stage(total);
    for (int x = 0; x < NP; ++x) if (sz[x]) std::memcpy(stage.data() + at[x], src[x], sz[x]);
    mark("stage");
    uint8_t *d = (uint8_t *)ix.blob;
    ix.codes = d + at[0];
    ix.ref_off = (int64_t *)(d + at[1]);
    ix.ref_len = (int32_t *)(d + at[2]);
    ix.hent = (uint4 *)(d + at[3]);
    ix.hits = (int2 *)(d + at[4]);
    ix.code2 = (uint32_t *)(d + at[5]);
    ix.ncode = (uint32_t *)(d + at[6]);
    ix.cplane = (uint32_t *)(d + at[7]);
    // callers synchronise the context stream first (mh_index_build)
    MH_HIP(hipMemcpy(ix.blob, stage.data(), total, hipMemcpyHostToDevice));
    mark("upload");
    return 0;
}

// Upload n reads (text at seq / qual + offsets) and pack them on the device.
// keep_host copies the text to `host`; `adopt` (the FASTQ ingest, whose
// buffers are already laid out) moves its buffers there instead.
static int load_reads(CtxEx &c, DevReads &dst, HostReads &host, int64_t n, int paired,
                      const uint8_t *seq, const uint8_t *qual, const int64_t *offsets,
                      const int32_t *lens, bool keep_host, HostReads *adopt = nullptr)
{
    if (n < 0 || (paired && (n & 1))) { set_error("reads: bad count"); return -3; }
    int max_len = 0;
    int64_t src_total = 0;
    for (int64_t r = 0; r < n; ++r) {
        if (lens[r] < 0 || lens[r] > MAXLEN) {
            set_error("reads: read %lld has length %d (max %d)", (long long)r, lens[r], MAXLEN);
            return -3;
        }
        max_len = std::max(max_len, (int)lens[r]);
        src_total = std::max(src_total, offsets[r] + lens[r]);
    }
    std::vector<int64_t> off(n > 0 ? n : 1);
    int64_t total = 0;
    for (int64_t r = 0; r < n; ++r) {
        off[r] = total;
        total += ((int64_t)lens[r] + 31) / 32 * 32;
    }
    // the device buffers of the last load are reused when large enough
    // (a chain of samples in one process frees and maps GBs otherwise)
    MH_HIP(hipStreamSynchronize(c.stream));   // nothing may still read the old reads
    dst.n = n;
    dst.paired = paired;
    dst.max_len = max_len;
    dst.total_bases = total;
    MH_HIP(grow_dev(c, dst.seq2, sizeof(uint32_t) * (total / 16 + 8)));
    MH_HIP(grow_dev(c, dst.nmask, sizeof(uint32_t) * (total / 32 + 8)));
    MH_HIP(grow_dev(c, dst.qual, (size_t)total + 64));
    MH_HIP(grow_dev(c, dst.off, sizeof(int64_t) * (n > 0 ? n : 1)));
    MH_HIP(grow_dev(c, dst.len, sizeof(int32_t) * (n > 0 ? n : 1)));
    MH_HIP(hipMemsetAsync(dst.seq2, 0, sizeof(uint32_t) * (total / 16 + 8), c.stream));
    MH_HIP(hipMemsetAsync(dst.nmask, 0, sizeof(uint32_t) * (total / 32 + 8), c.stream));
    if (n > 0) {
        MH_HIP(hipMemcpyAsync(dst.off, off.data(), sizeof(int64_t) * n, hipMemcpyHostToDevice, c.stream));
        MH_HIP(hipMemcpyAsync(dst.len, lens, sizeof(int32_t) * n, hipMemcpyHostToDevice, c.stream));
        MH_HIP(grow_dev(c, c.stage_seq, (size_t)src_total + 1));
        MH_HIP(grow_dev(c, c.stage_qual, (size_t)src_total + 1));
        MH_HIP(grow_dev(c, c.stage_off, sizeof(int64_t) * (size_t)n));
        MH_HIP(hipMemcpyAsync(c.stage_seq, seq, src_total, hipMemcpyHostToDevice, c.stream));
        MH_HIP(hipMemcpyAsync(c.stage_qual, qual, src_total, hipMemcpyHostToDevice, c.stream));
        MH_HIP(hipMemcpyAsync(c.stage_off, offsets, sizeof(int64_t) * n, hipMemcpyHostToDevice, c.stream));
        MH_HIP(launch_pack_reads(dst, c.stage_seq, c.stage_qual, c.stage_off, c.stream));
        MH_HIP(hipStreamSynchronize(c.stream));
    }
    if (adopt) {
        host = std::move(*adopt);
    } else if (keep_host) {
        host.seq.assign(seq, seq + src_total);
        host.qual.assign(qual, qual + src_total);
        host.off.assign(offsets, offsets + n);
        host.len.assign(lens, lens + n);
    }
    return 0;
}

// bowtie2 read name: header up to the first whitespace, /1 or /2 dropped
// for mates; the span [*at, *at + *len) of the header h
static inline void qname_span(const char *h, size_t n, bool paired, size_t *at, size_t *len)
{
    size_t a = (n && h[0] == '@') ? 1 : 0;
    while (a < n && (h[a] == ' ' || h[a] == '\t')) ++a;
    size_t b = a;
    // 8 bytes at a time while none of them is <= ' ' (space, tab and '\r'
    // all are): the classic has-less-than test, exact for bytes < 0x80 and
    // never missing a small byte (a byte >= 0x80 only sends the word to the
    // byte-wise loop)
    constexpr uint64_t ONES = 0x0101010101010101ull, HIGH = 0x8080808080808080ull;
    while (b + 8 <= n) {
        uint64_t w;
        std::memcpy(&w, h + b, 8);
        if (((w - ONES * 0x21) | w) & HIGH) break;
        b += 8;
    }
    while (b < n && h[b] != ' ' && h[b] != '\t' && h[b] != '\r') ++b;
    if (paired && b - a > 2 && h[b - 2] == '/' && (h[b - 1] == '1' || h[b - 1] == '2')) b -= 2;
    *at = a;
    *len = b - a;
}

// A FASTQ file decoded to text and indexed in place: per record the start
// and length of its header, sequence and quality lines.
struct Fastq {
    TextBuf data;
    std::vector<int64_t> name_at, seq_at, qual_at;
    std::vector<int32_t> name_len, len, qual_len;
    size_t size() const { return len.size(); }
};

int s2a_threads();   // mh_s2a_host.cpp: host worker count

// fn(0) .. fn(nt-1) on nt threads (the caller's is thread 0).  An
// exception on any thread (bad_alloc from a text buffer) is kept, every
// thread is joined, then the first one is rethrown on the caller's thread:
// none escapes a std::thread (that would terminate the process).
static void par_for(int nt, const std::function<void(int)> &fn)
{
    if (nt <= 1) { fn(0); return; }
    std::mutex mu;
    std::exception_ptr first;
    auto guarded = [&](int t) {
        try {
            fn(t);
        } catch (...) {
            std::lock_guard<std::mutex> lk(mu);
            if (!first) first = std::current_exception();
        }
    };
    std::vector<std::thread> th;
    th.reserve((size_t)nt - 1);
    try {
        for (int t = 1; t < nt; ++t) th.emplace_back(guarded, t);
    } catch (...) {           // thread creation failed: run the rest here
        for (int t = (int)th.size() + 1; t < nt; ++t) guarded(t);
    }
    guarded(0);
    for (auto &x : th) x.join();
    if (first) std::rethrow_exception(first);
}

// The whole (gzip or plain) file; every concatenated gzip member is decoded
// (as gzread does), in parallel when there are several (mh_gunzip.cpp).
static int slurp(const char *path, TextBuf &data)
{
    data.clear();
    const int fd = open(path, O_RDONLY | O_CLOEXEC);
    if (fd < 0) { set_error("cannot open FASTQ %s", path); return -3; }
    struct stat st;
    if (fstat(fd, &st) != 0) { close(fd); set_error("cannot stat FASTQ %s", path); return -3; }
    const int64_t sz = (int64_t)st.st_size;
    // the file mapped (no copy); a file that cannot be mapped is read
    const uint8_t *raw = nullptr;
    void *map = MAP_FAILED;
    TextBuf copy;
    if (sz > 0 && S_ISREG(st.st_mode)) map = mmap(nullptr, (size_t)sz, PROT_READ, MAP_PRIVATE, fd, 0);
    if (map != MAP_FAILED) {
        raw = (const uint8_t *)map;
    } else if (sz > 0) {
        copy.resize((size_t)sz);
        int64_t got = 0;
        while (got < sz) {
            const ssize_t r = pread(fd, copy.data() + got, (size_t)(sz - got), (off_t)got);
            if (r <= 0) break;
            got += r;
        }
        if (got != sz) { close(fd); set_error("cannot read FASTQ %s", path); return -3; }
        raw = (const uint8_t *)copy.data();
    }
    close(fd);
    int rc = 0;
    if (sz >= 2 && raw[0] == 0x1f && raw[1] == 0x8b) {
        std::string why;
        if (gunzip_buffer(raw, sz, data, why)) {
            set_error("gzip error reading %s: %s", path, why.c_str());
            rc = -3;
        }
    } else if (sz > 0) {
        if (map != MAP_FAILED) data.assign((const char *)raw, (size_t)sz);
        else data.swap(copy);
    }
    if (map != MAP_FAILED) munmap(map, (size_t)sz);
    return rc;
}

// Index the FASTQ records of fq.data (blank lines between records skipped,
// '\r' before '\n' dropped): the newline scan runs on host threads.
static int index_fastq(Fastq &fq, const char *path, int64_t *newlines)
{
    const TextBuf &data = fq.data;
    const int64_t n = (int64_t)data.size();
    const char *D = data.data();
    const int nt = std::max(1, std::min(s2a_threads(), (int)(n >> 20) + 1));
    std::vector<std::vector<int64_t>> ls(nt);
    par_for(nt, [&](int t) {
        const int64_t a = n * t / nt, b = n * (t + 1) / nt;
        const char *p = D + a, *e = D + b;
        ls[t].reserve((size_t)((b - a) / 60 + 16));
        while (p < e) {
            const char *nl = (const char *)memchr(p, '\n', (size_t)(e - p));
            if (!nl) break;
            ls[t].push_back(nl - D);
            p = nl + 1;
        }
    });
    std::vector<int64_t> nlpos;
    std::vector<size_t> at((size_t)nt + 1, 0);
    for (int t = 0; t < nt; ++t) at[(size_t)t + 1] = at[(size_t)t] + ls[(size_t)t].size();
    nlpos.resize(at[(size_t)nt]);
    std::vector<int64_t> before((size_t)nt, -1);   // the last newline before part t
    for (int t = 1; t < nt; ++t)
        before[(size_t)t] = ls[(size_t)t - 1].empty() ? before[(size_t)t - 1] : ls[(size_t)t - 1].back();
    std::atomic<int> blank(0);   // an empty line (or one holding only '\r') anywhere
    par_for(nt, [&](int t) {
        const auto &v = ls[(size_t)t];
        if (!v.empty()) std::memcpy(nlpos.data() + at[(size_t)t], v.data(), sizeof(int64_t) * v.size());
        int64_t prev = before[(size_t)t];
        bool b = false;
        for (int64_t x : v) {
            const int64_t st = prev + 1;
            if (x == st || (x == st + 1 && D[st] == '\r')) b = true;
            prev = x;
        }
        if (b) blank = 1;
    });
    std::vector<std::vector<int64_t>>().swap(ls);
    if (newlines) *newlines = (int64_t)nlpos.size();
    // line k spans [start_k, end_k) without '\n' / trailing '\r'
    const int64_t nl = (int64_t)nlpos.size() + (nlpos.empty() || nlpos.back() + 1 < n ? 1 : 0);
    auto lstart = [&](int64_t k) { return k == 0 ? (int64_t)0 : nlpos[k - 1] + 1; };
    auto lend = [&](int64_t k) {
        int64_t e = k < (int64_t)nlpos.size() ? nlpos[k] : n;
        if (e > lstart(k) && D[e - 1] == '\r') --e;
        return e;
    };
    // first line of each record: every fourth line when no line is empty
    // (the last line, after the final newline, is checked on its own)
    std::vector<int64_t> rec;
    const bool tail_blank = nl > (int64_t)nlpos.size() && lend(nl - 1) == lstart(nl - 1);
    const bool simple = !blank && !tail_blank;
    if (simple) {
        if (nl % 4) { set_error("truncated FASTQ record in %s", path); return -3; }
    } else {
        rec.reserve((size_t)(nl / 4 + 1));
        for (int64_t k = 0; k < nl;) {
            if (lend(k) == lstart(k)) { ++k; continue; }
            if (k + 3 >= nl) { set_error("truncated FASTQ record in %s", path); return -3; }
            rec.push_back(k);
            k += 4;
        }
    }
    const int64_t nr = simple ? nl / 4 : (int64_t)rec.size();
    fq.name_at.resize(nr); fq.seq_at.resize(nr); fq.qual_at.resize(nr);
    fq.name_len.resize(nr); fq.len.resize(nr); fq.qual_len.resize(nr);
    std::atomic<int64_t> too_long(-1);
    par_for(nt, [&](int t) {
        for (int64_t r = nr * t / nt; r < nr * (t + 1) / nt; ++r) {
            const int64_t k = simple ? 4 * r : rec[r];
            fq.name_at[r] = lstart(k);
            fq.name_len[r] = (int32_t)(lend(k) - lstart(k));
            const int64_t L = lend(k + 1) - lstart(k + 1);
            if (L > MAXLEN) { too_long = r; continue; }
            fq.seq_at[r] = lstart(k + 1);
            fq.len[r] = (int32_t)L;
            fq.qual_at[r] = lstart(k + 3);
            fq.qual_len[r] = (int32_t)(lend(k + 3) - lstart(k + 3));
        }
    });
    if (too_long >= 0) { set_error("read longer than %d in %s", MAXLEN, path); return -3; }
    return 0;
}

static double ms_since(std::chrono::steady_clock::time_point t)
{
    return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t).count();
}

// decode + index one file; the wall time of each half in *dec_ms / *ix_ms
static int read_fastq(const char *path, Fastq &fq, int64_t *newlines, double *dec_ms, double *ix_ms)
{
    const auto t0 = std::chrono::steady_clock::now();
    const int st = slurp(path, fq.data);
    *dec_ms = ms_since(t0);
    if (st) return st;
    const auto t1 = std::chrono::steady_clock::now();
    const int si = index_fastq(fq, path, newlines);
    *ix_ms = ms_since(t1);
    return si;
}

}  // namespace mh

using namespace mh;

static CtxEx *X(mh_ctx *c) { return reinterpret_cast<CtxEx *>(c); }
namespace mh {
Ctx *ctx_of(mh_ctx *c) { return static_cast<Ctx *>(X(c)); }
}

extern "C" {

int mh_version(void) { return 1; }

int mh_last_error(char *buf, size_t cap)
{
    if (!buf || cap == 0) return -3;
    snprintf(buf, cap, "%s", g_err);
    return 0;
}

int mh_device_count(int *n)
{
    int k = 0;
    hipError_t e = hipGetDeviceCount(&k);
    if (e != hipSuccess) { *n = 0; return hip_fail(e, "hipGetDeviceCount") == -4 ? -5 : -5; }
    *n = k;
    return 0;
}

int mh_ctx_create(int device, mh_ctx **out)
{
    if (!out) return -3;
    *out = nullptr;
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n == 0) {
        set_error("no HIP device available (the MI355X path has no CPU fallback)");
        return -5;
    }
    if (device < 0 || device >= n) { set_error("bad device %d", device); return -3; }
    MH_HIP(hipSetDevice(device));
    hipDeviceProp_t prop;
    MH_HIP(hipGetDeviceProperties(&prop, device));
    if (std::strncmp(prop.gcnArchName, "gfx950", 6) != 0) {
        set_error("device %d is %s, libmicall_hip is built for gfx950 only", device, prop.gcnArchName);
        return -5;
    }
    CtxEx *c = new (std::nothrow) CtxEx();
    if (!c) return -2;
    c->device = device;
    hipError_t e = hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking);
    if (e != hipSuccess) { delete c; return hip_fail(e, "hipStreamCreate"); }
    *out = reinterpret_cast<mh_ctx *>(c);
    return 0;
}

int mh_ctx_destroy(mh_ctx *ctx)
{
    if (!ctx) return 0;
    CtxEx *c = X(ctx);
    hipSetDevice(c->device);
    hipStreamSynchronize(c->stream);
    free_reads(c->reads);
    free_reads(c->rows.reads);
    hipFree(c->stage_seq); hipFree(c->stage_qual); hipFree(c->stage_off);
    for (auto &ix : c->cache) free_index(ix);   // c->index only views one of these
    free_index(c->small);
    MapState &M = c->map;
    hipFree(M.cand); hipFree(M.n_cand); hipFree(M.yf); hipFree(M.work); hipFree(M.rwork); hipFree(M.skey); hipFree(M.sinfo);
    hipFree(M.pool); hipFree(M.pool_used); hipFree(M.rec); hipFree(M.counters); hipFree(M.ref_stats);
    if (M.stats_pin) hipHostFree(M.stats_pin);
    M.stats_pin = nullptr;
    M.stats_pin_cap = 0;
    RowState &R = c->rows;
    hipFree(R.flag); hipFree(R.ref); hipFree(R.pos); hipFree(R.cig_off); hipFree(R.n_cigar);
    hipFree(R.cigar); hipFree(R.units);
    PileState &P = c->pile;
    hipFree(c->gotoh_buf);
    hipFree(P.dense); hipFree(P.nflag); hipFree(P.dflag); hipFree(P.read_counts);
    hipFree(P.first_unit); hipFree(P.max_pos); hipFree(P.ev); hipFree(P.ev_pool);
    hipFree(P.tok_slot); hipFree(P.tok_cnt); hipFree(P.tok_used); hipFree(P.tok_meta);
    hipFree(P.tok_bytes);
    hipFree(P.ev_counters);
    if (P.land) hipHostFree(P.land);
    P.land = nullptr;
    if (P.tok_pin) hipHostFree(P.tok_pin);
    P.tok_pin = nullptr;
    P.tok_pin_cap = 0;
    P.land_cap = 0;
    P.land_ok = false;
    hipFree(P.ins_scratch);
    hipFree(P.sel);
    hipFree(P.win_map);
    for (auto &kv : c->len_tabs) hipFree(kv.second);
    if (c->pin) hipHostFree(c->pin);
    s2a_free(*c);
    censor_free(*c);
    a2c_free(*c);
    hipStreamDestroy(c->stream);
    delete c;
    return 0;
}

int mh_ctx_sync(mh_ctx *ctx)
{
    if (!ctx) return -3;
    MH_HIP(hipSetDevice(X(ctx)->device));
    MH_HIP(hipStreamSynchronize(X(ctx)->stream));
    return 0;
}

int mh_ctx_stream(mh_ctx *ctx, void **stream)
{
    if (!ctx || !stream) return -3;
    *stream = (void *)X(ctx)->stream;
    return 0;
}

int mh_index_build(mh_ctx *ctx, int n_refs, const char *const *seqs, int seedlen)
{
    if (!ctx || n_refs < 0 || (n_refs > 0 && !seqs) || seedlen < 8 || seedlen > 32) {
        set_error("mh_index_build: bad arguments");
        return -3;
    }
    CtxEx *c = X(ctx);
    MH_HIP(hipSetDevice(c->device));
    MH_HIP(hipStreamSynchronize(c->stream));
    int64_t total = 0;
    for (int r = 0; r < n_refs; ++r) total += (int64_t)std::strlen(seqs[r]);
    // MH_INDEX_FORCE_COLLISION=1 (tests): every reference set gets the same
    // signature, so only the content comparison tells two sets apart
    const char *force = getenv("MH_INDEX_FORCE_COLLISION");
    const uint64_t sig = force && *force == '1' ? 0x5eedull : signature(n_refs, seqs, seedlen);
    const bool cacheable = total > 65536;
    c->index = DevIndex{};   // cache entries and c->small own their buffers
    for (size_t e = 0; e < c->cache.size(); ++e) {
        const DevIndex &ix = c->cache[e];
        if (ix.sig != sig || ix.n_refs != n_refs || ix.seedlen != seedlen) continue;
        // a 64-bit hash can collide: compare the bytes (~0.6 MB memcmp for
        // the 74 seeds, well under a millisecond)
        const std::string &t = c->cache_text[e];
        bool same = t.size() == (size_t)(total + n_refs);
        size_t at = 0;
        for (int r = 0; same && r < n_refs; ++r) {
            const size_t len = std::strlen(seqs[r]);
            same = std::memcmp(t.data() + at, seqs[r], len + 1) == 0;
            at += len + 1;
        }
        if (same) {
            c->index = ix;
            return 0;
        }
    }
    if (!cacheable) {
        if (int st = build_index(c->small, n_refs, seqs, seedlen)) return st;
        c->small.sig = sig;
        c->index = c->small;
        return 0;
    }
    DevIndex ix;
    if (int st = build_index(ix, n_refs, seqs, seedlen)) { free_index(ix); return st; }
    ix.sig = sig;
    if (c->cache.size() >= 2) {
        free_index(c->cache.front());
        c->cache.erase(c->cache.begin());
        c->cache_text.erase(c->cache_text.begin());
    }
    std::string text;
    text.reserve((size_t)(total + n_refs));
    for (int r = 0; r < n_refs; ++r) text.append(seqs[r], std::strlen(seqs[r]) + 1);
    c->cache.push_back(ix);
    c->cache_text.push_back(std::move(text));
    c->index = ix;
    return 0;
}

int mh_reads_load(mh_ctx *ctx, int64_t n_reads, int paired, const uint8_t *seq,
                  const uint8_t *qual, const int64_t *offsets, const int32_t *lens)
{
    if (!ctx || (n_reads > 0 && (!seq || !qual || !offsets || !lens))) return -3;
    CtxEx *c = X(ctx);
    MH_HIP(hipSetDevice(c->device));
    c->names.clear();
    c->map.valid = false;
    return load_reads(*c, c->reads, c->host, n_reads, paired, seq, qual, offsets, lens, true);
}

int mh_reads_load_fastq(mh_ctx *ctx, const char *path1, const char *path2, int64_t *n_reads)
{
    return mh_reads_load_fastq_part(ctx, path1, path2, 0, 1, n_reads, nullptr);
}

// The reads of units [a0, a1) of FASTQ a (and [b0, b1) of b, the mates):
// copied once from the decoded text into the buffers the context keeps for
// the SAM text, uploaded and packed.
// The host half of a FASTQ load: the reads of units [a0, a1) of FASTQ a
// (and [b0, b1) of b, the mates, interleaved) copied once from the decoded
// text into `h` (SEQ / QUAL of the SAM rows) and their QNAMEs into `names`.
static int host_reads_from(Fastq &a, Fastq *b, int64_t a0, int64_t a1, int64_t b0, int64_t b1,
                           HostReads &h, NameTable &names, double *names_ms, double *copy_ms)
{
    const bool paired = b != nullptr;
    if (a0 < 0 || a1 < a0 || a1 > (int64_t)a.size() ||
        (paired && (b0 < 0 || b1 < b0 || b1 > (int64_t)b->size() || b1 - b0 != a1 - a0))) {
        set_error("paired FASTQ blocks hold %lld and %lld reads", (long long)(a1 - a0),
                  (long long)(paired ? b1 - b0 : a1 - a0));
        return -3;
    }
    const int per = paired ? 2 : 1;
    const int64_t n = per * (a1 - a0);
    h.off.resize((size_t)n);
    h.len.resize((size_t)n);
    int64_t total = 0;
    for (int64_t i = 0; i < n; ++i) {
        const bool mate2 = paired && (i & 1);
        const Fastq &f = mate2 ? *b : a;
        h.off[i] = total;
        h.len[i] = f.len[(mate2 ? b0 : a0) + i / per];
        total += h.len[i];
    }
    const auto t_setup = std::chrono::steady_clock::now();
    h.seq.alloc((size_t)total);
    h.qual.alloc((size_t)total);
    const auto tn = std::chrono::steady_clock::now();
    // names: spans first (sizes), then every thread copies its names into the pool
    names.clear();
    names.off.resize((size_t)n + 1);
    std::vector<int64_t> nstart((size_t)n);
    const int nt = std::max(1, std::min(s2a_threads(), (int)(n >> 14) + 1));
    std::vector<int64_t> tsum(nt + 1, 0);
    std::vector<double> t_go((size_t)nt, 0.0), t_end((size_t)nt, 0.0);
    par_for(nt, [&](int t) {
        t_go[(size_t)t] = ms_since(tn);
        int64_t sum = 0;
        for (int64_t i = n * t / nt; i < n * (t + 1) / nt; ++i) {
            const bool mate2 = paired && (i & 1);
            const Fastq &f = mate2 ? *b : a;
            const int64_t r = (mate2 ? b0 : a0) + i / per;
            size_t at = 0, len = 0;
            qname_span(f.data.data() + f.name_at[r], (size_t)f.name_len[r], paired, &at, &len);
            nstart[i] = f.name_at[r] + (int64_t)at;
            names.off[i + 1] = (int64_t)len;
            sum += (int64_t)len;
        }
        tsum[t + 1] = sum;
        t_end[(size_t)t] = ms_since(tn);
    });
    const double names_pass1 = ms_since(tn);
    if (getenv("MH_INGEST_TRACE")) {
        double g = 0, e = 0, w = 0;
        for (int t = 0; t < nt; ++t) {
            g = std::max(g, t_go[(size_t)t]);
            e = std::max(e, t_end[(size_t)t]);
            w = std::max(w, t_end[(size_t)t] - t_go[(size_t)t]);
        }
        fprintf(stderr, "ingest: name spans: last start %.1f ms, last end %.1f ms, longest %.1f ms (%d threads)\n",
                g, e, w, nt);
    }
    for (int t = 0; t < nt; ++t) tsum[t + 1] += tsum[t];
    names.pool.resize((size_t)tsum[nt]);
    par_for(nt, [&](int t) {
        int64_t o = tsum[t];
        for (int64_t i = n * t / nt; i < n * (t + 1) / nt; ++i) {
            const bool mate2 = paired && (i & 1);
            const Fastq &f = mate2 ? *b : a;
            const int64_t len = names.off[i + 1];
            memcpy(&names.pool[(size_t)o], f.data.data() + nstart[i], (size_t)len);
            names.off[i + 1] = o + len;
            o += len;
        }
    });
    names.off[0] = 0;
    *names_ms = ms_since(tn);
    if (getenv("MH_INGEST_TRACE"))
        fprintf(stderr, "ingest: names setup %.1f ms, spans %.1f ms, copies to %.1f ms\n", ms_since(t_setup) - ms_since(tn),
                names_pass1, *names_ms);
    const auto tc = std::chrono::steady_clock::now();
    par_for(nt, [&](int t) {
        for (int64_t i = n * t / nt; i < n * (t + 1) / nt; ++i) {
            const bool mate2 = paired && (i & 1);
            const Fastq &f = mate2 ? *b : a;
            const int64_t r = (mate2 ? b0 : a0) + i / per;
            const char *D = f.data.data();
            const int64_t L = h.len[i];
            memcpy(h.seq.data() + h.off[i], D + f.seq_at[r], (size_t)L);
            const int64_t cq = std::min<int64_t>(L, f.qual_len[r]);
            if (cq > 0) memcpy(h.qual.data() + h.off[i], D + f.qual_at[r], (size_t)cq);
            for (int64_t x = cq; x < L; ++x) h.qual.data()[h.off[i] + x] = 'I';
        }
    });
    *copy_ms = ms_since(tc);
    return 0;
}

static int load_fastq_units(CtxEx *c, Fastq &a, Fastq *b, int64_t a0, int64_t a1, int64_t b0,
                            int64_t b1, int64_t lines1, int64_t *n_reads)
{
    const bool paired = b != nullptr;
    const auto t0 = std::chrono::steady_clock::now();
    HostReads h;
    NameTable names;
    double names_ms = 0, copy_ms = 0;
    if (int st = host_reads_from(a, b, a0, a1, b0, b1, h, names, &names_ms, &copy_ms)) return st;
    const int64_t n = (int64_t)h.len.size();
    const auto tf = std::chrono::steady_clock::now();
    // the decoded texts (GBs) are released on a thread of their own after the
    // upload: giving the pages back takes ~0.13 s per C2 pair of files, which
    // nothing needs to wait for
    auto *box = new std::pair<Fastq, Fastq>(std::move(a), b ? std::move(*b) : Fastq{});
    a = Fastq{};
    if (b) *b = Fastq{};
    if (getenv("MH_INGEST_TRACE"))
        fprintf(stderr, "ingest: names %.1f ms, copy %.1f ms, free %.1f ms\n", names_ms, copy_ms,
                ms_since(tf));
    c->phase_ms[MH_PHASE_PARSE] += ms_since(t0);
    const auto t1 = std::chrono::steady_clock::now();
    const uint8_t *sq = h.seq.data(), *ql = h.qual.data();
    const int64_t *of = h.off.data();
    const int32_t *ln = h.len.data();
    int st = load_reads(*c, c->reads, c->host, n, paired, sq, ql, of, ln, false, &h);
    c->phase_ms[MH_PHASE_UPLOAD] += ms_since(t1);
    std::thread([box] { delete box; }).detach();
    if (st) return st;
    c->names.swap(names);
    c->map.valid = false;
    c->fastq_lines1 = lines1;
    if (n_reads) *n_reads = n;
    return 0;
}

int mh_reads_load_fastq_part(mh_ctx *ctx, const char *path1, const char *path2, int part, int parts,
                             int64_t *n_reads, int64_t *first_unit)
{
    if (!ctx || !path1 || parts < 1 || part < 0 || part >= parts) {
        set_error("mh_reads_load_fastq_part: bad arguments");
        return -3;
    }
    CtxEx *c = X(ctx);
    MH_HIP(hipSetDevice(c->device));
    const bool paired = path2 != nullptr;
    Fastq a, b;
    int64_t lines1 = 0;
    int st2 = 0;
    std::string err2;
    double dec1 = 0, dec2 = 0, ix1 = 0, ix2 = 0;
    // the two files are decoded concurrently
    std::thread t2;
    if (paired)
        t2 = std::thread([&]() {
            st2 = read_fastq(path2, b, nullptr, &dec2, &ix2);
            if (st2) err2 = last_error_text();
        });
    const int st1 = read_fastq(path1, a, &lines1, &dec1, &ix1);
    if (paired) t2.join();
    c->phase_ms[MH_PHASE_INFLATE] += std::max(dec1, dec2);
    c->phase_ms[MH_PHASE_PARSE] += std::max(ix1, ix2);
    if (getenv("MH_INGEST_TRACE"))
        fprintf(stderr, "ingest: decode %.1f / %.1f ms, index %.1f / %.1f ms\n", dec1, dec2, ix1, ix2);
    if (st1) return st1;
    if (st2) { set_error("%s", err2.c_str()); return st2; }
    if (paired && a.size() != b.size()) {
        set_error("paired FASTQ files hold %zu and %zu reads", a.size(), b.size());
        return -3;
    }
    // this part's contiguous block of units (pairs, or reads when unpaired):
    // [U * part / parts, U * (part + 1) / parts), so every unit is in one
    // block and the blocks differ in size by at most one
    const int64_t units_all = (int64_t)a.size();
    const int64_t u0 = units_all * part / parts, u1 = units_all * (part + 1) / parts;
    if (first_unit) *first_unit = u0;
    return load_fastq_units(c, a, paired ? &b : nullptr, u0, u1, u0, u1, lines1, n_reads);
}

int mh_reads_load_staged(mh_ctx *ctx, mh_fastq *fq1, mh_fastq *fq2, const int64_t *range4,
                         int64_t fastq_lines1, int64_t *n_reads)
{
    if (!ctx || !fq1 || !range4) { set_error("mh_reads_load_staged: bad arguments"); return -3; }
    CtxEx *c = X(ctx);
    MH_HIP(hipSetDevice(c->device));
    const bool paired = fq2 != nullptr;
    Fastq a, b;
    double ix1 = 0, ix2 = 0;
    int st1 = 0, st2 = 0;
    std::string err2;
    try {
        a.data = take_fastq_text(fq1);
        if (paired) b.data = take_fastq_text(fq2);
    } catch (const std::bad_alloc &) {
        set_error("mh_reads_load_staged: out of memory");
        return -2;
    }
    std::thread t2;
    if (paired)
        t2 = std::thread([&]() {
            const auto t = std::chrono::steady_clock::now();
            st2 = index_fastq(b, "FASTQ 2", nullptr);
            ix2 = ms_since(t);
            if (st2) err2 = last_error_text();
        });
    {
        const auto t = std::chrono::steady_clock::now();
        st1 = index_fastq(a, "FASTQ 1", nullptr);
        ix1 = ms_since(t);
    }
    if (paired) t2.join();
    c->phase_ms[MH_PHASE_PARSE] += std::max(ix1, ix2);
    if (st1) return st1;
    if (st2) { set_error("%s", err2.c_str()); return st2; }
    const int64_t a0 = range4[0] < 0 ? 0 : range4[0];
    const int64_t a1 = range4[1] < 0 ? (int64_t)a.size() : range4[1];
    const int64_t b0 = range4[2] < 0 ? 0 : range4[2];
    const int64_t b1 = range4[3] < 0 ? (int64_t)b.size() : range4[3];
    return load_fastq_units(c, a, paired ? &b : nullptr, a0, a1, b0, b1, fastq_lines1, n_reads);
}

int mh_fastq_parse(mh_fastq *fq1, mh_fastq *fq2, char *names, size_t names_cap, uint8_t *seq,
                   uint8_t *qual, size_t bases_cap, int32_t *lens, int64_t reads_cap, int64_t *n_reads,
                   int64_t *n_bases, size_t *names_used)
{
    if (!fq1 || !n_reads || !n_bases || !names_used) { set_error("mh_fastq_parse: bad arguments"); return -3; }
    try {
        const bool paired = fq2 != nullptr;
        Fastq a, b;
        a.data.assign(fastq_text(fq1).data(), fastq_text(fq1).size());
        if (paired) b.data.assign(fastq_text(fq2).data(), fastq_text(fq2).size());
        if (int st = index_fastq(a, "FASTQ 1", nullptr)) return st;
        if (paired)
            if (int st = index_fastq(b, "FASTQ 2", nullptr)) return st;
        if (paired && a.size() != b.size()) {
            set_error("paired FASTQ files hold %zu and %zu reads", a.size(), b.size());
            return -3;
        }
        HostReads h;
        NameTable nt;
        double x = 0, y = 0;
        if (int st = host_reads_from(a, paired ? &b : nullptr, 0, (int64_t)a.size(), 0,
                                     paired ? (int64_t)b.size() : 0, h, nt, &x, &y))
            return st;
        const int64_t n = (int64_t)h.len.size();
        const int64_t bases = n ? h.off[n - 1] + h.len[n - 1] : 0;
        *n_reads = n;
        *n_bases = bases;
        *names_used = nt.pool.size() + (size_t)n;
        if (!names || !seq || !qual || !lens) return 0;   // a size query
        if (reads_cap < n || bases_cap < (size_t)bases || names_cap < *names_used) {
            set_error("mh_fastq_parse: buffers too small");
            return -2;
        }
        size_t at = 0;
        for (int64_t r = 0; r < n; ++r) {
            const std::string_view v = nt[(size_t)r];
            memcpy(names + at, v.data(), v.size());
            at += v.size();
            names[at++] = '\n';
            lens[r] = h.len[r];
        }
        if (bases) {
            memcpy(seq, h.seq.data(), (size_t)bases);
            memcpy(qual, h.qual.data(), (size_t)bases);
        }
        return 0;
    } catch (const std::bad_alloc &) {
        set_error("mh_fastq_parse: out of memory");
        return -2;
    }
}

int mh_reads_count(mh_ctx *ctx, int64_t *n_reads, int *paired)
{
    if (!ctx) return -3;
    if (n_reads) *n_reads = X(ctx)->reads.n;
    if (paired) *paired = X(ctx)->reads.paired;
    return 0;
}

int mh_reads_set_names(mh_ctx *ctx, int64_t n, const char *const *names)
{
    if (!ctx || n != X(ctx)->reads.n) { set_error("mh_reads_set_names: count mismatch"); return -3; }
    CtxEx *c = X(ctx);
    c->names.assign(names, n);
    return 0;
}

int mh_map(mh_ctx *ctx, const mh_params *par)
{
    if (!ctx || !par) return -3;
    CtxEx *c = X(ctx);
    MH_HIP(hipSetDevice(c->device));
    if (int st = prepare_len_tab(*c, *par)) return st;
    int st = run_map(*c, *par);
    if (st == 0) MH_HIP(hipStreamSynchronize(c->stream));
    prof_flush(*c);
    c->rec_cache.clear();
    ++c->map_gen;
    c->fmt_valid = false;
    c->fmt_chunks.clear();
    return st;
}

int mh_probe_extend(mh_ctx *ctx, const mh_params *par, int n, const int32_t *items, int32_t *out)
{
    if (!ctx || !par || n < 0 || (n > 0 && (!items || !out))) return -3;
    CtxEx *c = X(ctx);
    MH_HIP(hipSetDevice(c->device));
    if (int st = prepare_len_tab(*c, *par)) return st;
    return run_probe_ext(*c, *par, n, items, out);
}

int mh_profile(mh_ctx *ctx, int enable)
{
    if (!ctx) return -3;
    CtxEx *c = X(ctx);
    c->prof = enable != 0;
    c->prof_acc.clear();
    return 0;
}

int mh_profile_get(mh_ctx *ctx, const char *kernel, double *total_ms, int64_t *launches)
{
    if (!ctx || !kernel) return -3;
    CtxEx *c = X(ctx);
    prof_flush(*c);
    auto it = c->prof_acc.find(kernel);
    if (total_ms) *total_ms = it == c->prof_acc.end() ? 0.0 : it->second.ms;
    if (launches) *launches = it == c->prof_acc.end() ? 0 : it->second.launches;
    return 0;
}

static int fetch_recs(CtxEx *c, int64_t first, int64_t n, std::vector<Rec> &rec,
                      std::vector<uint32_t> &pool)
{
    MapState &M = c->map;
    if (!M.valid) { set_error("no mapping results (call mh_map)"); return -3; }
    if (first < 0 || n < 0 || first + n > M.n_reads) { set_error("record range out of bounds"); return -3; }
    rec.resize(n > 0 ? n : 1);
    if (n > 0)
        MH_HIP(copy_sync(*c, rec.data(), M.rec + first, sizeof(Rec) * n, hipMemcpyDeviceToHost));
    // the words claimed by the last pass (its chunks end within the pool:
    // a pass that overflowed was run again with a larger one)
    int64_t used = M.last_cigar < M.pool_cap ? M.last_cigar : M.pool_cap;
    pool.resize(used > 0 ? used : 1);
    if (used > 0)
        MH_HIP(copy_sync(*c, pool.data(), M.pool, sizeof(uint32_t) * used, hipMemcpyDeviceToHost));
    return 0;
}

int mh_alns_fetch(mh_ctx *ctx, int64_t first, int64_t n, mh_aln *out)
{
    if (!ctx || (n > 0 && !out)) return -3;
    CtxEx *c = X(ctx);
    MH_HIP(hipSetDevice(c->device));
    std::vector<Rec> rec;
    std::vector<uint32_t> pool;
    if (int st = fetch_recs(c, first, n, rec, pool)) return st;
    for (int64_t i = 0; i < n; ++i) {
        const Rec &r = rec[i];
        mh_aln &o = out[i];
        std::memcpy(&o, &r, sizeof(int32_t) * 20);
        std::memset(o.cigar, 0, sizeof(o.cigar));
        for (int k = 0; k < r.n_cigar && k < MH_MAXOPS; ++k) o.cigar[k] = pool[r.cig_off + k];
    }
    return 0;
}

int mh_map_counts(mh_ctx *ctx, int64_t *lines, int64_t *filtered, int64_t *mapped,
                  int64_t *first_row, int64_t *first_mapped, int64_t *unmapped,
                  int64_t *star_lines, int64_t *star_first)
{
    if (!ctx) return -3;
    CtxEx *c = X(ctx);
    MapState &M = c->map;
    if (!M.valid) { set_error("no mapping results (call mh_map)"); return -3; }
    MH_HIP(hipSetDevice(c->device));
    const int n = M.n_refs;
    const int64_t *s = map_stats_host(*c);
    if (!s) return -1;
    if (lines) std::memcpy(lines, s, sizeof(int64_t) * n);
    if (filtered) std::memcpy(filtered, s + n, sizeof(int64_t) * n);
    if (mapped) std::memcpy(mapped, s + 2 * n, sizeof(int64_t) * n);
    if (first_row) std::memcpy(first_row, s + 3 * n, sizeof(int64_t) * n);
    if (first_mapped) std::memcpy(first_mapped, s + 4 * n, sizeof(int64_t) * n);
    if (unmapped) *unmapped = s[5 * n];
    if (star_lines) *star_lines = s[5 * n + 1];
    if (star_first) *star_first = s[5 * n + 2];
    return 0;
}

int mh_map_stats(mh_ctx *ctx, int64_t *out5)
{
    if (!ctx || !out5) return -3;
    int64_t *out4 = out5;
    CtxEx *c = X(ctx);
    MapState &M = c->map;
    if (!M.valid) { set_error("no mapping results (call mh_map)"); return -3; }
    out4[0] = M.n_reads;
    out4[1] = M.last_work;
    out4[2] = M.last_cigar;
    out4[3] = M.last_fast;
    out5[4] = M.last_rescue;
    return 0;
}

int mh_test_set_capacities(mh_ctx *ctx, int64_t cigar_pool_words, int64_t pileup_events,
                           int64_t pileup_event_bytes, int64_t token_bytes)
{
    if (!ctx || cigar_pool_words < 0 || pileup_events < 0 || pileup_event_bytes < 0 || token_bytes < 0) {
        set_error("mh_test_set_capacities: bad arguments");
        return -3;
    }
    CtxEx *c = X(ctx);
    MH_HIP(hipSetDevice(c->device));
    MH_HIP(hipStreamSynchronize(c->stream));
    // the next call sizes every one of these buffers again
    MapState &M = c->map;
    PileState &P = c->pile;
    hipFree(M.pool); M.pool = nullptr; M.pool_cap = 0;
    hipFree(P.ev); P.ev = nullptr; P.ev_cap = 0;
    hipFree(P.ev_pool); P.ev_pool = nullptr; P.pool_cap = 0;
    hipFree(P.tok_bytes); P.tok_bytes = nullptr; P.tok_bytes_cap = 0;
    M.valid = false;   // the records of the last pass pointed into the pool
    TestCaps &t = c->test_caps;
    t.cigar_pool_words = cigar_pool_words;
    t.pile_events = pileup_events;
    t.pile_event_bytes = pileup_event_bytes;
    t.token_bytes = token_bytes;
    return 0;
}

int mh_retry_counts(mh_ctx *ctx, int64_t *out4)
{
    if (!ctx || !out4) return -3;
    for (int k = 0; k < RETRY_KINDS; ++k) out4[k] = X(ctx)->retries[k];
    return 0;
}

int mh_test_set_gotoh_wait(mh_ctx *ctx, int64_t ticks)
{
    if (!ctx || ticks < 0) { set_error("mh_test_set_gotoh_wait: bad arguments"); return -3; }
    X(ctx)->test_caps.gotoh_wait_ticks = ticks;
    return 0;
}

int mh_recs_fetch(mh_ctx *ctx, int64_t first, int64_t n, int32_t *out20)
{
    if (!ctx || (n > 0 && !out20)) return -3;
    CtxEx *c = X(ctx);
    MapState &M = c->map;
    if (!M.valid) { set_error("no mapping results (call mh_map)"); return -3; }
    if (first < 0 || n < 0 || first + n > M.n_reads) { set_error("record range out of bounds"); return -3; }
    MH_HIP(hipSetDevice(c->device));
    if (n == 0) return 0;
    // Rec is 22 int32; copy with a 2D memcpy that keeps the first 20 of each
    MH_HIP(hipMemcpy2DAsync(out20, sizeof(int32_t) * 20, M.rec + first, sizeof(Rec), sizeof(int32_t) * 20,
                            (size_t)n, hipMemcpyDeviceToHost, c->stream));
    MH_HIP(hipStreamSynchronize(c->stream));
    return 0;
}

int mh_recs_fetch_fields(mh_ctx *ctx, int64_t first, int64_t n, int field0, int nfields, int32_t *out)
{
    if (!ctx || (n > 0 && !out) || field0 < 0 || nfields < 1 || field0 + nfields > 20) return -3;
    CtxEx *c = X(ctx);
    MapState &M = c->map;
    if (!M.valid) { set_error("no mapping results (call mh_map)"); return -3; }
    if (first < 0 || n < 0 || first + n > M.n_reads) { set_error("record range out of bounds"); return -3; }
    MH_HIP(hipSetDevice(c->device));
    if (n == 0) return 0;
    MH_HIP(hipMemcpy2DAsync(out, sizeof(int32_t) * nfields, (const int32_t *)(M.rec + first) + field0, sizeof(Rec),
                            sizeof(int32_t) * nfields, (size_t)n, hipMemcpyDeviceToHost, c->stream));
    MH_HIP(hipStreamSynchronize(c->stream));
    return 0;
}

// decimal text of v appended to out (no locale, no allocation)
// decimal text of v at o; returns the end
static inline char *put_int(char *o, int64_t v)
{
    char t[24];
    int n = 0;
    uint64_t u = v < 0 ? (uint64_t)(-(v + 1)) + 1 : (uint64_t)v;
    do { t[n++] = (char)('0' + u % 10); u /= 10; } while (u);
    if (v < 0) *o++ = '-';
    while (n) *o++ = t[--n];
    return o;
}

static inline char *put_str(char *o, const char *s, size_t n)
{
    std::memcpy(o, s, n);
    return o + n;
}

// csv.writer QUOTE_MINIMAL (csv_field) into a buffer with room for 2n + 2
// any byte of w equal to c (bit tricks over 8 bytes at a time)
static inline uint64_t has_byte(uint64_t w, uint8_t c)
{
    const uint64_t x = w ^ (0x0101010101010101ull * c);
    return (x - 0x0101010101010101ull) & ~x & 0x8080808080808080ull;
}

static inline bool needs_quotes(const char *s, size_t n)
{
    size_t i = 0;
    uint64_t hit = 0;
    for (; i + 8 <= n; i += 8) {
        uint64_t w;
        std::memcpy(&w, s + i, 8);
        hit |= has_byte(w, ',') | has_byte(w, '"') | has_byte(w, '\n') | has_byte(w, '\r');
    }
    bool quote = hit != 0;
    for (; i < n; ++i) {
        const char ch = s[i];
        quote |= ch == ',' || ch == '"' || ch == '\n' || ch == '\r';
    }
    return quote;
}

static inline char *put_csv(char *o, const char *s, size_t n)
{
    const bool quote = needs_quotes(s, n);
    if (!quote) return put_str(o, s, n);
    *o++ = '"';
    for (size_t i = 0; i < n; ++i) {
        if (s[i] == '"') *o++ = '"';
        *o++ = s[i];
    }
    *o++ = '"';
    return o;
}

// bowtie2 prints a read's bases as ACGTN, reverse-complemented on the
// reverse strand (code_of: a/c/g/t in either case, anything else N)
struct BaseTables {
    char fw[256], rc[256];
    BaseTables()
    {
        for (int ch = 0; ch < 256; ++ch) {
            const uint8_t cd = code_of((char)ch);
            fw[ch] = "ACGTN"[cd];
            rc[ch] = "TGCAN"[cd];
        }
    }
};
static const BaseTables kBases;

// One row of SAM (style 0) or CSV (style 1) text, appended to out at *used
// (out grows as needed; it is not zero-filled beyond what is written).
static void format_row(const CtxEx *c, int style, const Rec &a, int64_t r, const uint32_t *pool,
                       const char *const *refnames, const size_t *refname_len, TextBuf &out,
                       size_t &used, std::string &tmp)
{
    static const char *ytn[4] = {"CP", "DP", "UP", "UU"};
    static const char *yfn[3] = {"", "NS", "LN"};
    const char sep = style == 0 ? '\t' : ',';
    const int L = c->host.len[r];
    const uint8_t *s = c->host.seq.data() + c->host.off[r];
    const uint8_t *q = c->host.qual.data() + c->host.off[r];
    const std::string_view qn = c->names[r];
    const char *rn = a.sam_ref >= 0 ? refnames[a.sam_ref] : "*";
    const size_t rnl = a.sam_ref >= 0 ? refname_len[a.sam_ref] : 1;
    const size_t nxl = a.rnext >= 0 ? refname_len[a.rnext] : 1;
    const size_t bound = 2 * qn.size() + 2 * rnl + 2 * nxl + 3 * (size_t)L + 8 +
                         12 * (size_t)(a.ref >= 0 ? a.n_cigar : 1) + 16 * 12 + 160;
    if (used + bound > out.size()) out.resize(std::max(out.size() * 2, used + bound));
    char *o = &out[used];
    const bool rev = a.ref >= 0 && a.rev;
    o = style == 1 ? put_csv(o, qn.data(), qn.size()) : put_str(o, qn.data(), qn.size());
    *o++ = sep;
    o = put_int(o, a.flag);
    *o++ = sep;
    o = style == 1 ? put_csv(o, rn, rnl) : put_str(o, rn, rnl);
    *o++ = sep;
    o = put_int(o, a.sam_pos);
    *o++ = sep;
    o = put_int(o, a.mapq);
    *o++ = sep;
    if (a.ref < 0) {
        *o++ = '*';
    } else {
        for (int z = 0; z < a.n_cigar; ++z) {
            const uint32_t op = pool[a.cig_off + z];
            o = put_int(o, op >> 4);
            *o++ = "MIDxS"[op & 7];
        }
    }
    *o++ = sep;
    if (a.rnext == -2) *o++ = '*';
    else if (a.rnext == -1) *o++ = '=';
    else o = style == 1 ? put_csv(o, refnames[a.rnext], nxl) : put_str(o, refnames[a.rnext], nxl);
    *o++ = sep;
    o = put_int(o, a.pnext);
    *o++ = sep;
    o = put_int(o, a.tlen);
    *o++ = sep;
    if (L == 0) {
        *o++ = '*';
        *o++ = sep;
        *o++ = '*';
    } else {
        // SEQ has no character csv quotes; QUAL may (',' is Phred 11)
        if (rev) for (int x = 0; x < L; ++x) o[L - 1 - x] = kBases.rc[s[x]];
        else for (int x = 0; x < L; ++x) o[x] = kBases.fw[s[x]];
        o += L;
        *o++ = sep;
        const char *qq = (const char *)q;
        if (rev) {
            tmp.resize((size_t)L);
            for (int x = 0; x < L; ++x) tmp[L - 1 - x] = (char)q[x];
            qq = tmp.data();
        }
        o = style == 1 ? put_csv(o, qq, (size_t)L) : put_str(o, qq, (size_t)L);
    }
    if (style == 0) {
        auto tag = [&](const char *t, int64_t v) { o = put_str(o, t, std::strlen(t)); o = put_int(o, v); };
        if (a.ref >= 0) {
            tag("\tAS:i:", a.score);
            if (a.secbest != I32MIN) tag("\tXS:i:", a.secbest);
            tag("\tXN:i:0\tXM:i:", a.xm);
            tag("\tXO:i:", a.xo);
            tag("\tXG:i:", a.xg);
            tag("\tNM:i:", a.nm);
            if (a.ys != I32MIN) tag("\tYS:i:", a.ys);
        } else {
            if (a.ys != I32MIN) tag("\tYS:i:", a.ys);
            if (a.yf) { o = put_str(o, "\tYF:Z:", 6); o = put_str(o, yfn[a.yf], 2); }
        }
        o = put_str(o, "\tYT:Z:", 6);
        o = put_str(o, ytn[a.yt & 3], 2);
    }
    *o++ = '\n';
    used = (size_t)(o - out.data());
}

// Bytes at file offsets, written by host threads with pwrite.  (Buffered
// writes to one file serialise on its inode lock; a shared writable mapping
// filled by every thread instead -- MICALL_WRITE_MMAP=1: the file extended
// by fallocate, which never shrinks it, so ranks of a sharded job writing
// their own ranges cannot cut each other's bytes -- measured slower on the
// GPU box's overlay file system: 0.45 vs 0.24 s for a 1.17 GB prelim.csv.)
// 0, or an errno.
struct WritePiece {
    const char *src;
    size_t len;
    int64_t off;
};

static int write_pieces(int fd, std::vector<WritePiece> pieces)
{
    pieces.erase(std::remove_if(pieces.begin(), pieces.end(),
                                [](const WritePiece &p) { return p.len == 0; }),
                 pieces.end());
    if (pieces.empty()) return 0;
    int64_t lo = INT64_MAX, hi = 0;
    for (const WritePiece &p : pieces) {
        lo = std::min(lo, p.off);
        hi = std::max(hi, p.off + (int64_t)p.len);
    }
    // balance: pieces of at most 4 MiB
    std::vector<WritePiece> work;
    for (const WritePiece &p : pieces)
        for (size_t a = 0; a < p.len; a += (size_t)4 << 20)
            work.push_back(WritePiece{p.src + a, std::min(p.len - a, (size_t)4 << 20), p.off + (int64_t)a});
    const int nt = std::max(1, std::min<int>(s2a_threads(), (int)work.size()));
    std::atomic<size_t> next(0);
    std::atomic<int> bad(0);
    const long pg = sysconf(_SC_PAGESIZE);
    const int64_t base = lo / pg * pg;
    void *map = MAP_FAILED;
    static const bool use_map = getenv("MICALL_WRITE_MMAP") && *getenv("MICALL_WRITE_MMAP") == '1';
    if (use_map && hi - lo >= ((int64_t)1 << 20) && fallocate(fd, 0, lo, hi - lo) == 0) {
        // a shared writable mapping needs a descriptor open for reading too:
        // an output opened 'w' is write-only, so it is opened again read-write
        // through /proc (the same file; its own offset is not used)
        char self[64];
        snprintf(self, sizeof(self), "/proc/self/fd/%d", fd);
        const int rw = open(self, O_RDWR | O_CLOEXEC);
        if (rw >= 0) {
            struct stat a, b;
            if (fstat(fd, &a) == 0 && fstat(rw, &b) == 0 && a.st_dev == b.st_dev && a.st_ino == b.st_ino)
                map = mmap(nullptr, (size_t)(hi - base), PROT_WRITE, MAP_SHARED, rw, (off_t)base);
            close(rw);
        }
    }
    if (map != MAP_FAILED) {
        char *m = (char *)map;
        par_for(nt, [&](int) {
            for (size_t i; (i = next.fetch_add(1)) < work.size();)
                std::memcpy(m + (work[i].off - base), work[i].src, work[i].len);
        });
        munmap(map, (size_t)(hi - base));
        return 0;
    }
    par_for(nt, [&](int) {
        for (size_t i; (i = next.fetch_add(1)) < work.size();) {
            const char *src = work[i].src;
            size_t left = work[i].len;
            int64_t pos = work[i].off;
            while (left > 0) {
                const ssize_t w = pwrite(fd, src, left, (off_t)pos);
                if (w <= 0) { bad = errno ? errno : EIO; return; }
                src += w; left -= (size_t)w; pos += w;
            }
        }
    });
    return bad.load();
}

// The text of rows first .. first+n (or order[first ..]) as one chunk per
// host thread, in order.  With segment row bounds seg_rows[0 .. n_seg]
// (relative to `first`, ascending), *seg_at gets the byte offset in the
// concatenated text at which each bound row starts.
static int format_chunks_unguarded(CtxEx *c, int style, const int64_t *order, int64_t first,
                                   int64_t n, const char *const *refnames,
                                   std::vector<TextBuf> &chunks, int n_seg,
                                   const int64_t *seg_rows, std::vector<int64_t> *seg_at);

// format_chunks_unguarded with an allocation failure on any formatting
// thread (par_for rethrows it here) reported as -2, not thrown across the ABI
static int format_chunks(CtxEx *c, int style, const int64_t *order, int64_t first, int64_t n,
                         const char *const *refnames, std::vector<TextBuf> &chunks,
                         int n_seg = 0, const int64_t *seg_rows = nullptr,
                         std::vector<int64_t> *seg_at = nullptr)
{
    try {
        return format_chunks_unguarded(c, style, order, first, n, refnames, chunks, n_seg, seg_rows,
                                       seg_at);
    } catch (const std::bad_alloc &) {
        chunks.clear();
        set_error("row formatting: out of memory");
        return -2;
    } catch (const std::exception &e) {
        chunks.clear();
        set_error("row formatting: %s", e.what());
        return -2;
    }
}

static int format_chunks_unguarded(CtxEx *c, int style, const int64_t *order, int64_t first,
                                   int64_t n, const char *const *refnames,
                                   std::vector<TextBuf> &chunks, int n_seg,
                                   const int64_t *seg_rows, std::vector<int64_t> *seg_at)
{
    const auto t0 = std::chrono::steady_clock::now();
    std::vector<Rec> rec;
    std::vector<uint32_t> pool;
    if (order) {
        if (int st = fetch_recs(c, 0, c->map.n_reads, rec, pool)) return st;
        for (int64_t k = 0; k < n; ++k)
            if (order[first + k] < 0 || order[first + k] >= c->map.n_reads) {
                set_error("format order index out of range");
                return -3;
            }
    } else if (int st = fetch_recs(c, first, n, rec, pool)) {
        return st;
    }
    std::vector<size_t> rn_len(c->index.n_refs > 0 ? (size_t)c->index.n_refs : 1, 0);
    for (int k = 0; k < c->index.n_refs; ++k) rn_len[k] = std::strlen(refnames[k]);
    const int nt = std::max(1, std::min(s2a_threads(), (int)(n >> 14) + 1));
    chunks.clear();
    chunks.resize(nt);
    // a chunk's bytes are reserved for its rows' upper bound up front (not
    // touched until written: no zero fill, no regrowth copies)
    size_t name_max = 1;
    for (size_t r = 0; r < c->names.size(); ++r)
        name_max = std::max(name_max, (size_t)(c->names.off[r + 1] - c->names.off[r]));
    size_t ref_max = 1;
    for (int k = 0; k < c->index.n_refs; ++k) ref_max = std::max(ref_max, rn_len[k]);
    const size_t row_max = 2 * name_max + 4 * ref_max + 3 * (size_t)std::max(c->reads.max_len, 1) +
                           12 * MH_MAXOPS + 16 * 12 + 200;
    // per thread: (segment bound, byte offset in the thread's chunk)
    std::vector<std::vector<std::pair<int, size_t>>> marks(nt);
    par_for(nt, [&](int t) {
        const int64_t k0 = n * t / nt, k1 = n * (t + 1) / nt;
        TextBuf &out = chunks[t];
        out.reserve((size_t)(k1 - k0) * row_max + 1);
        out.resize((size_t)(k1 - k0) * row_max + 1);
        size_t used = 0;
        std::string tmp;
        int sb = 0;
        if (seg_rows) {
            while (sb <= n_seg && seg_rows[sb] < k0) ++sb;
        }
        for (int64_t k = k0; k < k1; ++k) {
            while (seg_rows && sb <= n_seg && seg_rows[sb] == k) marks[t].emplace_back(sb++, used);
            const int64_t r = order ? order[first + k] : first + k;
            format_row(c, style, order ? rec[r] : rec[k], r, pool.data(), refnames, rn_len.data(),
                       out, used, tmp);
        }
        out.resize(used);
    });
    if (seg_at) {
        seg_at->assign((size_t)n_seg + 1, -1);
        int64_t base = 0;
        for (int t = 0; t < nt; ++t) {
            for (auto &m : marks[t]) (*seg_at)[m.first] = base + (int64_t)m.second;
            base += (int64_t)chunks[t].size();
        }
        for (int sb = 0; sb <= n_seg; ++sb)   // bounds at the end (row n)
            if ((*seg_at)[sb] < 0) (*seg_at)[sb] = base;
    }
    c->phase_ms[MH_PHASE_FORMAT] += ms_since(t0);
    return 0;
}

// Rows formatted and written in one stream: the rows are cut into many
// chunks, formatted by host threads in chunk order, and one writer thread
// writes each chunk as soon as it and every chunk before it are done (a
// file's buffered writes are serialised by its inode lock, so one writer
// loses nothing, and the formatting hides under the write).  *crc_out =
// crc32 of everything written.
static int format_write_stream(CtxEx *c, int style, const int64_t *order, int64_t first, int64_t n,
                               const char *const *refnames, int fd, int64_t offset,
                               int64_t *written, uint32_t *crc_out)
{
    const auto t0 = std::chrono::steady_clock::now();
    std::vector<Rec> rec;
    std::vector<uint32_t> pool;
    if (order) {
        if (int st = fetch_recs(c, 0, c->map.n_reads, rec, pool)) return st;
        for (int64_t k = 0; k < n; ++k)
            if (order[first + k] < 0 || order[first + k] >= c->map.n_reads) {
                set_error("format order index out of range");
                return -3;
            }
    } else if (int st = fetch_recs(c, first, n, rec, pool)) {
        return st;
    }
    std::vector<size_t> rn_len(c->index.n_refs > 0 ? (size_t)c->index.n_refs : 1, 0);
    for (int k = 0; k < c->index.n_refs; ++k) rn_len[k] = std::strlen(refnames[k]);
    size_t name_max = 1, ref_max = 1;
    for (size_t r = 0; r < c->names.size(); ++r)
        name_max = std::max(name_max, (size_t)(c->names.off[r + 1] - c->names.off[r]));
    for (int k = 0; k < c->index.n_refs; ++k) ref_max = std::max(ref_max, rn_len[k]);
    const size_t row_max = 2 * name_max + 4 * ref_max + 3 * (size_t)std::max(c->reads.max_len, 1) +
                           12 * MH_MAXOPS + 16 * 12 + 200;
    const int64_t nch = std::max<int64_t>(1, std::min<int64_t>(n / 4096 + 1, 1024));
    std::vector<TextBuf> buf((size_t)nch);
    std::vector<uint32_t> crc((size_t)nch, 0);
    std::unique_ptr<std::atomic<int>[]> done(new std::atomic<int>[(size_t)nch]);
    for (int64_t k = 0; k < nch; ++k) done[k].store(0);
    std::atomic<int64_t> next(0);
    std::mutex mu;
    std::condition_variable cv;
    const int nf = std::max(1, s2a_threads() - 1);
    std::atomic<int> finished(0);
    std::atomic<double> fmt_end(0.0);
    std::vector<std::thread> fmt;
    // a formatter that throws (bad_alloc from a row buffer) stores the
    // exception and raises `failed`; the writer stops waiting on it, every
    // thread is joined, and the exception is rethrown to mh_write_rows_crc
    std::exception_ptr err;
    std::atomic<bool> failed(false);
    auto fail = [&](std::exception_ptr e) {
        {
            std::lock_guard<std::mutex> lk(mu);
            if (!err) err = e;
            failed.store(true);
        }
        next.store(nch);        // no formatter starts another chunk
        cv.notify_all();
    };
    auto worker = [&]() {
        try {
            std::string tmp;
            for (int64_t k; (k = next.fetch_add(1)) < nch;) {
                const int64_t k0 = n * k / nch, k1 = n * (k + 1) / nch;
                TextBuf &out = buf[(size_t)k];
                out.resize((size_t)(k1 - k0) * row_max + 1);
                size_t used = 0;
                for (int64_t j = k0; j < k1; ++j) {
                    const int64_t r = order ? order[first + j] : first + j;
                    format_row(c, style, order ? rec[r] : rec[j], r, pool.data(), refnames, rn_len.data(),
                               out, used, tmp);
                }
                out.resize(used);
                if (crc_out) crc[(size_t)k] = crc32_update(0, out.data(), used);
                {
                    std::lock_guard<std::mutex> lk(mu);
                    done[k].store(1);
                }
                cv.notify_all();
            }
        } catch (...) {
            fail(std::current_exception());
        }
        if (finished.fetch_add(1) + 1 == nf) fmt_end.store(ms_since(t0));
    };
    try {
        for (int t = 0; t < nf; ++t) fmt.emplace_back(worker);
    } catch (...) {
        fail(std::current_exception());
    }
    int bad = 0;
    int64_t pos = offset;
    uint32_t total_crc = 0;
    for (int64_t k = 0; k < nch && !failed.load(); ++k) {
        {
            std::unique_lock<std::mutex> lk(mu);
            cv.wait(lk, [&] { return done[k].load() != 0 || failed.load(); });
        }
        if (failed.load()) break;
        const char *p = buf[(size_t)k].data();
        size_t left = buf[(size_t)k].size();
        if (crc_out) total_crc = crc32_join(total_crc, crc[(size_t)k], (int64_t)left);
        while (left > 0 && !bad) {
            const ssize_t w = pwrite(fd, p, left, (off_t)pos);
            if (w <= 0) { bad = errno ? errno : EIO; break; }
            p += w; left -= (size_t)w; pos += w;
        }
        buf[(size_t)k].release();
    }
    for (auto &t : fmt) t.join();
    if (err) std::rethrow_exception(err);
    // the formatting (overlapped with the first writes), then the write tail
    const double all_ms = ms_since(t0), f_ms = fmt_end.load();
    c->phase_ms[MH_PHASE_FORMAT] += f_ms;
    c->phase_ms[MH_PHASE_WRITE] += all_ms - f_ms;
    if (bad) { set_error("mh_write_rows: write failed (%s)", strerror(bad)); return -4; }
    if (written) *written = pos - offset;
    if (crc_out) *crc_out = total_crc;
    return 0;
}

int mh_write_rows(mh_ctx *ctx, int style, const int64_t *order, int64_t first, int64_t n,
                  const char *const *refnames, int fd, int64_t offset, int64_t *written)
{
    return mh_write_rows_crc(ctx, style, order, first, n, refnames, fd, offset, written, nullptr);
}

int mh_write_rows_crc(mh_ctx *ctx, int style, const int64_t *order, int64_t first, int64_t n,
                      const char *const *refnames, int fd, int64_t offset, int64_t *written,
                      uint32_t *crc)
{
    if (!ctx || !refnames || (style != 0 && style != 1) || fd < 0 || offset < 0 || n < 0) return -3;
    CtxEx *c = X(ctx);
    MH_HIP(hipSetDevice(c->device));
    if ((int64_t)c->names.size() != c->reads.n) { set_error("no read names loaded"); return -3; }
    try {
        return format_write_stream(c, style, order, first, n, refnames, fd, offset, written, crc);
    } catch (const std::bad_alloc &) {
        set_error("mh_write_rows: out of memory");
        return -2;
    } catch (const std::exception &e) {
        set_error("mh_write_rows: %s", e.what());
        return -2;
    }
}

int mh_format_segments(mh_ctx *ctx, int style, const int64_t *order, int64_t n,
                       const char *const *refnames, int n_seg, const int64_t *seg_rows,
                       int64_t *seg_bytes)
{
    if (!ctx || !refnames || (style != 0 && style != 1) || n < 0 || n_seg < 1 || !seg_rows ||
        !seg_bytes) {
        set_error("mh_format_segments: bad arguments");
        return -3;
    }
    // the bounds cover rows 0 .. n exactly: every formatted byte belongs
    // to one segment (mh_write_segments indexes seg_at by segment)
    if (seg_rows[0] != 0 || seg_rows[n_seg] != n) {
        set_error("mh_format_segments: segment bounds must start at row 0 and end at row n");
        return -3;
    }
    for (int k = 0; k < n_seg; ++k)
        if (seg_rows[k] < 0 || seg_rows[k + 1] < seg_rows[k] || seg_rows[k + 1] > n) {
            set_error("mh_format_segments: segment bounds out of order");
            return -3;
        }
    CtxEx *c = X(ctx);
    MH_HIP(hipSetDevice(c->device));
    if ((int64_t)c->names.size() != c->reads.n) { set_error("no read names loaded"); return -3; }
    c->seg_chunks.clear();
    c->seg_at.clear();
    if (int st = format_chunks(c, style, order, 0, n, refnames, c->seg_chunks, n_seg, seg_rows,
                               &c->seg_at))
        return st;
    for (int k = 0; k < n_seg; ++k) seg_bytes[k] = c->seg_at[k + 1] - c->seg_at[k];
    return 0;
}

int mh_write_segments(mh_ctx *ctx, int fd, const int64_t *seg_off, uint32_t *crc)
{
    if (!ctx || fd < 0 || !seg_off) { set_error("mh_write_segments: bad arguments"); return -3; }
    CtxEx *c = X(ctx);
    const int n_seg = (int)c->seg_at.size() - 1;
    if (n_seg < 1) { set_error("mh_write_segments: nothing formatted"); return -3; }
    for (int k = 0; k < n_seg; ++k)
        if (seg_off[k] < 0) { set_error("mh_write_segments: negative offset"); return -3; }
    const auto tw = std::chrono::steady_clock::now();
    std::vector<TextBuf> &ch = c->seg_chunks;
    const int nt = (int)ch.size();
    std::vector<int64_t> cbase(nt + 1, 0);
    for (int t = 0; t < nt; ++t) cbase[t + 1] = cbase[t] + (int64_t)ch[t].size();
    // pieces: a chunk cut at the segment starts; each written at its
    // segment's file offset, its crc32 computed beside the write
    struct Piece { int t, seg; int64_t a, b; uint32_t crc; };
    std::vector<Piece> pieces;
    for (int t = 0; t < nt; ++t) {
        int64_t a = cbase[t];
        while (a < cbase[t + 1]) {
            // the segment holding byte a: the last start <= a with a non-empty span
            int sg = (int)(std::upper_bound(c->seg_at.begin(), c->seg_at.end(), a) - c->seg_at.begin()) - 1;
            while (sg < n_seg - 1 && c->seg_at[sg + 1] <= a) ++sg;
            const int64_t b = std::min(cbase[t + 1], c->seg_at[sg + 1]);
            pieces.push_back(Piece{t, sg, a, b, 0});
            a = b;
        }
    }
    std::vector<WritePiece> wp;
    for (const Piece &p : pieces)
        wp.push_back(WritePiece{ch[p.t].data() + (p.a - cbase[p.t]), (size_t)(p.b - p.a),
                                seg_off[p.seg] + (p.a - c->seg_at[p.seg])});
    if (crc) {
        std::atomic<size_t> next(0);
        const int nw = std::max(1, std::min<int>(s2a_threads(), (int)pieces.size()));
        par_for(nw, [&](int) {
            for (size_t i; (i = next.fetch_add(1)) < pieces.size();)
                pieces[i].crc = crc32_update(0, wp[i].src, wp[i].len);
        });
    }
    const int bad = write_pieces(fd, wp);
    if (crc) {
        for (int k = 0; k < n_seg; ++k) crc[k] = 0;
        for (const Piece &p : pieces) crc[p.seg] = crc32_join(crc[p.seg], p.crc, p.b - p.a);
    }
    c->seg_chunks.clear();
    c->seg_at.clear();
    c->phase_ms[MH_PHASE_WRITE] += ms_since(tw);
    if (bad) { set_error("mh_write_segments: write failed (%s)", strerror(bad)); return -4; }
    return 0;
}

uint32_t mh_crc32_combine(uint32_t a, uint32_t b, int64_t len_b) { return crc32_join(a, b, len_b); }

int mh_file_crc32(int fd, int64_t *size, uint32_t *crc)
{
    if (fd < 0 || !crc) return -3;
    struct stat st;
    if (fstat(fd, &st) != 0) { set_error("mh_file_crc32: fstat failed"); return -4; }
    const int64_t n = (int64_t)st.st_size;
    const int64_t CH = (int64_t)16 << 20;
    const int64_t nc = (n + CH - 1) / CH;
    std::vector<uint32_t> part((size_t)std::max<int64_t>(nc, 1), 0);
    std::atomic<int64_t> next(0);
    std::atomic<int> bad(0);
    const int nt = std::max(1, std::min<int>(s2a_threads(), (int)std::max<int64_t>(nc, 1)));
    par_for(nt, [&](int) {
        std::vector<unsigned char> buf((size_t)CH);
        for (int64_t k; (k = next.fetch_add(1)) < nc;) {
            const int64_t a = k * CH, len = std::min(CH, n - a);
            int64_t got = 0;
            while (got < len) {
                const ssize_t r = pread(fd, buf.data() + got, (size_t)(len - got), (off_t)(a + got));
                if (r <= 0) { bad = 1; return; }
                got += r;
            }
            part[k] = crc32_update(0, buf.data(), (size_t)len);
        }
    });
    if (bad) { set_error("mh_file_crc32: read failed"); return -4; }
    uint32_t c0 = 0;
    for (int64_t k = 0; k < nc; ++k) c0 = crc32_join(c0, part[k], std::min(CH, n - k * CH));
    if (size) *size = n;
    *crc = c0;
    return 0;
}

int mh_phase_times(mh_ctx *ctx, double *ms, int reset)
{
    if (!ctx) return -3;
    CtxEx *c = X(ctx);
    for (int k = 0; k < MH_PHASES; ++k) {
        if (ms) ms[k] = c->phase_ms[k];
        if (reset) c->phase_ms[k] = 0.0;
    }
    return 0;
}

// crc32 and adler32 of a whole open file (zlib's, combined over chunks read
// on host threads): (crc32 << 32) | adler32, and its size.
int mh_file_checksum(int fd, int64_t *size, uint64_t *sum)
{
    if (fd < 0 || !sum) return -3;
    struct stat st;
    if (fstat(fd, &st) != 0) { set_error("mh_file_checksum: fstat failed"); return -4; }
    const int64_t n = (int64_t)st.st_size;
    const int64_t CH = (int64_t)16 << 20;
    const int64_t nc = (n + CH - 1) / CH;
    std::vector<uLong> crc((size_t)std::max<int64_t>(nc, 1)), adl((size_t)std::max<int64_t>(nc, 1));
    std::atomic<int64_t> next(0);
    std::atomic<int> bad(0);
    const int nt = std::max(1, std::min<int>(s2a_threads(), (int)std::max<int64_t>(nc, 1)));
    par_for(nt, [&](int) {
        std::vector<unsigned char> buf((size_t)CH);
        for (int64_t k; (k = next.fetch_add(1)) < nc;) {
            const int64_t a = k * CH, len = std::min(CH, n - a);
            int64_t got = 0;
            while (got < len) {
                const ssize_t r = pread(fd, buf.data() + got, (size_t)(len - got), (off_t)(a + got));
                if (r <= 0) { bad = 1; return; }
                got += r;
            }
            crc[k] = crc32(crc32(0L, Z_NULL, 0), buf.data(), (uInt)len);
            adl[k] = adler32(adler32(0L, Z_NULL, 0), buf.data(), (uInt)len);
        }
    });
    if (bad) { set_error("mh_file_checksum: read failed"); return -4; }
    uLong c0 = crc32(0L, Z_NULL, 0), a0 = adler32(0L, Z_NULL, 0);
    for (int64_t k = 0; k < nc; ++k) {
        const int64_t len = std::min(CH, n - k * CH);
        c0 = crc32_combine(c0, crc[k], (z_off_t)len);
        a0 = adler32_combine(a0, adl[k], (z_off_t)len);
    }
    if (size) *size = n;
    *sum = ((uint64_t)(c0 & 0xffffffffu) << 32) | (uint64_t)(a0 & 0xffffffffu);
    return 0;
}

int mh_format_rows(mh_ctx *ctx, int style, const int64_t *order, int64_t first, int64_t n,
                   const char *const *refnames, char *buf, size_t cap, size_t *used)
{
    if (!ctx || !refnames || (style != 0 && style != 1)) return -3;
    CtxEx *c = X(ctx);
    MH_HIP(hipSetDevice(c->device));
    if ((int64_t)c->names.size() != c->reads.n) { set_error("no read names loaded"); return -3; }
    // the text of a size query (buf NULL) is kept for the copy that follows it
    const uint64_t key = ((uint64_t)style << 62) ^ (uint64_t)(uintptr_t)order * 0x9e3779b97f4a7c15ull ^
                         ((uint64_t)first << 20) ^ (uint64_t)n ^ (uint64_t)c->map_gen * 0x100000001b3ull;
    if (buf && c->fmt_key == key && c->fmt_valid) {
        size_t total = 0;
        for (const TextBuf &t : c->fmt_chunks) total += t.size();
        if (used) *used = total;
        if (total > cap) { set_error("format buffer too small (%zu needed)", total); return -2; }
        size_t at = 0;
        for (const TextBuf &t : c->fmt_chunks) { std::memcpy(buf + at, t.data(), t.size()); at += t.size(); }
        c->fmt_chunks.clear();
        c->fmt_valid = false;
        return 0;
    }
    std::vector<TextBuf> chunks;
    if (int st = format_chunks(c, style, order, first, n, refnames, chunks)) return st;
    size_t total = 0;
    for (const TextBuf &t : chunks) total += t.size();
    if (used) *used = total;
    if (!buf) {
        c->fmt_chunks.swap(chunks);
        c->fmt_key = key;
        c->fmt_valid = true;
        return 0;
    }
    c->fmt_valid = false;
    if (total > cap) { set_error("format buffer too small (%zu needed)", total); return -2; }
    size_t at = 0;
    for (const TextBuf &t : chunks) { std::memcpy(buf + at, t.data(), t.size()); at += t.size(); }
    return 0;
}

int mh_rows_load(mh_ctx *ctx, int64_t n_rows, const int32_t *flag, const int32_t *ref,
                 const int32_t *pos, const int32_t *cigar_off, const int32_t *n_cigar,
                 const uint32_t *cigar, const uint8_t *seq, const uint8_t *qual,
                 const int64_t *offsets, const int32_t *lens, int64_t n_units,
                 const int64_t *unit_rows)
{
    if (!ctx || n_rows < 0 || n_units < 0) return -3;
    CtxEx *c = X(ctx);
    MH_HIP(hipSetDevice(c->device));
    RowState &R = c->rows;
    hipFree(R.flag); hipFree(R.ref); hipFree(R.pos); hipFree(R.cig_off); hipFree(R.n_cigar);
    hipFree(R.cigar); hipFree(R.units);
    R = RowState{};
    // row checks, the CIGAR extent, the hot reference (most mapped rows,
    // smallest id on ties) and the longest reference span, on host threads
    // over contiguous row blocks; the first bad row (in row order) reports
    const int nt = std::max(1, std::min(s2a_threads(), (int)(n_rows >> 16) + 1));
    std::vector<int64_t> t_ncig(nt, 0), t_bad(nt, -1);
    std::vector<int> t_kind(nt, 0), t_span(nt, 0);
    std::vector<char> t_ch(nt, 0);
    std::vector<std::unordered_map<int32_t, int64_t>> t_ref(nt);
    par_for(nt, [&](int t) {
        const int64_t a = n_rows * t / nt, b = n_rows * (t + 1) / nt;
        for (int64_t i = a; i < b; ++i) {
            if (n_cigar[i] < 0 || n_cigar[i] > MH_MAXOPS || cigar_off[i] < 0) {
                t_bad[t] = i; t_kind[t] = 1; return;
            }
            t_ncig[t] = std::max<int64_t>(t_ncig[t], (int64_t)cigar_off[i] + n_cigar[i]);
            int span = 0;
            for (int k = 0; k < n_cigar[i]; ++k) {
                const uint32_t w = cigar[cigar_off[i] + k], op = w & 15;
                if (op != MH_OP_M && op != MH_OP_I && op != MH_OP_D && op != MH_OP_S && op != 3) {
                    t_bad[t] = i; t_kind[t] = 2; return;
                }
                if (op == MH_OP_M || op == MH_OP_D) span += (int)(w >> 4);
            }
            if (!(flag[i] & 4)) {
                for (int x = 0; x < lens[i]; ++x) {
                    const char ch = (char)seq[offsets[i] + x];
                    if (ch != 'A' && ch != 'C' && ch != 'G' && ch != 'T' && ch != 'N') {
                        t_bad[t] = i; t_kind[t] = 3; t_ch[t] = ch; return;
                    }
                }
                t_span[t] = std::max(t_span[t], span);
                ++t_ref[t][ref[i]];
            }
        }
    });
    for (int t = 0; t < nt; ++t) {
        if (t_bad[t] < 0) continue;
        const long long i = (long long)t_bad[t];
        if (t_kind[t] == 1) set_error("rows: bad cigar in row %lld", i);
        else if (t_kind[t] == 2) set_error("Unsupported CIGAR token in row %lld", i);
        else set_error("row %lld: base letter '%c' (only ACGTN as bowtie2 prints)", i, t_ch[t]);
        return -3;
    }
    int64_t ncig = 0;
    {
        std::unordered_map<int32_t, int64_t> per_ref;
        for (int t = 0; t < nt; ++t) {
            ncig = std::max(ncig, t_ncig[t]);
            R.max_span = std::max(R.max_span, t_span[t]);
            for (auto &kv : t_ref[t]) per_ref[kv.first] += kv.second;
        }
        int64_t best = 0;
        for (auto &kv : per_ref) {
            if (kv.second > best || (kv.second == best && kv.first < R.hot_ref)) {
                best = kv.second;
                R.hot_ref = kv.first;
            }
            if (kv.first >= 0) {
                if ((size_t)kv.first >= R.ref_rows.size()) R.ref_rows.resize((size_t)kv.first + 1, 0);
                R.ref_rows[(size_t)kv.first] += kv.second;
            }
        }
    }
    const int64_t nr = n_rows > 0 ? n_rows : 1;
    MH_HIP(hipMalloc(&R.flag, sizeof(int32_t) * nr));
    MH_HIP(hipMalloc(&R.ref, sizeof(int32_t) * nr));
    MH_HIP(hipMalloc(&R.pos, sizeof(int32_t) * nr));
    MH_HIP(hipMalloc(&R.cig_off, sizeof(int32_t) * nr));
    MH_HIP(hipMalloc(&R.n_cigar, sizeof(int32_t) * nr));
    MH_HIP(hipMalloc(&R.cigar, sizeof(uint32_t) * (ncig > 0 ? ncig : 1)));
    MH_HIP(hipMalloc(&R.units, sizeof(int64_t) * 2 * (n_units > 0 ? n_units : 1)));
    if (n_rows > 0) {
        MH_HIP(copy_sync(*c, R.flag, flag, sizeof(int32_t) * n_rows, hipMemcpyHostToDevice));
        MH_HIP(copy_sync(*c, R.ref, ref, sizeof(int32_t) * n_rows, hipMemcpyHostToDevice));
        MH_HIP(copy_sync(*c, R.pos, pos, sizeof(int32_t) * n_rows, hipMemcpyHostToDevice));
        MH_HIP(copy_sync(*c, R.cig_off, cigar_off, sizeof(int32_t) * n_rows, hipMemcpyHostToDevice));
        MH_HIP(copy_sync(*c, R.n_cigar, n_cigar, sizeof(int32_t) * n_rows, hipMemcpyHostToDevice));
    }
    if (ncig > 0) MH_HIP(copy_sync(*c, R.cigar, cigar, sizeof(uint32_t) * ncig, hipMemcpyHostToDevice));
    if (n_units > 0)
        MH_HIP(copy_sync(*c, R.units, unit_rows, sizeof(int64_t) * 2 * n_units, hipMemcpyHostToDevice));
    R.n_rows = n_rows;
    R.n_units = n_units;
    HostReads dummy;
    return load_reads(*c, R.reads, dummy, n_rows, 0, seq, qual, offsets, lens, false);
}

// ---- prelim.csv reader ------------------------------------------------------
// std::atoi on a string_view (leading blanks and sign, then digits)
static int sv_atoi(std::string_view v)
{
    size_t i = 0;
    while (i < v.size() && (v[i] == ' ' || v[i] == '\t')) ++i;
    bool neg = false;
    if (i < v.size() && (v[i] == '-' || v[i] == '+')) neg = v[i++] == '-';
    long long x = 0;
    while (i < v.size() && v[i] >= '0' && v[i] <= '9') x = x * 10 + (v[i++] - '0');
    return (int)(neg ? -x : x);
}

// csv.DictReader semantics for the 11 SAM columns prelim_map writes
// (prelim_map.py:142-151), then remap.matchmaker (remap.py:853-889) over the
// rows whose rname is in the @SQ set, then the rows go to the device.
namespace mh {
struct CsvRows {
    std::vector<int32_t> flag, ref, pos, cig_off, n_cigar, maxm, name_id;
    std::vector<uint32_t> cigar;
    std::vector<uint8_t> seq, qual;
    std::vector<int64_t> off;
    std::vector<int32_t> len;
    std::vector<int64_t> units;
    std::vector<std::string> qnames_own;   // serial (quoted) path: owned names
};

}  // namespace mh

extern "C" int mh_rows_load_csv(mh_ctx *ctx, const char *text, int64_t len, int n_refs,
                                const char *const *refnames, int64_t *n_rows, int64_t *n_units,
                                int32_t *n_present)
{
    if (!ctx || !text || len < 0 || n_refs < 0) return -3;
    CtxEx *c = X(ctx);
    std::unordered_map<std::string, int> refidx;
    for (int r = 0; r < n_refs; ++r) refidx.emplace(refnames[r], r);
    const char *p = text, *end = text + len;
    std::vector<std::string> f;
    if (!csv_record(p, end, f)) { set_error("prelim csv: empty"); return -3; }
    const char *want[11] = {"qname", "flag", "rname", "pos", "mapq", "cigar", "rnext", "pnext",
                            "tlen", "seq", "qual"};
    int col[11];
    for (int k = 0; k < 11; ++k) {
        col[k] = -1;
        for (size_t z = 0; z < f.size(); ++z) if (f[z] == want[k]) col[k] = (int)z;
        if (col[k] < 0) { set_error("prelim csv: missing column %s", want[k]); return -3; }
    }
    CsvRows R;
    std::vector<std::string_view> qnames;   // per row, into text
    std::unordered_map<std::string, int> unknown;
    std::vector<uint32_t> ops;
    bool parallel_ok = true;
    std::vector<std::deque<std::string>> pown;   // unescaped names (stable addresses; qnames views them)
    {
        // rows parsed on host threads in contiguous blocks cut at record
        // ends (a newline outside quotes: the count of '"' before it is
        // even), concatenated in order.  A record this parser does not take
        // (a newline inside a quoted field, text after a closing quote)
        // sends the whole file to the serial csv_record path below.
        int ncol = 11;   // fields a row needs: up to the last column used
        for (int k = 0; k < 11; ++k) ncol = std::max(ncol, col[k] + 1);
        const int64_t bytes = end - p;
        const int nt = std::max(1, std::min(s2a_threads(), (int)(bytes >> 22) + 1));
        std::vector<const char *> cut(nt + 1);
        cut[0] = p;
        cut[nt] = end;
        for (int t = 1; t < nt; ++t) {
            const char *q = p + bytes * t / nt;
            if (q < cut[t - 1]) q = cut[t - 1];
            const char *nl = (const char *)std::memchr(q, '\n', (size_t)(end - q));
            cut[t] = nl ? nl + 1 : end;
        }
        std::vector<int64_t> nq(nt, 0);
        par_for(nt, [&](int t) {
            int64_t k = 0;
            for (const char *q = cut[t]; q < cut[t + 1]; ++q) k += *q == '"';
            nq[t] = k;
        });
        int64_t par = 0;
        for (int t = 1; t < nt; ++t) {
            par += nq[t - 1];
            if (par & 1) {   // this cut is inside a quoted field: move it on
                const char *q = cut[t];
                int64_t seen = 0;
                while (q < end && !(*q == '\n' && ((par + seen) & 1) == 0)) seen += *q++ == '"';
                cut[t] = q < end ? q + 1 : end;
                if (cut[t] > cut[t + 1]) cut[t + 1] = cut[t];
                par += seen;
                nq[t] -= seen;
            }
        }
        std::vector<CsvRows> part(nt);
        std::vector<std::vector<std::string_view>> pq(nt);
        std::vector<std::vector<std::string>> punk(nt);
        pown.resize(nt);
        std::vector<int> bad(nt, 0);
        par_for(nt, [&](int t) {
            CsvRows &P = part[t];
            std::vector<uint32_t> lops;
            std::vector<std::string_view> fv;
            std::vector<char> fe;   // field holds "" escapes
            std::string tmp, last_rname = "\x01", cig, seqv;
            int last_ref = -1;
            P.flag.reserve((size_t)((cut[t + 1] - cut[t]) / 500 + 16));
            auto value = [&](size_t i) -> std::string_view {   // unescaped view (tmp may back it)
                if (!fe[i]) return fv[i];
                tmp.clear();
                for (size_t x = 0; x < fv[i].size(); ++x) {
                    tmp.push_back(fv[i][x]);
                    if (fv[i][x] == '"') ++x;
                }
                return std::string_view(tmp);
            };
            const char *q = cut[t], *e = cut[t + 1];
            while (q < e) {
                const char *nl = (const char *)std::memchr(q, '\n', (size_t)(e - q));
                const char *le = nl ? nl : e;
                const char *next = nl ? nl + 1 : e;
                if (le > q && le[-1] == '\r') --le;
                fv.clear();
                fe.clear();
                for (const char *s0 = q;;) {
                    if (s0 < le && *s0 == '"') {
                        const char *c0 = s0 + 1, *x = c0;
                        bool esc = false, closed = false;
                        while (x < le) {
                            if (*x == '"') {
                                if (x + 1 < le && x[1] == '"') { esc = true; x += 2; continue; }
                                closed = true;
                                break;
                            }
                            ++x;
                        }
                        if (!closed || (x + 1 < le && x[1] != ',')) { bad[t] = 1; return; }
                        fv.emplace_back(c0, (size_t)(x - c0));
                        fe.push_back(esc);
                        if (x + 1 >= le) break;
                        s0 = x + 2;
                        continue;
                    }
                    const char *cm = (const char *)std::memchr(s0, ',', (size_t)(le - s0));
                    if (!cm) { fv.emplace_back(s0, (size_t)(le - s0)); fe.push_back(0); break; }
                    fv.emplace_back(s0, (size_t)(cm - s0));
                    fe.push_back(0);
                    s0 = cm + 1;
                }
                q = next;
                if (fv.size() == 1 && fv[0].empty()) continue;
                if ((int)fv.size() < ncol) { bad[t] = 2; return; }
                // rows come grouped by rname: look a name up only when it changes
                const std::string_view rn = value(col[2]);
                if (rn != last_rname) {
                    last_rname.assign(rn.data(), rn.size());
                    auto it = refidx.find(last_rname);
                    last_ref = it == refidx.end() ? -1 : it->second;
                }
                const int ref = last_ref;
                const int flag = sv_atoi(value(col[1]));
                int maxm = 0;
                P.cig_off.push_back((int32_t)P.cigar.size());
                if (!(flag & 4)) {
                    cig.assign(value(col[5]));
                    if (!parse_cigar_ops(cig, lops, maxm)) lops.assign(1, 3u);
                    if (lops.size() > MH_MAXOPS) lops.assign(1, 3u);
                } else {
                    lops.clear();
                }
                P.cigar.insert(P.cigar.end(), lops.begin(), lops.end());
                P.n_cigar.push_back((int32_t)lops.size());
                P.flag.push_back(flag);
                P.ref.push_back(ref);
                P.name_id.push_back(ref);
                P.pos.push_back(sv_atoi(value(col[3])));
                P.maxm.push_back(maxm);
                seqv.assign(value(col[9]));   // (escapes are possible in principle)
                const std::string_view quals = value(col[10]);
                P.off.push_back((int64_t)P.seq.size());
                P.len.push_back((int32_t)seqv.size());
                P.seq.insert(P.seq.end(), seqv.begin(), seqv.end());
                const size_t nqk = std::min(quals.size(), seqv.size());
                P.qual.insert(P.qual.end(), quals.begin(), quals.begin() + nqk);
                P.qual.insert(P.qual.end(), seqv.size() - nqk, 'J');
                if (fe[col[0]]) {
                    pown[t].emplace_back(value(col[0]));
                    pq[t].emplace_back(pown[t].back());
                } else {
                    pq[t].push_back(fv[col[0]]);
                }
                punk[t].push_back(ref < 0 ? last_rname : std::string());
            }
        });
        for (int t = 0; t < nt; ++t)
            if (bad[t] == 1) parallel_ok = false;
        if (parallel_ok)
            for (int t = 0; t < nt; ++t)
                if (bad[t] == 2) { set_error("prelim csv: short row"); return -3; }
        if (parallel_ok) {
            // sizes, then every part copied to its place on its own thread
            std::vector<int64_t> rb(nt + 1, 0), cb(nt + 1, 0), sb(nt + 1, 0);
            for (int t = 0; t < nt; ++t) {
                rb[t + 1] = rb[t] + (int64_t)part[t].flag.size();
                cb[t + 1] = cb[t] + (int64_t)part[t].cigar.size();
                sb[t + 1] = sb[t] + (int64_t)part[t].seq.size();
            }
            const int64_t nrw = rb[nt];
            R.flag.resize(nrw); R.ref.resize(nrw); R.pos.resize(nrw); R.cig_off.resize(nrw);
            R.n_cigar.resize(nrw); R.maxm.resize(nrw); R.name_id.resize(nrw); R.off.resize(nrw);
            R.len.resize(nrw); R.cigar.resize(cb[nt]); R.seq.resize(sb[nt]); R.qual.resize(sb[nt]);
            qnames.resize(nrw);
            for (int t = 0; t < nt; ++t)   // '*' and other names outside @SQ, ids in first-seen order
                for (size_t i = 0; i < part[t].flag.size(); ++i)
                    if (part[t].ref[i] < 0) {
                        auto u = unknown.emplace(punk[t][i], (int)unknown.size());
                        part[t].name_id[i] = -1 - u.first->second;
                    }
            par_for(nt, [&](int t) {
                const CsvRows &P = part[t];
                const size_t n0 = P.flag.size(), r0 = (size_t)rb[t];
                std::copy(P.flag.begin(), P.flag.end(), R.flag.begin() + r0);
                std::copy(P.ref.begin(), P.ref.end(), R.ref.begin() + r0);
                std::copy(P.pos.begin(), P.pos.end(), R.pos.begin() + r0);
                std::copy(P.n_cigar.begin(), P.n_cigar.end(), R.n_cigar.begin() + r0);
                std::copy(P.maxm.begin(), P.maxm.end(), R.maxm.begin() + r0);
                std::copy(P.name_id.begin(), P.name_id.end(), R.name_id.begin() + r0);
                std::copy(P.len.begin(), P.len.end(), R.len.begin() + r0);
                for (size_t i = 0; i < n0; ++i) {
                    R.cig_off[r0 + i] = P.cig_off[i] + (int32_t)cb[t];
                    R.off[r0 + i] = P.off[i] + sb[t];
                }
                std::copy(P.cigar.begin(), P.cigar.end(), R.cigar.begin() + cb[t]);
                std::copy(P.seq.begin(), P.seq.end(), R.seq.begin() + sb[t]);
                std::copy(P.qual.begin(), P.qual.end(), R.qual.begin() + sb[t]);
                std::copy(pq[t].begin(), pq[t].end(), qnames.begin() + r0);
            });
        }
    }
    if (!parallel_ok) {
        while (csv_record(p, end, f)) {
            if (f.size() == 1 && f[0].empty()) continue;
            if ((int)f.size() < 11) { set_error("prelim csv: short row"); return -3; }
            const std::string &rname = f[col[2]], &seqs = f[col[9]], &quals = f[col[10]];
            const int flag = std::atoi(f[col[1]].c_str());
            auto it = refidx.find(rname);
            int ref = it == refidx.end() ? -1 : it->second;
            int nid = ref;
            if (ref < 0) {
                auto u = unknown.emplace(rname, (int)unknown.size());
                nid = -1 - u.first->second;   // '*' and other names outside @SQ
            }
            int maxm = 0;
            R.cig_off.push_back((int32_t)R.cigar.size());
            if (!(flag & 4)) {
                if (!parse_cigar_ops(f[col[5]], ops, maxm)) ops.assign(1, 3u);  // invalid: fails if used
                if (ops.size() > MH_MAXOPS) ops.assign(1, 3u);
            } else {
                ops.clear();
            }
            R.cigar.insert(R.cigar.end(), ops.begin(), ops.end());
            R.n_cigar.push_back((int32_t)ops.size());
            R.flag.push_back(flag);
            R.ref.push_back(ref);
            R.name_id.push_back(nid);
            R.pos.push_back(std::atoi(f[col[3]].c_str()));
            R.maxm.push_back(maxm);
            R.off.push_back((int64_t)R.seq.size());
            R.len.push_back((int32_t)seqs.size());
            R.seq.insert(R.seq.end(), seqs.begin(), seqs.end());
            std::string q = quals;
            q.resize(seqs.size(), 'J');
            R.qual.insert(R.qual.end(), q.begin(), q.end());
            R.qnames_own.push_back(f[col[0]]);
        }
        for (const std::string &x : R.qnames_own) qnames.emplace_back(x);
    }
    // matchmaker (remap.py:853-889) over the rows whose rname is in @SQ
    const int64_t nrow = (int64_t)R.flag.size();
    std::unordered_map<std::string_view, int64_t> pending;   // qname -> slot in order
    pending.reserve((size_t)nrow);
    std::vector<std::pair<int64_t, bool>> order;             // (row, alive) insertion order
    order.reserve((size_t)nrow);
    for (int64_t row = 0; row < nrow; ++row) {
        if (R.ref[row] < 0) continue;
        const std::string_view qname = qnames[row];
        auto pit = pending.find(qname);
        if (pit == pending.end()) {
            pending.emplace(qname, (int64_t)order.size());
            order.push_back({row, true});
        } else {
            order[pit->second].second = false;
            R.units.push_back(order[pit->second].first);
            R.units.push_back(row);
            pending.erase(pit);
        }
    }
    for (auto &o : order) if (o.second) { R.units.push_back(o.first); R.units.push_back(-1); }
    const int64_t nr = (int64_t)R.flag.size();
    const int64_t nu = (int64_t)R.units.size() / 2;
    // compact reference ids: only references some unit row names, in @SQ
    // order (keeps the dense counters small); rows outside @SQ are never
    // paired and get compact id 0 (unused)
    std::vector<int32_t> used(n_refs > 0 ? n_refs : 1, 0);
    for (int64_t k = 0; k < 2 * nu; ++k) if (R.units[k] >= 0) used[R.ref[R.units[k]]] = 1;
    std::vector<int32_t> compact(n_refs > 0 ? n_refs : 1, -1);
    c->csv_present.clear();
    for (int r = 0; r < n_refs; ++r)
        if (used[r]) { compact[r] = (int32_t)c->csv_present.size(); c->csv_present.push_back(r); }
    std::vector<int32_t> dref(R.ref);
    for (auto &x : dref) x = (x >= 0 && compact[x] >= 0) ? compact[x] : 0;
    c->csv_unknown.assign(unknown.size(), std::string());
    for (auto &kv : unknown) c->csv_unknown[kv.second] = kv.first;
    int st = mh_rows_load(ctx, nr, R.flag.data(), dref.data(), R.pos.data(), R.cig_off.data(),
                          R.n_cigar.data(), R.cigar.empty() ? nullptr : R.cigar.data(),
                          R.seq.data(), R.qual.data(), R.off.data(), R.len.data(), nu,
                          R.units.data());
    if (st) return st;
    c->csv_rows_info.clear();
    c->csv_rows_info.reserve(nr * 4);
    for (int64_t i = 0; i < nr; ++i) {
        c->csv_rows_info.push_back(R.name_id[i]);
        c->csv_rows_info.push_back(R.flag[i]);
        c->csv_rows_info.push_back(R.maxm[i]);
        c->csv_rows_info.push_back(dref[i]);
    }
    if (n_rows) *n_rows = nr;
    if (n_units) *n_units = nu;
    if (n_present) *n_present = (int32_t)c->csv_present.size();
    return 0;
}

extern "C" int mh_rows_info(mh_ctx *ctx, int32_t *out4, int32_t *present, char *unknown,
                            size_t cap)
{
    if (!ctx) return -3;
    CtxEx *c = X(ctx);
    if (out4) std::memcpy(out4, c->csv_rows_info.data(), sizeof(int32_t) * c->csv_rows_info.size());
    if (present) std::memcpy(present, c->csv_present.data(), sizeof(int32_t) * c->csv_present.size());
    if (unknown) {
        std::string all;
        for (auto &u : c->csv_unknown) { all += u; all.push_back('\n'); }
        if (all.size() + 1 > cap) { set_error("mh_rows_info: name buffer too small"); return -2; }
        std::memcpy(unknown, all.c_str(), all.size() + 1);
    }
    return 0;
}

extern "C" int mh_reads_fastq_lines(mh_ctx *ctx, int64_t *lines1)
{
    if (!ctx || !lines1) return -3;
    *lines1 = X(ctx)->fastq_lines1;
    return 0;
}

int mh_pileup(mh_ctx *ctx, int source, int q_cutoff, int n_refs, const int32_t *ref_lens)
{
    return mh_pileup_only(ctx, source, q_cutoff, n_refs, ref_lens, -1, nullptr);
}

int mh_pileup_only(mh_ctx *ctx, int source, int q_cutoff, int n_refs, const int32_t *ref_lens, int n_sel,
                   const int32_t *sel)
{
    if (!ctx || n_refs < 0 || (n_refs > 0 && !ref_lens) || (source != 0 && source != 1) ||
        (n_sel > 0 && !sel))
        return -3;
    CtxEx *c = X(ctx);
    MH_HIP(hipSetDevice(c->device));
    c->pile.only.clear();
    if (n_sel >= 0) {
        c->pile.only.assign((size_t)n_refs, 0);
        for (int k = 0; k < n_sel; ++k) {
            if (sel[k] < 0 || sel[k] >= n_refs) { set_error("mh_pileup_only: reference %d out of range", sel[k]); return -3; }
            c->pile.only[(size_t)sel[k]] = 1;
        }
    }
    int32_t cap = 1;
    for (int r = 0; r < n_refs; ++r) cap = std::max(cap, ref_lens[r] + MH_PILEUP_SLACK);
    c->pile.n_refs = n_refs;
    c->pile.cap = cap;
    c->pile.ref_lens.assign(ref_lens, ref_lens + n_refs);
    c->pile.land_ok = false;
    int st = run_pileup(*c, source, q_cutoff);
    if (st == 0) {
        PileState &P = c->pile;
        const size_t nr = (size_t)P.n_refs, need = 16 * nr + 4 * nr + 64;
        if (P.land_cap < need) {
            if (P.land) hipHostFree(P.land);
            P.land = nullptr;
            P.land_cap = 0;
            if (hipHostMalloc((void **)&P.land, need, hipHostMallocDefault) == hipSuccess) P.land_cap = need;
            else P.land = nullptr;
        }
        if (P.land && P.read_counts && P.first_unit && P.max_pos) {
            bool ok = hipMemcpyAsync(P.land, P.read_counts, 8 * nr, hipMemcpyDeviceToHost, c->stream) == hipSuccess &&
                      hipMemcpyAsync(P.land + 8 * nr, P.first_unit, 8 * nr, hipMemcpyDeviceToHost, c->stream) == hipSuccess &&
                      hipMemcpyAsync(P.land + 16 * nr, P.max_pos, 4 * nr, hipMemcpyDeviceToHost, c->stream) == hipSuccess;
            if (ok && P.ev_counters)
                ok = hipMemcpyAsync(P.land + ((20 * nr + 7) & ~(size_t)7), P.ev_counters, 32,
                                    hipMemcpyDeviceToHost, c->stream) == hipSuccess;
            P.land_ok = ok;
        }
        MH_HIP(hipStreamSynchronize(c->stream));
    }
    prof_flush(*c);
    return st;
}

// The kernel emits one event per merged pair and position carrying a base +
// insertion token; a pass over a 3-base insertion site yields one per
// covering pair.  They are aggregated here to (ref, pos, token) -> count, in
// (ref, pos, token) order, so the host never handles per-pair records.
static int aggregate_tokens(CtxEx &c)
{
    PileState &P = c.pile;
    if (c.tok_gen == P.gen) return 0;
    c.tok_ref.clear(); c.tok_pos.clear(); c.tok_off.clear(); c.tok_len.clear();
    c.tok_count.clear(); c.tok_pool.clear();
    int64_t ctr[4] = {0, 0, 0, 0};
    if (P.ev_counters && P.land_ok)   // landed behind mh_pileup
        std::memcpy(ctr, P.land + ((20 * (size_t)P.n_refs + 7) & ~(size_t)7), sizeof(ctr));
    else if (P.ev_counters)
        MH_HIP(copy_sync(c, ctr, P.ev_counters, sizeof(ctr), hipMemcpyDeviceToHost));
    const int64_t ne = ctr[0];
    if (ne > 0) {
        // distinct (ref, pos, token) keys and their counts come from the
        // device (run_token_aggregate); only their order is fixed here
        std::vector<int32_t> meta;
        std::string bytes;
        if (int st = run_token_aggregate(c, ne, ctr[1], meta, bytes)) return st;
        struct Key { int32_t ref, pos, off, len; int64_t count; };
        const size_t nd = meta.size() / 5;
        std::vector<Key> uniq(nd);
        for (size_t d = 0; d < nd; ++d)
            uniq[d] = Key{meta[5 * d], meta[5 * d + 1], meta[5 * d + 2], meta[5 * d + 3], meta[5 * d + 4]};
        const char *pb = bytes.data();
        std::sort(uniq.begin(), uniq.end(), [pb](const Key &a, const Key &b) {
            if (a.ref != b.ref) return a.ref < b.ref;
            if (a.pos != b.pos) return a.pos < b.pos;
            const int cmp = std::memcmp(pb + a.off, pb + b.off, (size_t)std::min(a.len, b.len));
            if (cmp != 0) return cmp < 0;
            return a.len < b.len;
        });
        for (const Key &k : uniq) {
            c.tok_ref.push_back(k.ref);
            c.tok_pos.push_back(k.pos);
            c.tok_off.push_back((int32_t)c.tok_pool.size());
            c.tok_len.push_back(k.len);
            c.tok_count.push_back(k.count);
            c.tok_pool.append(pb + k.off, (size_t)k.len);
        }
    }
    c.tok_gen = P.gen;
    return 0;
}

int mh_pileup_dims(mh_ctx *ctx, int *n_refs, int32_t *cap, int64_t *n_events, int64_t *event_bytes)
{
    if (!ctx) return -3;
    CtxEx *c = X(ctx);
    PileState &P = c->pile;
    if (n_refs) *n_refs = P.n_refs;
    if (cap) *cap = P.cap;
    MH_HIP(hipSetDevice(c->device));
    if (int st = aggregate_tokens(*c)) return st;
    if (n_events) *n_events = (int64_t)c->tok_ref.size();
    if (event_bytes) *event_bytes = (int64_t)c->tok_pool.size();
    return 0;
}

// Device-to-host copies of up to 6 (source, size, destination) parts: the
// parts go through the context's pinned staging buffer with one stream
// synchronisation; parts too large for it are copied directly.
struct FetchPart {
    const void *src;
    size_t bytes;
    void *dst;
};

static int fetch_parts(CtxEx &c, const FetchPart *parts, int n)
{
    size_t total = 0;
    for (int i = 0; i < n; ++i) if (parts[i].dst) total += (parts[i].bytes + 255) & ~(size_t)255;
    if (total > ((size_t)64 << 20)) {   // large fetches (all 74 seeds): plain copies
        for (int i = 0; i < n; ++i)
            if (parts[i].dst && parts[i].bytes)
                MH_HIP(copy_sync(c, parts[i].dst, parts[i].src, parts[i].bytes, hipMemcpyDeviceToHost));
        return 0;
    }
    if (c.pin_cap < total) {
        if (c.pin) hipHostFree(c.pin);
        c.pin = nullptr;
        c.pin_cap = 0;
        const size_t cap = total > ((size_t)1 << 20) ? total : ((size_t)1 << 20);
        MH_HIP(hipHostMalloc(&c.pin, cap, hipHostMallocDefault));
        c.pin_cap = cap;
    }
    size_t at = 0;
    for (int i = 0; i < n; ++i) {
        if (!parts[i].dst) continue;
        if (parts[i].bytes)
            MH_HIP(hipMemcpyAsync((char *)c.pin + at, parts[i].src, parts[i].bytes, hipMemcpyDeviceToHost,
                                  c.stream));
        at += (parts[i].bytes + 255) & ~(size_t)255;
    }
    MH_HIP(hipStreamSynchronize(c.stream));
    at = 0;
    for (int i = 0; i < n; ++i) {
        if (!parts[i].dst) continue;
        if (parts[i].bytes) std::memcpy(parts[i].dst, (const char *)c.pin + at, parts[i].bytes);
        at += (parts[i].bytes + 255) & ~(size_t)255;
    }
    return 0;
}

int mh_pileup_fetch(mh_ctx *ctx, int32_t *dense, uint8_t *nflag, uint8_t *dflag,
                    int64_t *read_counts, int64_t *first_unit, int32_t *max_pos)
{
    if (!ctx) return -3;
    CtxEx *c = X(ctx);
    PileState &P = c->pile;
    if (!P.dense) { set_error("no pileup (call mh_pileup)"); return -3; }
    MH_HIP(hipSetDevice(c->device));
    const size_t cells = (size_t)P.n_refs * P.cap, nr = (size_t)P.n_refs;
    if (!dense && !nflag && !dflag && P.land_ok) {   // the scalars, landed behind mh_pileup
        if (read_counts) std::memcpy(read_counts, P.land, 8 * nr);
        if (first_unit) std::memcpy(first_unit, P.land + 8 * nr, 8 * nr);
        if (max_pos) std::memcpy(max_pos, P.land + 16 * nr, 4 * nr);
        return 0;
    }
    const FetchPart parts[6] = {{P.dense, sizeof(int32_t) * 4 * cells, dense},
                                {P.nflag, cells, nflag},
                                {P.dflag, cells, dflag},
                                {P.read_counts, sizeof(int64_t) * nr, read_counts},
                                {P.first_unit, sizeof(int64_t) * nr, first_unit},
                                {P.max_pos, sizeof(int32_t) * nr, max_pos}};
    return fetch_parts(*c, parts, 6);
}

int mh_pileup_fetch_ref(mh_ctx *ctx, int ref, int32_t *dense, uint8_t *nflag, uint8_t *dflag)
{
    if (!ctx) return -3;
    CtxEx *c = X(ctx);
    PileState &P = c->pile;
    if (!P.dense) { set_error("no pileup (call mh_pileup)"); return -3; }
    if (ref < 0 || ref >= P.n_refs) { set_error("mh_pileup_fetch_ref: ref %d out of range", ref); return -3; }
    MH_HIP(hipSetDevice(c->device));
    const int64_t base = (int64_t)ref * P.cap;
    const FetchPart parts[3] = {{P.dense + 4 * base, sizeof(int32_t) * 4 * (size_t)P.cap, dense},
                                {P.nflag + base, (size_t)P.cap, nflag},
                                {P.dflag + base, (size_t)P.cap, dflag}};
    return fetch_parts(*c, parts, 3);
}

int mh_pileup_fetch_refs(mh_ctx *ctx, int n_sel, const int32_t *refs, int32_t *dense, uint8_t *nflag,
                         uint8_t *dflag)
{
    if (!ctx || n_sel < 0 || (n_sel > 0 && (!refs || !dense || !nflag || !dflag))) return -3;
    CtxEx *c = X(ctx);
    PileState &P = c->pile;
    if (!P.dense) { set_error("no pileup (call mh_pileup)"); return -3; }
    MH_HIP(hipSetDevice(c->device));
    // each reference's last counted position (landed behind mh_pileup, else fetched)
    std::vector<int32_t> mx((size_t)std::max(P.n_refs, 1));
    if (P.land_ok && P.land)
        std::memcpy(mx.data(), P.land + 16 * (size_t)P.n_refs, sizeof(int32_t) * (size_t)P.n_refs);
    else
        MH_HIP(copy_sync(*c, mx.data(), P.max_pos, sizeof(int32_t) * (size_t)P.n_refs, hipMemcpyDeviceToHost));
    std::vector<FetchPart> parts;
    parts.reserve(3 * (size_t)n_sel);
    for (int k = 0; k < n_sel; ++k) {
        const int r = refs[k];
        if (r < 0 || r >= P.n_refs) { set_error("mh_pileup_fetch_refs: ref %d out of range", r); return -3; }
        const int64_t rows = std::min<int64_t>(P.cap, std::max(mx[(size_t)r], 0));
        if (rows == 0) continue;
        const int64_t base = (int64_t)r * P.cap;
        parts.push_back({P.dense + 4 * base, sizeof(int32_t) * 4 * (size_t)rows, dense + 4 * base});
        parts.push_back({P.nflag + base, (size_t)rows, nflag + base});
        parts.push_back({P.dflag + base, (size_t)rows, dflag + base});
    }
    return parts.empty() ? 0 : fetch_parts(*c, parts.data(), (int)parts.size());
}

int mh_pileup_events(mh_ctx *ctx, int32_t *ref, int32_t *pos, int32_t *tok_off, int32_t *tok_len,
                     int64_t *count, char *pool)
{
    if (!ctx) return -3;
    CtxEx *c = X(ctx);
    MH_HIP(hipSetDevice(c->device));
    if (int st = aggregate_tokens(*c)) return st;
    const size_t n = c->tok_ref.size();
    if (ref) std::memcpy(ref, c->tok_ref.data(), sizeof(int32_t) * n);
    if (pos) std::memcpy(pos, c->tok_pos.data(), sizeof(int32_t) * n);
    if (tok_off) std::memcpy(tok_off, c->tok_off.data(), sizeof(int32_t) * n);
    if (tok_len) std::memcpy(tok_len, c->tok_len.data(), sizeof(int32_t) * n);
    if (count) std::memcpy(count, c->tok_count.data(), sizeof(int64_t) * n);
    if (pool) std::memcpy(pool, c->tok_pool.data(), c->tok_pool.size());
    return 0;
}

int mh_gotoh_align(mh_ctx *ctx, const char *seq1, const char *seq2, int gop, int gep,
                   int is_global, const char *alphabet, const int *matrix, char *out1, char *out2,
                   int cap, int *score)
{
    if (!ctx || !seq1 || !seq2 || !alphabet || !matrix || !out1 || !out2 || !score) return -3;
    CtxEx *c = X(ctx);
    MH_HIP(hipSetDevice(c->device));
    return run_gotoh(*c, seq1, seq2, gop, gep, is_global, alphabet, matrix, out1, out2, cap, score);
}

int mh_gotoh_align_batch(mh_ctx *ctx, int count, const char *const *seq1,
                         const char *const *seq2, int gop, int gep, int is_global,
                         const char *alphabet, const int *matrix, char *const *out1,
                         char *const *out2, const int *cap, int *score, int *status)
{
    if (!ctx || count < 0 || (count > 0 && (!seq1 || !seq2 || !out1 || !out2 || !cap || !score ||
                                            !status)) || !alphabet || !matrix)
        return -3;
    CtxEx *c = X(ctx);
    MH_HIP(hipSetDevice(c->device));
    return run_gotoh_batch(*c, count, seq1, seq2, gop, gep, is_global, alphabet, matrix, out1,
                           out2, cap, score, status);
}

int mh_gotoh_distance_batch(mh_ctx *ctx, int count, const char *const *seq1, const char *const *seq2,
                            const char *const *text, int gop, int gep, int is_global,
                            const char *alphabet, const int *matrix, int *dist, int *score, int *status)
{
    if (!ctx || count < 0 || (count > 0 && (!seq1 || !seq2 || !text || !dist || !score || !status)) ||
        !alphabet || !matrix)
        return -3;
    CtxEx *c = X(ctx);
    MH_HIP(hipSetDevice(c->device));
    return run_gotoh_distance_batch(*c, count, seq1, seq2, text, gop, gep, is_global, alphabet, matrix,
                                    dist, score, status);
}

int mh_top_tokens(int32_t length, int32_t rows, const int32_t *dense, const uint8_t *nflag,
                  const uint8_t *dflag, const char *seed, int32_t seed_len, uint8_t *tok,
                  int32_t *any_positive)
{
    if (length < 0 || rows < 0 || (rows > 0 && (!dense || !nflag || !dflag)) || (length > 0 && !tok) ||
        seed_len < 0 || (seed_len > 0 && !seed))
        return -3;
    // branch-free (the counts are data: a branch per position mispredicts)
    // and in two passes the compiler vectorises: the fill of each position
    // (seed prefill 0 > 'N' -1 > '-' -2 > none), then the counted bases
    const int32_t n = std::min(length, rows);
    const int32_t ns = std::min(seed_len, length);
    std::memcpy(tok, seed, (size_t)std::max(ns, 0));
    for (int32_t i = ns; i < n; ++i) {
        const uint8_t nf = nflag[i] != 0, df = dflag[i] != 0;
        tok[i] = (uint8_t)(nf * 'N' + (1 - nf) * df * '-');
    }
    for (int32_t i = std::max(ns, n); i < length; ++i) tok[i] = 0;
    int positive = 0;
    {
        const int32_t *__restrict__ dd = dense;
        uint8_t *__restrict__ tt = tok;
        for (int32_t i = 0; i < n; ++i) {
            const int32_t c0 = dd[4 * i], c1 = dd[4 * i + 1], c2 = dd[4 * i + 2], c3 = dd[4 * i + 3];
            const int32_t top = std::max(std::max(c0, c1), std::max(c2, c3));
            // a positive count wins; ties go to the first of A < C < G < T
            // the first index holding top, as arithmetic (a compare chain
            // becomes branches that mispredict on count data)
            const uint32_t n0 = c0 != top, n1 = n0 & (c1 != top), n2 = n1 & (c2 != top);
            const uint32_t t = (uint32_t)(0x54474341u >> (8 * (n0 + n1 + n2))) & 0xffu;   // "ACGT"
            const uint32_t pos = top > 0;
            tt[i] = (uint8_t)((t & (0u - pos)) | (tt[i] & (pos - 1u)));
            positive |= (int)pos;
        }
    }
    for (int32_t i = n; i < rows && !positive; ++i) {
        const int32_t *d = dense + 4 * (size_t)i;
        positive = d[0] > 0 || d[1] > 0 || d[2] > 0 || d[3] > 0;
    }
    if (any_positive) *any_positive = positive;
    return 0;
}

// counts_to_conseqs (remap.py:309-333) for many references at once: per
// position the reference's Counter -- the seed's character at 0, the counted
// bases, 'N' := -1, '-' := -2, then every insertion token's pairs added --
// its top token (find_top_token, :892-902: the most pairs, ties to the
// smallest string), and the deletion-run rule of the assembly.
int mh_conseqs_build(int n_sel, const int32_t *rows_of, const int32_t *lengths, const char *const *seeds,
                     const int32_t *seed_lens, int32_t cap, const int32_t *dense, const uint8_t *nflag,
                     const uint8_t *dflag, int64_t n_ev, const int32_t *ev_row, const int32_t *ev_pos,
                     const int64_t *ev_off, const int32_t *ev_len, const int64_t *ev_cnt, const char *pool,
                     char *out, int64_t out_cap, int64_t *out_off, int32_t *present)
{
    if (n_sel < 0 || n_ev < 0 || cap < 0 || !out_off || !present ||
        (n_sel > 0 && (!rows_of || !lengths || !seeds || !seed_lens || !out)) ||
        (n_ev > 0 && (!ev_row || !ev_pos || !ev_off || !ev_len || !ev_cnt || !pool)) ||
        (cap > 0 && n_sel > 0 && (!dense || !nflag || !dflag))) {
        set_error("mh_conseqs_build: bad arguments");
        return -3;
    }
    for (int k = 0; k < n_sel; ++k)
        if (lengths[k] < 0 || seed_lens[k] < 0 || (seed_lens[k] > 0 && !seeds[k]) || rows_of[k] < 0) {
            set_error("mh_conseqs_build: bad reference %d", k);
            return -3;
        }
    // events grouped by (row, pos), tokens in order
    std::vector<int64_t> ev((size_t)n_ev);
    for (int64_t e = 0; e < n_ev; ++e) ev[(size_t)e] = e;
    std::sort(ev.begin(), ev.end(), [&](int64_t a, int64_t b) {
        if (ev_row[a] != ev_row[b]) return ev_row[a] < ev_row[b];
        return ev_pos[a] < ev_pos[b];
    });
    std::vector<std::string> texts((size_t)n_sel);

    // one reference: its consensus into texts[k], present[k]
    auto build_one = [&](int k, std::vector<uint8_t> &tok) {
        const int32_t row = rows_of[k], length = lengths[k], slen = seed_lens[k];
        const char *seed = slen > 0 ? seeds[k] : "";
        const int32_t rows = std::min(length, cap);
        const int32_t *d = dense + (size_t)row * cap * 4;
        const uint8_t *nf = nflag + (size_t)row * cap, *df = dflag + (size_t)row * cap;
        if (tok.size() < (size_t)std::max(length, 1)) tok.resize((size_t)std::max(length, 1));
        int32_t pos_any = 0;
        mh_top_tokens(length, rows, d, nf, df, seed, std::min(slen, length), tok.data(), &pos_any);
        auto lo = std::lower_bound(ev.begin(), ev.end(), row, [&](int64_t e, int32_t r) { return ev_row[e] < r; });
        auto hi = std::upper_bound(ev.begin(), ev.end(), row, [&](int32_t r, int64_t e) { return r < ev_row[e]; });
        present[k] = pos_any || lo != hi;
        // positions with events: the whole Counter (longer tokens kept aside)
        std::vector<std::pair<int32_t, std::string>> longer;   // (0-based position, token)
        for (auto it = lo; it != hi;) {
            const int32_t pos = ev_pos[*it];
            auto jt = it;
            while (jt != hi && ev_pos[*jt] == pos) ++jt;
            if (pos >= 1 && pos <= length) {
                std::vector<std::pair<std::string, int64_t>> c;   // insertion order irrelevant to the top
                auto add = [&](const std::string &t, int64_t v, bool assign) {
                    for (auto &x : c) if (x.first == t) { x.second = assign ? v : x.second + v; return; }
                    c.emplace_back(t, v);
                };
                const int32_t i = pos - 1;
                if (pos <= slen) add(std::string(1, seed[i]), 0, false);
                if (i < rows) {
                    static const char B[4] = {'A', 'C', 'G', 'T'};
                    for (int b = 0; b < 4; ++b) if (d[4 * (size_t)i + b]) add(std::string(1, B[b]), d[4 * (size_t)i + b], false);
                    if (nf[i]) add("N", -1, true);
                    if (df[i]) add("-", -2, true);
                }
                for (auto e = it; e != jt; ++e)
                    add(std::string(pool + ev_off[*e], (size_t)ev_len[*e]), ev_cnt[*e], false);
                const std::pair<std::string, int64_t> *top = nullptr;
                for (auto &x : c)
                    if (!top || x.second > top->second || (x.second == top->second && x.first < top->first)) top = &x;
                tok[(size_t)i] = top && !top->first.empty() ? (uint8_t)top->first[0] : 0;
                if (top && top->first.size() > 1) longer.emplace_back(i, top->first);
            }
            it = jt;
        }
        std::sort(longer.begin(), longer.end());
        if (!present[k]) return;
        // assembly: a missing token writes 'N' at once, a '-' opens or grows
        // the deletion, any other token first writes the open deletion when
        // its length is not a multiple of 3; a trailing deletion is dropped.
        // At most one byte per position plus the longer tokens' extra bytes.
        size_t need = (size_t)length;
        for (auto &x : longer) need += x.second.size() - 1;
        std::string &text = texts[(size_t)k];
        text.resize(need);
        char *o = &text[0], *o0 = o;
        const uint8_t *t = tok.data();
        size_t li = 0;
        int32_t dels = 0;
        for (int32_t i = 0; i < length;) {
            // a span of plain tokens (no 0, no '-', no longer token) is copied
            // as it is: the common case, one byte per position
            const int32_t stop = li < longer.size() ? longer[li].first : length;
            int32_t j = i;
            while (j < stop && t[j] != 0 && t[j] != '-') ++j;
            if (j > i) {
                if (dels) {
                    if (dels % 3 != 0) { std::memset(o, '-', (size_t)dels); o += dels; }
                    dels = 0;
                }
                std::memcpy(o, t + i, (size_t)(j - i));
                o += j - i;
                i = j;
                continue;
            }
            const uint8_t c = t[i];
            if (c == 0) { *o++ = 'N'; ++i; continue; }
            const bool is_longer = li < longer.size() && longer[li].first == i;
            if (c == '-' && !is_longer) { ++dels; ++i; continue; }
            if (dels) {
                if (dels % 3 != 0) { std::memset(o, '-', (size_t)dels); o += dels; }
                dels = 0;
            }
            const std::string &x = longer[li++].second;   // (is_longer here)
            std::memcpy(o, x.data(), x.size());
            o += x.size();
            ++i;
        }
        text.resize((size_t)(o - o0));
    };

    // one thread: ~3.5 ns per position (C4-all's ~0.7 M positions in ~2.5
    // ms); threads measured slower (their start-up and the texts' first
    // touch outweigh the work)
    {
        std::vector<uint8_t> tok;
        for (int k = 0; k < n_sel; ++k) build_one(k, tok);
    }
    int64_t at = 0;
    out_off[0] = 0;
    for (int k = 0; k < n_sel; ++k) {
        const std::string &text = texts[(size_t)k];
        if (at + (int64_t)text.size() > out_cap) { set_error("mh_conseqs_build: output capacity"); return -2; }
        std::memcpy(out + at, text.data(), text.size());
        at += (int64_t)text.size();
        out_off[k + 1] = at;
    }
    return 0;
}

int mh_levenshtein_batch(int count, const char *const *a, const char *const *b, int *out)
{
    if (count < 0 || (count > 0 && (!a || !b || !out))) return -3;
    for (int t = 0; t < count; ++t)
        if (!a[t] || !b[t]) return -3;
    // one pair per thread: the pairs of a consensus-distance filter are few and
    // long, so they are taken longest first (cost |a| * |b|) to balance the threads
    const int threads = count < 16 ? count : 16;
    std::vector<int> order((size_t)count);
    std::vector<double> cost((size_t)count);
    for (int t = 0; t < count; ++t) {
        order[(size_t)t] = t;
        cost[(size_t)t] = (double)std::strlen(a[t]) * (double)std::strlen(b[t]);
    }
    std::stable_sort(order.begin(), order.end(), [&](int x, int y) { return cost[(size_t)x] > cost[(size_t)y]; });
    std::vector<std::thread> pool;
    std::atomic<int> next(0);
    for (int w = 0; w < threads; ++w)
        pool.emplace_back([&]() {
            for (int i = next++; i < count; i = next++) {
                const int t = order[(size_t)i];
                out[t] = mh_levenshtein(a[t], b[t]);
            }
        });
    for (auto &th : pool) th.join();
    return 0;
}

// Unit-cost edit distance (python-Levenshtein's distance, remap.py:259) by
// the bit-vector recurrence of Myers / Hyyro: a's characters in 64-row
// blocks, one pass over b, ~15 word operations per block and column instead
// of one DP cell per (i, j).  a is padded to whole blocks with rows that match
// every character; their vertical deltas in the last column are taken back
// off the bottom-row score at the end, so the result is D[|a|][|b|] exactly.
int mh_levenshtein(const char *a, const char *b)
{
    if (!a || !b) return -3;
    const size_t m = std::strlen(a), n = std::strlen(b);
    if (m == 0) return (int)n;
    if (n == 0) return (int)m;
    const size_t nb = (m + 63) / 64;
    const size_t pad = nb * 64 - m;
    const uint64_t padmask = pad ? ~0ull << (64 - pad) : 0;   // padded rows of the last block
    // a's alphabet compacted: symbol s's match vectors are peq[s * nb ..], one
    // contiguous row per symbol; characters a does not hold map to the last
    // symbol, which matches only the padded rows
    uint8_t sym[256];
    int ns = 0;
    std::memset(sym, 0xff, sizeof(sym));
    for (size_t i = 0; i < m; ++i) {
        const unsigned char ch = (unsigned char)a[i];
        if (sym[ch] == 0xff) sym[ch] = (uint8_t)ns++;
    }
    const int none = ns++;
    for (int ch = 0; ch < 256; ++ch) if (sym[ch] == 0xff) sym[ch] = (uint8_t)none;
    std::vector<uint64_t> peq((size_t)ns * nb, 0);
    for (int s = 0; s < ns; ++s) peq[(size_t)s * nb + nb - 1] = padmask;
    for (size_t i = 0; i < m; ++i) peq[(size_t)sym[(unsigned char)a[i]] * nb + i / 64] |= 1ull << (i % 64);
    std::vector<uint64_t> P(nb, ~0ull), M(nb, 0);   // vertical deltas +1 / -1 (D[i][0] = i)
    uint64_t *Pp = P.data(), *Mp = M.data();
    long long score = (long long)(nb * 64);         // D[bottom row][0]
    for (size_t j = 0; j < n; ++j) {
        const uint64_t *eqc = &peq[(size_t)sym[(unsigned char)b[j]] * nb];
        // horizontal delta into the block's top row as two bits (+1: hp, -1: hn);
        // D[0][j+1] - D[0][j] = +1 (global)
        uint64_t hp = 1, hn = 0;
        for (size_t k = 0; k < nb; ++k) {
            const uint64_t Pv = Pp[k], Mv = Mp[k];
            const uint64_t Xv = eqc[k] | Mv;
            const uint64_t Eq = eqc[k] | hn;
            const uint64_t Xh = (((Eq & Pv) + Pv) ^ Pv) | Eq;
            uint64_t Ph = Mv | ~(Xh | Pv);
            uint64_t Mh = Pv & Xh;
            const uint64_t op = Ph >> 63, on = Mh >> 63;
            Ph = (Ph << 1) | hp;
            Mh = (Mh << 1) | hn;
            Pp[k] = Mh | ~(Xv | Ph);
            Mp[k] = Ph & Xv;
            hp = op;
            hn = on;
        }
        score += (long long)hp - (long long)hn;
    }
    // D[m][n] = D[bottom][n] - (deltas of the padded rows in the last column)
    score -= (long long)__builtin_popcountll(P[nb - 1] & padmask) -
             (long long)__builtin_popcountll(M[nb - 1] & padmask);
    return (int)score;
}

}  // extern "C"
