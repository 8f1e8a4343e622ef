// mh_gunzip.cpp -- whole-buffer gunzip for the FASTQ ingest and the censor
// stage.  Decodes every concatenated member (as GzipFile and gzread do).
// libdeflate (libdeflate.so.0, loaded with dlopen: the image ships the
// library without its header) decodes ~3x faster than zlib's inflate and is
// used when present; zlib otherwise.  Host code only.
#include <dlfcn.h>
#include <sys/mman.h>
#include <cerrno>
#include <sys/stat.h>
#include <zlib.h>

#include <algorithm>
#include <atomic>
#include <exception>
#include <cstring>
#include <functional>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "mh_gunzip.h"

namespace mh {

void set_error(const char *fmt, ...);   // mh_api.cpp
int gunzip_threads();

namespace {

// libdeflate's C API (libdeflate.h, v1.x), declared here
struct Ld;
enum { LD_SUCCESS = 0, LD_BAD_DATA = 1, LD_SHORT_OUTPUT = 2, LD_INSUFFICIENT_SPACE = 3 };
typedef Ld *(*ld_alloc_t)(void);
typedef void (*ld_free_t)(Ld *);
typedef int (*ld_gunzip_ex_t)(Ld *, const void *, size_t, void *, size_t, size_t *, size_t *);
struct Lc;
typedef Lc *(*lc_alloc_t)(int);
typedef void (*lc_free_t)(Lc *);
typedef size_t (*lc_gzip_t)(Lc *, const void *, size_t, void *, size_t);
typedef size_t (*lc_bound_t)(Lc *, size_t);
typedef uint32_t (*l_crc32_t)(uint32_t, const void *, size_t);
typedef int (*ld_raw_ex_t)(Ld *, const void *, size_t, void *, size_t, size_t *, size_t *);

struct LdApi {
    ld_alloc_t alloc = nullptr;
    ld_free_t free_ = nullptr;
    ld_gunzip_ex_t gunzip = nullptr;
    lc_alloc_t c_alloc = nullptr;
    lc_free_t c_free = nullptr;
    lc_gzip_t c_gzip = nullptr;
    lc_bound_t c_bound = nullptr;
    l_crc32_t crc32 = nullptr;
    ld_raw_ex_t raw = nullptr;
    bool ok = false, c_ok = false;
};

const LdApi &ld_api()
{
    static LdApi api;
    static std::once_flag once;
    std::call_once(once, [] {
        if (getenv("MICALL_NO_LIBDEFLATE")) return;
        void *h = dlopen("libdeflate.so.0", RTLD_NOW | RTLD_LOCAL);
        if (!h) return;
        api.alloc = (ld_alloc_t)dlsym(h, "libdeflate_alloc_decompressor");
        api.free_ = (ld_free_t)dlsym(h, "libdeflate_free_decompressor");
        api.gunzip = (ld_gunzip_ex_t)dlsym(h, "libdeflate_gzip_decompress_ex");
        api.ok = api.alloc && api.free_ && api.gunzip;
        api.c_alloc = (lc_alloc_t)dlsym(h, "libdeflate_alloc_compressor");
        api.c_free = (lc_free_t)dlsym(h, "libdeflate_free_compressor");
        api.c_gzip = (lc_gzip_t)dlsym(h, "libdeflate_gzip_compress");
        api.c_bound = (lc_bound_t)dlsym(h, "libdeflate_gzip_compress_bound");
        api.c_ok = api.c_alloc && api.c_free && api.c_gzip && api.c_bound;
        api.crc32 = (l_crc32_t)dlsym(h, "libdeflate_crc32");
        api.raw = (ld_raw_ex_t)dlsym(h, "libdeflate_deflate_decompress_ex");
    });
    return api;
}

template <class Buf>
int gunzip_zlib(const uint8_t *src, int64_t len, Buf &out, std::string &why)
{
    z_stream z{};
    if (inflateInit2(&z, 15 + 32) != Z_OK) { why = "zlib init"; return -3; }
    std::string buf(1u << 22, '\0');
    int64_t pos = 0;
    bool ended = false;
    for (;;) {
        if (z.avail_in == 0) {
            if (pos >= len) break;
            const int64_t take = std::min<int64_t>(len - pos, 1 << 30);
            z.next_in = (Bytef *)(src + pos);
            z.avail_in = (uInt)take;
            pos += take;
        }
        z.next_out = (Bytef *)&buf[0];
        z.avail_out = (uInt)buf.size();
        const int st = inflate(&z, Z_NO_FLUSH);
        out.append(buf.data(), buf.size() - z.avail_out);
        if (st == Z_STREAM_END) {
            ended = true;
            if (z.avail_in == 0 && pos >= len) break;
            inflateReset(&z);
            ended = false;
            continue;
        }
        if (st != Z_OK && !(st == Z_BUF_ERROR && z.avail_in == 0)) {
            inflateEnd(&z);
            why = "not a valid gzip stream";
            return -3;
        }
    }
    inflateEnd(&z);
    if (!ended) { why = "truncated gzip stream"; return -3; }
    return 0;
}

template <class Buf>
int gunzip_ld(const LdApi &api, const uint8_t *src, int64_t len, Buf &out, std::string &why)
{
    Ld *d = api.alloc();
    if (!d) { why = "libdeflate: out of memory"; return -2; }
    // the last member's ISIZE (size mod 2^32) sizes the first attempt
    size_t guess = len >= 18 ? (size_t)src[len - 4] | (size_t)src[len - 3] << 8 |
                                   (size_t)src[len - 2] << 16 | (size_t)src[len - 1] << 24
                             : 0;
    guess = std::max<size_t>(guess, (size_t)len * 3);
    int64_t pos = 0;
    int rc = 0;
    while (pos < len) {
        size_t cap = guess + 64;
        for (;;) {
            const size_t base = out.size();
            out.resize(base + cap);
            size_t in_used = 0, out_used = 0;
            const int r = api.gunzip(d, src + pos, (size_t)(len - pos), &out[base], cap, &in_used,
                                     &out_used);
            if (r == LD_SUCCESS) {
                out.resize(base + out_used);
                pos += (int64_t)in_used;
                break;
            }
            out.resize(base);
            if (r == LD_INSUFFICIENT_SPACE) { cap *= 2; continue; }
            why = r == LD_BAD_DATA ? "not a valid gzip stream" : "truncated gzip stream";
            rc = -3;
            break;
        }
        if (rc) break;
        guess = std::max<size_t>((size_t)(len - pos) * 4, 1u << 20);
    }
    api.free_(d);
    return rc;
}

// One whole member [src, src + len) into out[0 .. isize): true when it
// decodes, uses exactly len bytes and yields exactly isize bytes.
bool member_exact(const LdApi &api, const uint8_t *src, int64_t len, char *out, uint32_t isize)
{
    if (api.ok) {
        Ld *d = api.alloc();
        if (!d) return false;
        size_t in_used = 0, out_used = 0;
        const int r = api.gunzip(d, src, (size_t)len, out, isize, &in_used, &out_used);
        api.free_(d);
        return r == LD_SUCCESS && (int64_t)in_used == len && out_used == isize;
    }
    z_stream z{};
    if (inflateInit2(&z, 15 + 16) != Z_OK) return false;
    z.next_in = (Bytef *)src;
    z.avail_in = (uInt)len;
    z.next_out = (Bytef *)out;
    z.avail_out = isize;
    const int st = inflate(&z, Z_FINISH);
    const bool ok = st == Z_STREAM_END && z.avail_in == 0 && z.avail_out == 0;
    inflateEnd(&z);
    return ok;
}

// A gzip member header at p: magic, deflate, no reserved flag bits, a known
// XFL and OS byte (RFC 1952).  Inside compressed data this pattern is rare;
// a false candidate is caught by member_exact.
bool member_header(const uint8_t *p, int64_t avail)
{
    return avail >= 18 && p[0] == 0x1f && p[1] == 0x8b && p[2] == 8 && (p[3] & 0xe0) == 0 &&
           (p[8] == 0 || p[8] == 2 || p[8] == 4) && (p[9] <= 13 || p[9] == 255);
}

uint32_t le32(const uint8_t *p) { return p[0] | p[1] << 8 | p[2] << 16 | (uint32_t)p[3] << 24; }

void run_threads(int nt, const std::function<void(int)> &fn)
{
    if (nt <= 1) { fn(0); return; }
    std::vector<std::thread> th;
    for (int t = 1; t < nt; ++t) th.emplace_back(fn, t);
    fn(0);
    for (auto &x : th) x.join();
}

// Concatenated members decoded in parallel.  Every header-shaped offset is a
// candidate member start; the member ending at the next candidate has its
// size (ISIZE) in the 4 bytes before it.  Each candidate span is decoded
// straight into its place in `out` and accepted only when it is exactly one
// whole member of exactly that size.  Spans that fail (a false candidate
// split a member) are merged with the next span(s) and decoded again;
// -1 when that does not resolve them (the caller then decodes serially).
template <class Buf>
int gunzip_members(const LdApi &api, const uint8_t *src, int64_t len, Buf &out, int threads)
{
    std::vector<int64_t> cand;
    {
        const int nt = threads;
        std::vector<std::vector<int64_t>> part(nt);
        run_threads(nt, [&](int t) {
            const int64_t a = len * t / nt, b = len * (t + 1) / nt;
            const uint8_t *p = src + a;
            while (p < src + b) {
                p = (const uint8_t *)memchr(p, 0x1f, (size_t)(src + b - p));
                if (!p) break;
                if (member_header(p, src + len - p)) part[t].push_back(p - src);
                ++p;
            }
        });
        for (auto &v : part) cand.insert(cand.end(), v.begin(), v.end());
    }
    if (cand.empty() || cand[0] != 0) return -1;
    {
        // header-shaped bytes inside compressed data are common (a few per
        // 16 MB): a candidate after the first must also start decoding (its
        // first 16 KB of output), else it is dropped here instead of splitting
        // a member into spans that fail to decode.  A single member (as
        // bcl2fastq writes it) is left with one candidate and decoded serially
        // by the caller.
        std::vector<char> keep(cand.size(), 1);
        std::atomic<size_t> next(1);
        run_threads(std::min<int>(threads, (int)cand.size()), [&](int) {
            for (size_t j; (j = next.fetch_add(1)) < cand.size();)
                keep[j] = gzip_member_probe(src + cand[j], len - cand[j], 16384);
        });
        size_t w = 0;
        for (size_t j = 0; j < cand.size(); ++j)
            if (keep[j]) cand[w++] = cand[j];
        cand.resize(w);
        if (cand.size() < 2) return -2;   // one member
    }
    cand.push_back(len);
    // spans [cand[j], cand[j + 1]) and their sizes, merging spans whose
    // decode failed until every span is one whole member
    std::vector<int64_t> beg(cand.begin(), cand.end() - 1), end(cand.begin() + 1, cand.end());
    for (int round = 0; round < 8; ++round) {
        const size_t k = beg.size();
        // a span's size is the ISIZE word before its end; deflate expands at
        // most 1032:1, so a larger word comes from a false boundary: the span
        // is not decoded (size 0) and fails, which merges it with the next
        std::vector<uint64_t> at(k + 1, 0);
        std::vector<char> plausible(k, 1);
        for (size_t j = 0; j < k; ++j) {
            const int64_t span = end[j] - beg[j];
            if (span < 18) return -1;
            const uint64_t isize = le32(src + end[j] - 4);
            plausible[j] = isize <= (uint64_t)span * 1032 + 64;
            at[j + 1] = at[j] + (plausible[j] ? isize : 0);
        }
        if (at[k] > (uint64_t)len * 1032 + (1u << 20)) return -1;
        out.resize(at[k]);
        std::vector<char> ok(k, 0);
        std::atomic<size_t> next(0);
        run_threads(std::min<int>(threads, (int)k), [&](int) {
            for (size_t j; (j = next.fetch_add(1)) < k;)
                ok[j] = plausible[j] &&
                        member_exact(api, src + beg[j], end[j] - beg[j], &out[at[j]],
                                     (uint32_t)(at[j + 1] - at[j]));
        });
        // a failed span absorbs the span after it (a false candidate split
        // one member in two)
        std::vector<int64_t> nb, ne;
        bool all = true, pending = false;
        for (size_t j = 0; j < k; ++j) {
            if (pending) { ne.back() = end[j]; pending = false; continue; }
            nb.push_back(beg[j]);
            ne.push_back(end[j]);
            if (!ok[j]) { all = false; pending = true; }
        }
        if (all) return 0;
        if (pending) return -1;   // the last span failed: nothing follows it
        beg.swap(nb);
        end.swap(ne);
    }
    return -1;
}

}  // namespace

void *ld_raw_alloc()
{
    const LdApi &api = ld_api();
    return api.ok && api.raw ? (void *)api.alloc() : nullptr;
}

void ld_raw_free(void *d)
{
    if (d) ld_api().free_((Ld *)d);
}

int ld_raw_inflate(void *d, const uint8_t *in, size_t n, char *out, size_t cap, size_t *in_used,
                   size_t *out_used)
{
    return ld_api().raw((Ld *)d, in, n, out, cap, in_used, out_used);
}

constexpr size_t BIG = (size_t)4 << 20;

char *big_alloc(size_t n)
{
    if (n < BIG) return new char[n > 0 ? n : 1];
    void *p = mmap(nullptr, n, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS, -1, 0);
    if (p == MAP_FAILED) throw std::bad_alloc();
    // MICALL_NO_THP=1: 4 KiB pages (for A/B timing)
    static const bool thp = !(getenv("MICALL_NO_THP") && *getenv("MICALL_NO_THP") == '1');
    if (thp) madvise(p, n, MADV_HUGEPAGE);
    return (char *)p;
}

void big_free(char *p, size_t n)
{
    if (!p) return;
    if (n < BIG) { delete[] p; return; }
    // The pages are given back by MADV_DONTNEED in 8 MiB pieces first, and
    // the emptied mapping is unmapped after.  A GB-sized munmap on a detached
    // thread holds the process's mmap lock for writing for tens of ms, and
    // every thread creation meanwhile (its stack is an mmap) waits for it.
    // MICALL_PLAIN_MUNMAP=1: one munmap (for A/B timing).
    static const bool plain = getenv("MICALL_PLAIN_MUNMAP") && *getenv("MICALL_PLAIN_MUNMAP") == '1';
    if (!plain && n >= ((size_t)64 << 20)) {
        const size_t piece = (size_t)8 << 20;
        for (size_t at = 0; at < n; at += piece) madvise(p + at, std::min(piece, n - at), MADV_DONTNEED);
    }
    munmap(p, n);
}

bool gunzip_fast_available() { return ld_api().ok; }

int map_text_file(int fd, const char **text, size_t *len)
{
    *text = nullptr;
    *len = 0;
    struct stat st;
    if (fd < 0 || fstat(fd, &st) != 0 || !S_ISREG(st.st_mode)) {
        set_error("map_text_file: not a regular file");
        return -3;
    }
    const size_t n = (size_t)st.st_size;
    if (n == 0) return 0;
    void *m = mmap(nullptr, n, PROT_READ, MAP_PRIVATE, fd, 0);
    if (m == MAP_FAILED) { set_error("map_text_file: mmap failed (%s)", strerror(errno)); return -3; }
    const char *t = (const char *)m;
    const int nt = std::max(1, std::min<int>(gunzip_threads(), (int)(n >> 20) + 1));
    std::vector<char> cr((size_t)nt, 0);
    run_threads(nt, [&](int k) {
        const size_t a = n * (size_t)k / (size_t)nt, b = n * (size_t)(k + 1) / (size_t)nt;
        cr[(size_t)k] = memchr(t + a, '\r', b - a) != nullptr;
    });
    for (char c : cr)
        if (c) { munmap(m, n); return 1; }
    *text = t;
    *len = n;
    return 0;
}

void unmap_text_file(const char *text, size_t len)
{
    if (text && len) munmap((void *)text, len);
}

uint32_t crc32_update(uint32_t crc, const void *p, size_t n)
{
    const LdApi &api = ld_api();
    if (api.crc32) return api.crc32(crc, p, n);
    const Bytef *b = (const Bytef *)p;
    uLong c = crc;
    while (n > 0) {
        const uInt take = (uInt)std::min<size_t>(n, 1u << 30);
        c = ::crc32(c, b, take);
        b += take;
        n -= take;
    }
    return (uint32_t)c;
}

namespace {
// GF(2) product of two polynomials mod the CRC-32 polynomial, bit-reflected
// (bit 31 is x^0)
uint32_t crc_mulmod(uint32_t a, uint32_t b)
{
    uint32_t m = 1u << 31, p = 0;
    for (;;) {
        if (a & m) {
            p ^= b;
            if ((a & (m - 1)) == 0) break;
        }
        m >>= 1;
        b = (b & 1) ? (b >> 1) ^ 0xedb88320u : b >> 1;
    }
    return p;
}

// x^(2^k) mod P for k = 0 .. 63
struct CrcPow {
    uint32_t x2k[64];
    CrcPow()
    {
        x2k[0] = 1u << 30;   // x^1
        for (int k = 1; k < 64; ++k) x2k[k] = crc_mulmod(x2k[k - 1], x2k[k - 1]);
    }
};
}  // namespace

// crc(A ++ B) = crc(A) * x^(8 |B|) mod P  xor  crc(B): the shift by |B| bytes
// as a product of the precomputed x^(2^k) (about 20 products for 1 MB; the
// zlib of this image squares a 32x32 bit matrix per bit of the length)
uint32_t crc32_join(uint32_t a, uint32_t b, int64_t len_b)
{
    static const CrcPow pw;
    if (len_b <= 0) return a ^ b;   // B empty: crc(B) = 0
    uint32_t x = 1u << 31;   // x^0
    uint64_t n = (uint64_t)len_b;
    for (int k = 3; n; n >>= 1, ++k)   // 8 |B| bits: start at 2^3
        if (n & 1) x = crc_mulmod(pw.x2k[k & 63], x);
    return crc_mulmod(x, a) ^ b;
}

bool gzip_header_at(const uint8_t *src, int64_t avail) { return member_header(src, avail); }

bool gzip_member_probe(const uint8_t *src, int64_t len, size_t probe)
{
    if (!member_header(src, len)) return false;
    std::string out(probe, '\0');
    const LdApi &api = ld_api();
    if (api.ok) {
        Ld *d = api.alloc();
        if (!d) return false;
        size_t in_used = 0, out_used = 0;
        const int r = api.gunzip(d, src, (size_t)len, &out[0], probe, &in_used, &out_used);
        api.free_(d);
        // a member longer than the probe stops with the output full
        return r == LD_SUCCESS || r == LD_INSUFFICIENT_SPACE;
    }
    z_stream z{};
    if (inflateInit2(&z, 15 + 16) != Z_OK) return false;
    z.next_in = (Bytef *)src;
    z.avail_in = (uInt)std::min<int64_t>(len, 1 << 30);
    z.next_out = (Bytef *)&out[0];
    z.avail_out = (uInt)probe;
    const int st = inflate(&z, Z_NO_FLUSH);
    const bool ok = st == Z_STREAM_END || (st == Z_OK && z.avail_out == 0);
    inflateEnd(&z);
    return ok;
}

static bool getenv_flag(const char *name)
{
    const char *e = getenv(name);
    return e && *e == '1';
}

int gunzip_threads()
{
    const char *e = getenv("OMP_NUM_THREADS");
    int n = e ? atoi(e) : 0;
    if (n <= 0) n = (int)std::thread::hardware_concurrency();
    return std::max(1, std::min(n, 64));
}

template <class Buf>
int gunzip_any(const uint8_t *src, int64_t len, Buf &out, std::string &why)
{
    out.clear();
    if (len <= 0) return 0;
    const LdApi &api = ld_api();
    // concatenated members (as a parallel gzip writes them) decode in
    // parallel; a single member, or anything the member scan cannot split,
    // decodes serially
    if (len > (1 << 22)) {
        int st = -1;
        try {
            st = gunzip_members(api, src, len, out, gunzip_threads());
            // one member: its deflate blocks found and inflated in parallel
            if (st == -2 && !getenv_flag("MICALL_SERIAL_INFLATE")) {
                Buf().swap(out);
                st = gunzip_single_parallel(src, len, out, gunzip_threads());
            }
        } catch (const std::exception &) {   // bad_alloc / length_error: decode serially
            st = -1;
        }
        if (st == 0) return 0;
        Buf().swap(out);
    }
    try {
        return api.ok ? gunzip_ld(api, src, len, out, why) : gunzip_zlib(src, len, out, why);
    } catch (const std::exception &) {
        Buf().swap(out);
        why = "out of memory";
        return -2;
    }
}

int gunzip_buffer(const uint8_t *src, int64_t len, std::string &out, std::string &why)
{
    return gunzip_any(src, len, out, why);
}

int gunzip_buffer(const uint8_t *src, int64_t len, TextBuf &out, std::string &why)
{
    return gunzip_any(src, len, out, why);
}

template <class Buf>
static int gzip_member_any(const char *src, size_t len, Buf &out, int level)
{
    const LdApi &api = ld_api();
    if (api.c_ok) {
        Lc *c = api.c_alloc(level);
        if (c) {
            out.resize(api.c_bound(c, len) + 64);
            const size_t n = api.c_gzip(c, src, len, &out[0], out.size());
            api.c_free(c);
            if (n) { out.resize(n); return 0; }
        }
    }
    z_stream z{};
    if (deflateInit2(&z, level, Z_DEFLATED, 15 + 16, 8, Z_DEFAULT_STRATEGY) != Z_OK) return -2;
    out.resize(deflateBound(&z, (uLong)len) + 64);
    z.next_in = (Bytef *)src;
    z.avail_in = (uInt)len;
    z.next_out = (Bytef *)&out[0];
    z.avail_out = (uInt)out.size();
    const int st = deflate(&z, Z_FINISH);
    out.resize(out.size() - z.avail_out);
    deflateEnd(&z);
    return st == Z_STREAM_END ? 0 : -2;
}

int gzip_member(const char *src, size_t len, std::string &out, int level)
{
    return gzip_member_any(src, len, out, level);
}

int gzip_member(const char *src, size_t len, TextBuf &out, int level)
{
    return gzip_member_any(src, len, out, level);
}

}  // namespace mh
