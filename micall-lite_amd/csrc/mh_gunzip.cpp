// mh_gunzip.cpp -- whole-buffer gunzip for the FASTQ ingest and the censor
// stage.  Decodes every concatenated member (as GzipFile and gzread do).
// libdeflate (libdeflate.so.0, loaded with dlopen: the image ships the
// library without its header) decodes ~3x faster than zlib's inflate and is
// used when present; zlib otherwise.  Host code only.
#include <dlfcn.h>
#include <zlib.h>

#include <algorithm>
#include <cstring>
#include <mutex>
#include <string>

#include "mh_gunzip.h"

namespace mh {

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

struct LdApi {
    ld_alloc_t alloc = nullptr;
    ld_free_t free_ = nullptr;
    ld_gunzip_ex_t gunzip = nullptr;
    lc_alloc_t c_alloc = nullptr;
    lc_free_t c_free = nullptr;
    lc_gzip_t c_gzip = nullptr;
    lc_bound_t c_bound = nullptr;
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
    });
    return api;
}

int gunzip_zlib(const uint8_t *src, int64_t len, std::string &out, std::string &why)
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

int gunzip_ld(const LdApi &api, const uint8_t *src, int64_t len, std::string &out, std::string &why)
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

}  // namespace

bool gunzip_fast_available() { return ld_api().ok; }

int gunzip_buffer(const uint8_t *src, int64_t len, std::string &out, std::string &why)
{
    out.clear();
    if (len <= 0) return 0;
    const LdApi &api = ld_api();
    return api.ok ? gunzip_ld(api, src, len, out, why) : gunzip_zlib(src, len, out, why);
}

int gzip_member(const char *src, size_t len, std::string &out, int level)
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

}  // namespace mh
