// mh_pinflate.cpp -- one gzip member inflated by many host threads.
//
// A FASTQ as bcl2fastq writes it is one gzip member: a plain inflate is one
// thread (≈ 0.75 GB/s of text on the GPU box; 0.75 s for a C2 R1 file, most
// of censor's time).  Deflate blocks can be found without decoding what
// comes before them, so the member is cut into one span per thread:
//
//   1. search: each span's first dynamic-Huffman block start at or after
//      its byte offset -- every bit position whose header (RFC 1951 3.2.7)
//      parses into complete code-length and literal/length codes with an
//      end-of-block code, then confirmed by decoding two blocks;
//   2. decode: every span inflated (zlib, raw) from its start to the next
//      span's start with a dictionary of 32 KiB of zero bytes in place of
//      the unknown window: the bytes copied out of that window come out as
//      NUL, which FASTQ text never holds, so everything past a span's last
//      NUL is exact; a span must end exactly on the next one's start (else
//      the start was false and the caller decodes serially);
//   3. resolve: each span's bytes up to its last NUL decoded twice more,
//      with windows whose bytes spell each window offset in base 255, so
//      every window-derived byte knows which window byte it copies; they are
//      replaced from the true window (the 32 KiB before the span) -- the last
//      32 KiB of every span in order, as each is the next span's window, then
//      everything else at once.  (Back-references keep window bytes alive
//      through most of a span of FASTQ: re-decoding the dirty part in order
//      with the true window would be nearly serial.)
//   4. check: the whole output's CRC-32 and size against the gzip trailer.
//
// Any failure returns -1 and the caller inflates serially, so the result is
// the plain inflate's or none.  Host code only.
#include <zlib.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <atomic>
#include <cstring>
#include <functional>
#include <thread>
#include <vector>

#include "mh_gunzip.h"

namespace mh {

namespace {

constexpr int WIN = 32768;

// up to 57 bits at bit position pos (LSB first), zero past the end
inline uint64_t peek_bits(const uint8_t *p, int64_t nbytes, int64_t pos)
{
    const int64_t b = pos >> 3;
    uint64_t v = 0;
    if (b + 8 <= nbytes) {
        memcpy(&v, p + b, 8);
    } else {
        for (int64_t i = b; i < nbytes; ++i) v |= (uint64_t)p[i] << (8 * (i - b));
    }
    return v >> (pos & 7);
}

// lengths[0 .. n) form a code zlib accepts: complete, or (litlen / dist) a
// single code of length 1; all-zero only where allowed
bool code_ok(const uint8_t *len, int n, int maxbits, bool allow_empty)
{
    int count[16] = {0};
    int used = 0, mx = 0;
    for (int i = 0; i < n; ++i)
        if (len[i]) { ++count[len[i]]; ++used; mx = std::max(mx, (int)len[i]); }
    if (used == 0) return allow_empty;
    int left = 1;
    for (int l = 1; l <= maxbits; ++l) {
        left <<= 1;
        left -= count[l];
        if (left < 0) return false;          // over-subscribed
    }
    return left == 0 || mx == 1;
}

// A dynamic-Huffman, non-final block header at bit position pos that zlib
// would accept (complete codes, an end-of-block code); *hdr_end = bits.
bool dyn_header_ok(const uint8_t *p, int64_t nbytes, int64_t pos)
{
    if ((pos >> 3) + 4 > nbytes) return false;
    uint64_t v = peek_bits(p, nbytes, pos);
    if ((v & 7) != 4) return false;           // BFINAL 0, BTYPE 10
    const int hlit = (int)((v >> 3) & 31) + 257, hdist = (int)((v >> 8) & 31) + 1;
    const int hclen = (int)((v >> 13) & 15) + 4;
    if (hlit > 286 || hdist > 30) return false;
    static const int ord[19] = {16, 17, 18, 0, 8, 7, 9, 6, 10, 5, 11, 4, 12, 3, 13, 2, 14, 1, 15};
    pos += 17;
    uint8_t cl[19] = {0};
    v = peek_bits(p, nbytes, pos);
    for (int i = 0; i < hclen; ++i) cl[ord[i]] = (uint8_t)((v >> (3 * i)) & 7);
    pos += 3 * hclen;
    if (!code_ok(cl, 19, 7, false)) return false;
    // canonical decoding of the code-length code, bit by bit (<= 7 bits)
    int count[8] = {0}, first_code[8] = {0}, first_sym[8] = {0};
    uint8_t sorted[19];
    for (int i = 0; i < 19; ++i) ++count[cl[i]];
    count[0] = 0;
    {
        int code = 0, k = 0;
        for (int l = 1; l <= 7; ++l) {
            code = (code + count[l - 1]) << 1;
            first_code[l] = code;
            first_sym[l] = k;
            for (int s = 0; s < 19; ++s) if (cl[s] == l) sorted[k++] = (uint8_t)s;
        }
    }
    uint8_t lens[286 + 30];
    const int total = hlit + hdist;
    int n = 0;
    while (n < total) {
        if ((pos >> 3) + 8 > nbytes) return false;
        v = peek_bits(p, nbytes, pos);
        int code = 0, sym = -1;
        for (int l = 1; l <= 7; ++l) {
            code |= (int)((v >> (l - 1)) & 1);
            const int idx = code - first_code[l];
            if (count[l] && idx >= 0 && idx < count[l]) { sym = sorted[first_sym[l] + idx]; pos += l; break; }
            code <<= 1;
        }
        if (sym < 0) return false;
        v = peek_bits(p, nbytes, pos);
        if (sym < 16) {
            lens[n++] = (uint8_t)sym;
        } else if (sym == 16) {
            if (n == 0) return false;
            const int r = 3 + (int)(v & 3);
            pos += 2;
            if (n + r > total) return false;
            for (int i = 0; i < r; ++i, ++n) lens[n] = lens[n - 1];
        } else {
            const int r = sym == 17 ? 3 + (int)(v & 7) : 11 + (int)(v & 127);
            pos += sym == 17 ? 3 : 7;
            if (n + r > total) return false;
            for (int i = 0; i < r; ++i) lens[n++] = 0;
        }
    }
    if (lens[256] == 0) return false;         // no end-of-block code
    return code_ok(lens, hlit, 15, false) && code_ok(lens + hlit, hdist, 15, true);
}

struct Span {
    z_stream z{};
    bool open = false;
    ~Span() { if (open) inflateEnd(&z); }
    // raw inflate positioned at bit `bit` of p with dictionary dict[0 .. dlen)
    bool start(const uint8_t *p, int64_t nbytes, int64_t bit, const uint8_t *dict, int dlen)
    {
        if (inflateInit2(&z, -15) != Z_OK) return false;
        open = true;
        if (dlen && inflateSetDictionary(&z, dict, (uInt)dlen) != Z_OK) return false;
        const int64_t b = bit >> 3;
        const int r = (int)(bit & 7);
        if (b >= nbytes) return false;
        if (r && inflatePrime(&z, 8 - r, p[b] >> r) != Z_OK) return false;
        base = p;
        z.next_in = (Bytef *)(p + b + (r ? 1 : 0));
        const int64_t avail = nbytes - (b + (r ? 1 : 0));
        z.avail_in = (uInt)std::min<int64_t>(avail, (int64_t)1 << 30);
        in_end = p + nbytes;
        return true;
    }
    // bits consumed so far (valid at a block boundary)
    int64_t bitpos() const { return (int64_t)((const uint8_t *)z.next_in - base) * 8 - (z.data_type & 7); }
    void refill()
    {
        if (z.avail_in == 0 && (const uint8_t *)z.next_in < in_end)
            z.avail_in = (uInt)std::min<int64_t>(in_end - (const uint8_t *)z.next_in, (int64_t)1 << 30);
    }
    const uint8_t *base = nullptr, *in_end = nullptr;
};

// Inflate from `bit` until the stream reaches stop_bit at a block boundary
// (stop_bit < 0: to the end of the deflate stream, *end_bit = the bit after
// it) into out (grown as needed).  0, or -1 (error, or stop_bit passed).
int inflate_to(const uint8_t *p, int64_t nbytes, int64_t bit, const uint8_t *dict, int dlen,
               int64_t stop_bit, TextBuf &out, int64_t *end_bit, int64_t max_blocks = -1)
{
    Span s;
    if (!s.start(p, nbytes, bit, dict, dlen)) return -1;
    size_t used = 0;
    int64_t blocks = 0;
    for (;;) {
        if (out.size() - used < (1u << 16)) out.resize(std::max<size_t>(out.size() * 2, used + (1u << 20)));
        s.refill();
        s.z.next_out = (Bytef *)out.data() + used;
        s.z.avail_out = (uInt)std::min<size_t>(out.size() - used, (size_t)1 << 30);
        const uInt before = s.z.avail_out;
        const int st = inflate(&s.z, Z_BLOCK);
        used += before - s.z.avail_out;
        if (st == Z_STREAM_END) {
            out.resize(used);
            if (stop_bit >= 0) return -1;
            *end_bit = s.bitpos();
            return 0;
        }
        if (st != Z_OK && st != Z_BUF_ERROR) return -1;
        if (st == Z_BUF_ERROR && s.z.avail_in == 0 && (const uint8_t *)s.z.next_in >= s.in_end) return -1;
        if (s.z.data_type & 128) {            // at a block boundary
            const int64_t at = s.bitpos();
            if (stop_bit >= 0 && at == stop_bit) { out.resize(used); *end_bit = at; return 0; }
            if (stop_bit >= 0 && at > stop_bit) return -1;
            if (max_blocks >= 0 && ++blocks >= max_blocks) { out.resize(used); *end_bit = at; return 0; }
        }
    }
}

// Exactly n output bytes from `bit` with dictionary dict into dst.
bool inflate_prefix(const uint8_t *p, int64_t nbytes, int64_t bit, const uint8_t *dict, int dlen,
                    char *dst, size_t n)
{
    Span s;
    if (!s.start(p, nbytes, bit, dict, dlen)) return false;
    size_t used = 0;
    while (used < n) {
        s.refill();
        s.z.next_out = (Bytef *)dst + used;
        s.z.avail_out = (uInt)std::min<size_t>(n - used, (size_t)1 << 30);
        const uInt before = s.z.avail_out;
        const int st = inflate(&s.z, Z_NO_FLUSH);
        used += before - s.z.avail_out;
        if (used >= n) break;
        if (st != Z_OK) return false;         // the stream ended or broke short of n
    }
    return true;
}

void threads_run(int nt, const std::function<void(int)> &fn)
{
    if (nt <= 1) { fn(0); return; }
    std::vector<std::thread> th;
    for (int t = 1; t < nt; ++t) th.emplace_back(fn, t);
    fn(0);
    for (auto &x : th) x.join();
}

inline uint32_t rd32(const uint8_t *p) { return p[0] | p[1] << 8 | p[2] << 16 | (uint32_t)p[3] << 24; }

// end of the gzip header at src (RFC 1952), or -1
int64_t gzip_header_end(const uint8_t *src, int64_t len)
{
    if (len < 18 || src[0] != 0x1f || src[1] != 0x8b || src[2] != 8) return -1;
    const int flg = src[3];
    int64_t at = 10;
    if (flg & 4) {                            // FEXTRA
        if (at + 2 > len) return -1;
        at += 2 + (src[at] | src[at + 1] << 8);
    }
    for (int bit : {8, 16}) {                 // FNAME, FCOMMENT
        if (flg & bit) {
            while (at < len && src[at]) ++at;
            ++at;
        }
    }
    if (flg & 2) at += 2;                     // FHCRC
    return at < len - 8 ? at : -1;
}

}  // namespace

template <class Buf>
int gunzip_single_parallel(const uint8_t *src, int64_t len, Buf &out, int threads)
{
    // MH_PINFLATE_TRACE=1: phase times to stderr
    static const bool trace = getenv("MH_PINFLATE_TRACE") && *getenv("MH_PINFLATE_TRACE") == '1';
    const auto t0 = std::chrono::steady_clock::now();
    auto mark = [&](const char *what) {
        if (trace)
            fprintf(stderr, "pinflate %s %.1f ms\n", what,
                    std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count());
    };
    const int64_t d0 = gzip_header_end(src, len);
    if (d0 < 0) return -1;
    const int64_t dend = len - 8;             // the deflate stream ends before the trailer
    const uint32_t crc_want = rd32(src + len - 8), isize = rd32(src + len - 4);
    const int64_t span_min = (int64_t)4 << 20;
    const int T = (int)std::min<int64_t>(threads, (dend - d0) / span_min);
    if (T < 2) return -1;
    // 1. span starts
    std::vector<int64_t> found((size_t)T, -1);
    found[0] = d0 * 8;
    std::vector<uint8_t> zeros(WIN, 0);
    threads_run(T - 1, [&](int i) {
        const int t = i + 1;
        const int64_t a = d0 + (dend - d0) * t / T, b = d0 + (dend - d0) * (t + 1) / T;
        TextBuf probe;
        for (int64_t bit = a * 8; bit < b * 8; ++bit) {
            if (!dyn_header_ok(src, dend, bit)) continue;
            int64_t e = 0;
            probe.clear();
            if (inflate_to(src, dend, bit, zeros.data(), WIN, -1, probe, &e, 2) == 0) {
                found[(size_t)t] = bit;
                return;
            }
        }
    });
    std::vector<int64_t> st;
    for (int64_t f : found) if (f >= 0) st.push_back(f);
    const int K = (int)st.size();
    mark("search");
    if (K < 2) return -1;
    // 2. every span with a window of zeros
    std::vector<TextBuf> part((size_t)K);
    std::vector<int64_t> end((size_t)K, -1);
    std::atomic<int> bad(0);
    threads_run(K, [&](int k) {
        part[(size_t)k].resize((size_t)std::max<int64_t>(1 << 20, ((k + 1 < K ? st[k + 1] : dend * 8) - st[k]) / 2));
        if (inflate_to(src, dend, st[k], k ? zeros.data() : nullptr, k ? WIN : 0, k + 1 < K ? st[k + 1] : -1,
                       part[(size_t)k], &end[(size_t)k]))
            bad = 1;
    });
    mark("decode");
    if (bad || (end[(size_t)K - 1] + 7) / 8 != dend) return -1;
    std::vector<size_t> off((size_t)K + 1, 0), dirty((size_t)K, 0);
    for (int k = 0; k < K; ++k) {
        off[(size_t)k + 1] = off[(size_t)k] + part[(size_t)k].size();
        if (k) {
            const char *b = part[(size_t)k].data();
            const void *z = memrchr(b, 0, part[(size_t)k].size());
            dirty[(size_t)k] = z ? (size_t)((const char *)z - b) + 1 : 0;
        }
    }
    if ((uint32_t)off[(size_t)K] != isize) return -1;
    out.resize(off[(size_t)K]);
    char *o = &out[0];
    threads_run(std::min(K, threads), [&](int t) {
        for (int k = t; k < K; k += std::min(K, threads)) {
            memcpy(o + off[(size_t)k], part[(size_t)k].data(), part[(size_t)k].size());
            part[(size_t)k].release();
        }
    });
    mark("place");
    // 3. the dirty bytes' window offsets: each span's dirty prefix decoded
    // twice more with windows whose bytes spell the offset (lo: i % 255 + 1,
    // hi: i / 255 + 1; never 0, so a byte that is NUL in all three decodes is
    // a NUL of the data), then every dirty byte replaced by the window byte
    // it copies -- first the last 32 KiB of every span in order (they are
    // the next span's window), then the rest of every span at once
    std::vector<TextBuf> lo((size_t)K), hi((size_t)K);
    std::vector<int> win((size_t)K, 0);
    std::vector<uint8_t> wlo(WIN), whi(WIN);
    for (int k = 1; k < K; ++k) win[(size_t)k] = (int)std::min<size_t>(WIN, off[(size_t)k]);
    {
        std::vector<std::pair<int, int>> jobs;   // (span, 0 lo / 1 hi)
        for (int k = 1; k < K; ++k)
            if (dirty[(size_t)k]) { jobs.emplace_back(k, 0); jobs.emplace_back(k, 1); }
        std::atomic<size_t> next(0);
        threads_run(std::min<int>((int)jobs.size(), threads), [&](int) {
            std::vector<uint8_t> dict(WIN);
            for (size_t j; (j = next.fetch_add(1)) < jobs.size();) {
                const int k = jobs[j].first, w = win[(size_t)k];
                for (int i = 0; i < w; ++i) dict[(size_t)i] = (uint8_t)(jobs[j].second ? i / 255 + 1 : i % 255 + 1);
                TextBuf &dst = jobs[j].second ? hi[(size_t)k] : lo[(size_t)k];
                dst.resize(dirty[(size_t)k]);
                if (!inflate_prefix(src, dend, st[k], dict.data(), w, dst.data(), dirty[(size_t)k])) bad = 1;
            }
        });
    }
    if (bad) return -1;
    auto resolve = [&](int k, size_t i0, size_t i1) {
        char *span = o + off[(size_t)k];
        const char *wb = o + off[(size_t)k] - win[(size_t)k];
        const uint8_t *L = (const uint8_t *)lo[(size_t)k].data(), *H = (const uint8_t *)hi[(size_t)k].data();
        for (size_t i = i0; i < i1; ++i) {
            if (span[i] != 0 || L[i] == 0) continue;      // exact, or a NUL of the data
            const int idx = (H[i] - 1) * 255 + (L[i] - 1);
            if (idx >= win[(size_t)k]) { bad = 1; return; }
            span[i] = wb[idx];
        }
    };
    for (int k = 1; k < K; ++k) {   // the tails, in order
        const size_t n = off[(size_t)k + 1] - off[(size_t)k];
        const size_t t0 = n > (size_t)WIN ? n - WIN : 0;
        if (dirty[(size_t)k] > t0) resolve(k, t0, dirty[(size_t)k]);
    }
    {
        std::atomic<int> next(1);
        threads_run(std::min(K, threads), [&](int) {
            for (int k; (k = next.fetch_add(1)) < K;) {
                const size_t n = off[(size_t)k + 1] - off[(size_t)k];
                const size_t t0 = n > (size_t)WIN ? n - WIN : 0;
                resolve(k, 0, std::min(dirty[(size_t)k], t0));
                lo[(size_t)k].release();
                hi[(size_t)k].release();
            }
        });
    }
    mark("fix");
    if (trace) {
        size_t d = 0;
        for (size_t x : dirty) d += x;
        fprintf(stderr, "pinflate spans %d dirty bytes %zu\n", K, d);
    }
    if (bad) return -1;
    // 4. CRC-32 of the whole output, in parallel pieces
    const size_t total = off[(size_t)K];
    const int P = std::max(1, std::min<int>(threads, (int)(total >> 22) + 1));
    std::vector<uint32_t> crc((size_t)P, 0);
    threads_run(P, [&](int t) {
        const size_t a = total * t / P, b = total * (t + 1) / P;
        crc[(size_t)t] = crc32_update(0, o + a, b - a);
    });
    uint32_t all = 0;
    for (int t = 0; t < P; ++t) all = crc32_join(all, crc[(size_t)t], (int64_t)(total * (t + 1) / P - total * t / P));
    mark("crc");
    return all == crc_want ? 0 : -1;
}

template int gunzip_single_parallel<std::string>(const uint8_t *, int64_t, std::string &, int);
template int gunzip_single_parallel<TextBuf>(const uint8_t *, int64_t, TextBuf &, int);

}  // namespace mh
