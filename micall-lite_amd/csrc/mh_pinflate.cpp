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
//   2. decode: every span after the first inflated twice from its start to
//      the next span's start (libdeflate when present: the span's bits are
//      laid out byte-aligned behind a stored block holding the window and
//      closed by an empty final block; zlib with inflatePrime and
//      inflateSetDictionary otherwise), in place of the unknown window
//      once with window bytes W1[i] = i % 255 + 1 and once with W2[i] =
//      (i / 255 + i % 255 + 1) % 255 + 1: a byte of the data comes out the
//      same in both, a byte copied out of the window at offset i comes out
//      as W1[i] / W2[i], which always differ and give i back; a span must
//      end exactly on the next one's start (else the start was false and the
//      caller decodes serially);
//   3. resolve: every window-derived byte replaced from the true window (the
//      32 KiB before its span) -- the last 32 KiB of every span in order, as
//      each is the next span's window, then everything else at once.  (Back-
//      references keep window bytes alive through most of a span of FASTQ,
//      so decoding the span again once its window is known would be nearly
//      serial.)
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
#include <memory>
#include <system_error>
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

// fn(t) on nt threads; an exception in a worker (an allocation failure)
// ends that worker and makes the call return false, so the caller falls
// back to the serial inflate instead of the process terminating
bool threads_run(int nt, const std::function<void(int)> &fn)
{
    std::atomic<int> failed(0);
    auto guarded = [&](int t) {
        try {
            fn(t);
        } catch (...) {
            failed = 1;
        }
    };
    if (nt <= 1) {
        guarded(0);
        return !failed;
    }
    std::vector<std::thread> th;
    try {
        for (int t = 1; t < nt; ++t) th.emplace_back(guarded, t);
    } catch (const std::system_error &) {   // no more threads: the rest run here
        for (int t = (int)th.size() + 1; t < nt; ++t) guarded(t);
    }
    guarded(0);
    for (auto &x : th) x.join();
    return !failed;
}

// The DEFLATE bits [b0, b1) of src, byte-aligned, into in[pre ..) (the
// caller fills in[0 .. pre)); with `close`, followed by a final empty stored
// block (BFINAL 1, BTYPE 00, LEN 0) so that a decoder stops at b1.
bool lay_out_span(const uint8_t *src, int64_t len, int64_t b0, int64_t b1, bool close, size_t pre,
                  TextBuf &in)
{
    const int64_t nbits = b1 - b0, nb = (nbits + 7) / 8;
    if (nbits <= 0 || (b1 + 7) / 8 > len) return false;
    in.resize(pre + (size_t)nb + (close ? 5 : 0));
    uint8_t *o = (uint8_t *)in.data() + pre;
    const uint8_t *p = src + (b0 >> 3);
    const int r = (int)(b0 & 7);
    const int64_t avail = len - (b0 >> 3);   // readable bytes from p
    int64_t j = 0;
    if (r == 0) {
        memcpy(o, p, (size_t)nb);
        j = nb;
    } else {
        for (; j + 8 < nb && j + 9 <= avail; j += 8) {
            uint64_t x;
            memcpy(&x, p + j, 8);
            const uint64_t y = (x >> r) | ((uint64_t)p[j + 8] << (64 - r));
            memcpy(o + j, &y, 8);
        }
        for (; j < nb; ++j)
            o[j] = (uint8_t)((p[j] >> r) | (j + 1 < avail ? p[j + 1] << (8 - r) : 0));
    }
    const int tail = (int)(nbits & 7);
    if (!close) return true;
    // the closing block's 3 header bits at bit nbits, then LEN 0 / NLEN 0xffff
    int64_t at = nb;
    if (tail) {
        o[nb - 1] &= (uint8_t)((1u << tail) - 1);
        if (tail <= 5) o[nb - 1] |= (uint8_t)(1u << tail);
        else { o[nb - 1] |= (uint8_t)(1u << tail); o[at++] = 0; }   // BTYPE spills into a new byte
    } else {
        o[at++] = 1;
    }
    o[at++] = 0; o[at++] = 0; o[at++] = 0xff; o[at++] = 0xff;
    in.resize(pre + (size_t)at);
    return true;
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

// W1[i] = i % 255 + 1 and W2[i] = (i / 255 + i % 255 + 1) % 255 + 1: the
// two stand-in windows.  A byte of the data comes out of a span's two
// decodes the same; a byte copied from window offset i comes out as W1[i]
// and W2[i], which always differ (i / 255 <= 128) and give i back (at_of).
struct Windows {
    uint8_t w1[WIN], w2[WIN];
    std::vector<uint16_t> at_of;
    Windows() : at_of(65536, 0xffff)
    {
        for (int i = 0; i < WIN; ++i) {
            w1[i] = (uint8_t)(i % 255 + 1);
            w2[i] = (uint8_t)((i / 255 + i % 255 + 1) % 255 + 1);
            at_of[(size_t)w1[i] << 8 | w2[i]] = (uint16_t)i;
        }
    }
};

const Windows &windows()
{
    static const Windows w;
    return w;
}

// The first dynamic-Huffman block start in bytes [a, b) of the deflate data
// src[0 .. dend) (a bit position whose header parses and from which two
// blocks decode with a zero window), or -1.
int64_t find_block(const uint8_t *src, int64_t dend, int64_t a, int64_t b)
{
    static const std::vector<uint8_t> zeros(WIN, 0);
    TextBuf probe;
    for (int64_t bit = a * 8; bit < b * 8; ++bit) {
        if (!dyn_header_ok(src, dend, bit)) continue;
        int64_t e = 0;
        probe.clear();
        if (inflate_to(src, dend, bit, zeros.data(), WIN, -1, probe, &e, 2) == 0) return bit;
    }
    return -1;
}

// Span starts in bytes [a, b): span 0 starts at first_bit (known), spans
// 1 .. T-1 at the first block start at or after a + (b - a) * t / T.
// Starts not found are dropped.  false on a worker failure.
bool find_spans(const uint8_t *src, int64_t dend, int64_t a, int64_t b, int T, int64_t first_bit,
                std::vector<int64_t> &st)
{
    std::vector<int64_t> found((size_t)T, -1);
    found[0] = first_bit;
    if (!threads_run(T - 1, [&](int i) {
            const int t = i + 1;
            found[(size_t)t] = find_block(src, dend, a + (b - a) * t / T, a + (b - a) * (t + 1) / T);
        }))
        return false;
    st.clear();
    for (int64_t f : found) if (f >= 0) st.push_back(f);
    return true;
}

// Decode spans k = 0 .. K-1 of src (deflate data ending at byte dend):
// bits [st[k], st[k + 1]), the last one to end_bit -- to the end of the
// deflate stream when end_bit is dend * 8, else closed there by an empty
// final block.  Span 0 has no window unless `windowed`; every windowed span
// is decoded twice, with W1 and with W2 in place of its window (p1 / p2;
// skip[k] bytes of p1 / p2 come before the span's data).  false on a decode
// error or a false start (a span that does not end exactly on the next one).
bool decode_spans(const uint8_t *src, int64_t len, int64_t dend, const std::vector<int64_t> &st,
                  int64_t end_bit, bool windowed, int threads, std::vector<TextBuf> &p1,
                  std::vector<TextBuf> &p2, std::vector<size_t> &skip, bool trace)
{
    const int K = (int)st.size();
    const Windows &W = windows();
    const bool to_stream_end = end_bit == dend * 8;
    auto has_window = [&](int k) { return k > 0 || windowed; };
    p1.clear();
    p1.resize((size_t)K);
    p2.clear();
    p2.resize((size_t)K);
    skip.assign((size_t)K, 0);
    std::atomic<int> bad(0);
    // MICALL_ZLIB_SPANS=1: the zlib span decode even when libdeflate is present
    static const bool zlib_spans = getenv("MICALL_ZLIB_SPANS") && *getenv("MICALL_ZLIB_SPANS") == '1';
    void *probe_ld = zlib_spans ? nullptr : ld_raw_alloc();
    if (probe_ld) {
        ld_raw_free(probe_ld);
        // libdeflate (raw, no dictionary or bit-offset API): each span is
        // re-laid out byte-aligned behind a stored block holding the window
        // (so back-references reach it), and a final empty stored block is
        // put where the next span starts, so the decode ends there
        std::atomic<int> next(0);
        if (!threads_run(std::min(K, threads), [&](int) {
                void *d = ld_raw_alloc();
                if (!d) { bad = 1; return; }
                TextBuf in;
                for (int k; (k = next.fetch_add(1)) < K;) {
                    const bool last = k + 1 == K;
                    const bool stream_end = last && to_stream_end;
                    const int64_t b0 = st[(size_t)k], b1 = last ? end_bit : st[(size_t)k + 1];
                    const size_t pre = has_window(k) ? 5 + WIN : 0;
                    if (!lay_out_span(src, len, b0, b1, !stream_end, pre, in)) { bad = 1; break; }
                    for (int which = 1; which <= (has_window(k) ? 2 : 1); ++which) {
                        if (has_window(k)) {
                            uint8_t *w = (uint8_t *)in.data();
                            w[0] = 0; w[1] = 0x00; w[2] = 0x80; w[3] = 0xff; w[4] = 0x7f;   // LEN 32768
                            memcpy(w + 5, which == 1 ? W.w1 : W.w2, WIN);
                        }
                        TextBuf &dst = which == 1 ? p1[(size_t)k] : p2[(size_t)k];
                        size_t cap = (size_t)WIN + (size_t)((b1 - b0) / 8) * 6 + ((size_t)1 << 20);
                        for (;;) {
                            dst.resize(cap);
                            size_t in_used = 0, out_used = 0;
                            const int r = ld_raw_inflate(d, (const uint8_t *)in.data(), in.size(), dst.data(),
                                                         cap, &in_used, &out_used);
                            if (r == 3) { cap *= 2; continue; }
                            // the stream's last span ends inside its last byte:
                            // libdeflate may leave that byte uncounted
                            const size_t unread = in.size() - std::min(in_used, in.size());
                            if (r != 0 || unread > (stream_end ? 1u : 0u) ||
                                out_used < (has_window(k) ? (size_t)WIN : 0)) {
                                if (trace)
                                    fprintf(stderr, "pinflate span %d rc %d in %zu of %zu out %zu\n", k, r,
                                            in_used, in.size(), out_used);
                                bad = 1;
                                break;
                            }
                            dst.resize(out_used);
                            break;
                        }
                        if (bad) break;
                    }
                    skip[(size_t)k] = has_window(k) ? WIN : 0;
                    if (bad) break;
                }
                ld_raw_free(d);
            }))
            bad = 1;
        return !bad;
    }
    std::vector<int64_t> e1((size_t)K, -1), e2((size_t)K, -1);
    std::vector<std::pair<int, int>> jobs;   // (span, window 1 / 2)
    for (int k = 0; k < K; ++k) {
        jobs.emplace_back(k, 1);
        if (has_window(k)) jobs.emplace_back(k, 2);
    }
    std::atomic<size_t> next(0);
    if (!threads_run(std::min<int>((int)jobs.size(), threads), [&](int) {
            for (size_t j; (j = next.fetch_add(1)) < jobs.size();) {
                const int k = jobs[j].first, which = jobs[j].second;
                const int64_t b1 = k + 1 < K ? st[(size_t)k + 1] : end_bit;
                const int64_t stop = k + 1 < K || !to_stream_end ? b1 : -1;
                TextBuf &dst = which == 1 ? p1[(size_t)k] : p2[(size_t)k];
                dst.resize((size_t)std::max<int64_t>(1 << 20, (b1 - st[(size_t)k]) / 2));
                const uint8_t *dict = !has_window(k) ? nullptr : which == 1 ? W.w1 : W.w2;
                if (inflate_to(src, dend, st[(size_t)k], dict, has_window(k) ? WIN : 0, stop, dst,
                               which == 1 ? &e1[(size_t)k] : &e2[(size_t)k]))
                    bad = 1;
            }
        }))
        bad = 1;
    if (bad) return false;
    if (to_stream_end && (e1[(size_t)K - 1] + 7) / 8 != dend) return false;
    for (int k = 0; k < K; ++k)
        if (has_window(k) && e1[(size_t)k] != e2[(size_t)k]) return false;
    return true;
}

// A run of decoded spans placed into one text.  Every window-derived byte
// of span k >= 1 is replaced by the byte it copies from the text before the
// span.  With `windowed`, span 0's window is not known here (it is another
// rank's text): span 0's window-derived bytes stay symbolic -- the pair
// (W1[i], W2[i]) of their window offset i, in the text (plane 1) and in o2
// (plane 2) -- and so does every byte that copies one.  Plane 2 is written
// only over each span's dirty prefix (dirty[k]: the end of the span's last
// byte that differs between its two decodes); beyond it a span is plain.
struct Placement {
    std::vector<size_t> off, dirty, skip;
    std::vector<TextBuf> p1, p2;
    TextBuf o2;
    bool windowed = false;
    int K = 0;
    size_t span_len(int k) const { return off[(size_t)k + 1] - off[(size_t)k]; }
    size_t tail0(int k) const { return span_len(k) > (size_t)WIN ? span_len(k) - WIN : (size_t)0; }
    size_t total() const { return off[(size_t)K]; }
};

// off[] from the decodes; false when they disagree on a span's length, or
// (windowed) a span before the last is shorter than a window (plane 2 of a
// span's window must lie in the span before it)
bool plan(Placement &P)
{
    const int K = P.K;
    P.off.assign((size_t)K + 1, 0);
    P.dirty.assign((size_t)K, 0);
    for (int k = 0; k < K; ++k) {
        if ((k || P.windowed) && P.p1[(size_t)k].size() != P.p2[(size_t)k].size()) return false;
        P.off[(size_t)k + 1] = P.off[(size_t)k] + P.p1[(size_t)k].size() - P.skip[(size_t)k];
    }
    if (P.windowed)
        for (int k = 0; k + 1 < K; ++k)
            if (P.span_len(k) < (size_t)WIN) return false;
    return true;
}

void find_dirty(Placement &P, int threads)
{
    std::atomic<int> next(P.windowed ? 0 : 1);
    threads_run(std::min(P.K, threads), [&](int) {
        for (int k; (k = next.fetch_add(1)) < P.K;) {
            const char *a1 = P.p1[(size_t)k].data() + P.skip[(size_t)k];
            const char *a2 = P.p2[(size_t)k].data() + P.skip[(size_t)k];
            size_t i = P.span_len(k);
            while (i >= 8) {
                uint64_t x, y;
                memcpy(&x, a1 + i - 8, 8);
                memcpy(&y, a2 + i - 8, 8);
                if (x != y) break;
                i -= 8;
            }
            while (i > 0 && a1[i - 1] == a2[i - 1]) --i;
            P.dirty[(size_t)k] = i;
        }
    });
}

// bytes [i0, i1) of span k into text o (and plane 2); false on a byte pair
// that names no window offset
bool place(Placement &P, char *o, int k, size_t i0, size_t i1)
{
    if (i0 >= i1) return true;
    const size_t base = P.off[(size_t)k];
    char *dst = o + base;
    const char *A = P.p1[(size_t)k].data() + P.skip[(size_t)k];
    const size_t dk = P.dirty[(size_t)k];
    const size_t d = std::min(std::max(dk, i0), i1);   // clean from d on
    if (d < i1) memcpy(dst + d, A + d, i1 - d);
    if (i0 >= d) return true;
    const uint8_t *B = (const uint8_t *)P.p2[(size_t)k].data() + P.skip[(size_t)k];
    const bool sym = P.windowed;
    char *dst2 = sym ? P.o2.data() + base : nullptr;
    if (k == 0) {            // windowed span 0: its window bytes stay symbolic
        memcpy(dst + i0, A + i0, d - i0);
        memcpy(dst2 + i0, B + i0, d - i0);
        return true;
    }
    const char *wb = o + base - WIN;
    const char *wb2 = sym ? P.o2.data() + base - WIN : nullptr;
    // window offsets below wsym are in the span before's dirty prefix (plane
    // 2 valid there); from wsym on that span is plain
    const size_t prev_end = P.off[(size_t)k - 1] + P.dirty[(size_t)k - 1];
    const size_t wsym = prev_end > base - WIN ? prev_end - (base - WIN) : 0;
    const uint16_t *T = windows().at_of.data();
    for (size_t i = i0; i < d;) {
        if (i + 8 <= d) {                              // 8 bytes of the data
            uint64_t x, y;
            memcpy(&x, A + i, 8);
            memcpy(&y, B + i, 8);
            if (x == y) {
                memcpy(dst + i, &x, 8);
                if (sym) memcpy(dst2 + i, &x, 8);
                i += 8;
                continue;
            }
        }
        const size_t e = std::min(i + 8, d);
        for (; i < e; ++i) {
            const int a1 = (uint8_t)A[i], a2 = B[i];
            if (a1 == a2) {                            // a byte of the data
                dst[i] = (char)a1;
                if (sym) dst2[i] = (char)a1;
                continue;
            }
            const int idx = T[a1 << 8 | a2];
            if (idx == 0xffff) return false;
            dst[i] = wb[idx];
            if (sym) dst2[i] = (size_t)idx < wsym ? wb2[idx] : wb[idx];
        }
    }
    return true;
}

// The spans placed into `out` (resized to the total): the tails in order
// (each is the next span's window), then the rest in pieces of about 4 MiB
// on `threads` threads.  Without a window (!P.windowed) the text is final
// and piece_crc gets each piece's CRC-32 (pieces: (start, length)).
template <class Buf>
bool place_all(Placement &P, Buf &out, int threads, std::vector<std::pair<size_t, size_t>> *pieces_out,
               std::vector<uint32_t> *piece_crc)
{
    out.resize(P.total());
    char *o = &out[0];
    if (P.windowed) P.o2.resize(P.total());    // pages touched only where written
    for (int k = 0; k < P.K; ++k)
        if (!place(P, o, k, P.tail0(k), P.span_len(k))) return false;
    struct Piece { int k; size_t a, b; };
    std::vector<Piece> pieces;
    for (int k = 0; k < P.K; ++k) {
        const size_t n = P.span_len(k);
        const size_t np = std::max<size_t>(1, n >> 22);
        for (size_t j = 0; j < np; ++j)
            pieces.push_back({k, n * j / np, j + 1 < np ? n * (j + 1) / np : n});
    }
    std::vector<uint32_t> crc(pieces.size(), 0);
    std::atomic<int> bad(0);
    std::atomic<size_t> next(0);
    const bool want_crc = piece_crc != nullptr;
    threads_run(std::min<int>((int)pieces.size(), threads), [&](int) {
        for (size_t j; (j = next.fetch_add(1)) < pieces.size();) {
            const Piece &pc = pieces[j];
            if (!place(P, o, pc.k, pc.a, std::min(pc.b, P.tail0(pc.k)))) bad = 1;
            if (want_crc) crc[j] = crc32_update(0, o + P.off[(size_t)pc.k] + pc.a, pc.b - pc.a);
        }
    });
    if (bad) return false;
    if (pieces_out) {
        pieces_out->clear();
        for (const Piece &pc : pieces) pieces_out->emplace_back(P.off[(size_t)pc.k] + pc.a, pc.b - pc.a);
    }
    if (piece_crc) piece_crc->swap(crc);
    return true;
}

// the span decodes freed on a detached thread (GBs of pages)
void free_later(std::vector<TextBuf> &a, std::vector<TextBuf> &b)
{
    auto hold = std::make_shared<std::pair<std::vector<TextBuf>, std::vector<TextBuf>>>(std::move(a),
                                                                                     std::move(b));
    std::thread([hold]() { hold->first.clear(); hold->second.clear(); }).detach();
}

// the smallest span of compressed bytes a thread is given (4 MiB;
// MH_PINFLATE_SPAN_MIN overrides it, so tests can make many spans of a few MB)
int64_t span_min_bytes()
{
    const char *e = getenv("MH_PINFLATE_SPAN_MIN");
    const int64_t v = e ? atoll(e) : 0;
    return v >= (1 << 16) ? v : (int64_t)4 << 20;
}

// bytes of memory the kernel reports available, or -1
int64_t mem_available()
{
    FILE *f = fopen("/proc/meminfo", "r");
    if (!f) return -1;
    char line[256];
    int64_t kb = -1;
    while (fgets(line, sizeof line, f))
        if (sscanf(line, "MemAvailable: %ld kB", &kb) == 1) break;
    fclose(f);
    return kb < 0 ? -1 : kb * 1024;
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
    // the two decodes of every span and the text are held at once (about
    // 3x the text; a span of FASTQ stays window-dependent nearly to its end,
    // 63.0 of 63.0 MB in a C2-like file, so plane 2 cannot be cut short):
    // leave this to the serial inflate when memory is short.  The trailer's
    // size is mod 2^32; FASTQ inflates about 4x, so that bounds it too.
    const int64_t avail = mem_available();
    const int64_t text = std::max<int64_t>((int64_t)isize, 4 * (dend - d0));
    if (avail >= 0 && 3 * text > avail / 2) return -1;
    const int64_t span_min = span_min_bytes();
    const int T = (int)std::min<int64_t>(threads, (dend - d0) / span_min);
    if (T < 2) return -1;
    // 1. span starts
    Placement P;
    std::vector<int64_t> st;
    if (!find_spans(src, dend, d0, dend, T, d0 * 8, st)) return -1;
    mark("search");
    if (st.size() < 2) return -1;
    P.K = (int)st.size();
    // 2. every span after the first decoded twice
    if (!decode_spans(src, len, dend, st, dend * 8, false, threads, P.p1, P.p2, P.skip, trace)) return -1;
    mark("decode");
    if (!plan(P)) return -1;
    // the first span's output must hold a whole window
    if ((uint32_t)P.total() != isize || P.off[1] < (size_t)WIN) return -1;
    // 3. the output placed with every window-derived byte replaced by the
    // window byte it copies, each piece's CRC-32 taken while in cache
    find_dirty(P, threads);
    mark("dirty");
    std::vector<std::pair<size_t, size_t>> pieces;
    std::vector<uint32_t> crc;
    const bool ok = place_all(P, out, threads, &pieces, &crc);
    mark("place");
    free_later(P.p1, P.p2);
    mark("free");
    if (trace) {
        size_t d = 0;
        for (size_t x : P.dirty) d += x;
        fprintf(stderr, "pinflate spans %d dirty bytes %zu\n", P.K, d);
    }
    if (!ok) return -1;
    // 4. the CRC-32 of the whole output against the trailer
    uint32_t all = 0;
    for (size_t j = 0; j < pieces.size(); ++j) all = crc32_join(all, crc[j], (int64_t)pieces[j].second);
    mark("crc");
    return all == crc_want ? 0 : -1;
}

template int gunzip_single_parallel<std::string>(const uint8_t *, int64_t, std::string &, int);
template int gunzip_single_parallel<TextBuf>(const uint8_t *, int64_t, TextBuf &, int);

// ---- one part of one gzip member, for a job of several ranks ----------------
//
// Rank p of P holds the deflate bits from its first block start in bytes
// [d0 + (dend - d0) * p / P, ...) to the next rank's first block start.  It
// decodes them on its threads (the spans above, span 0 with an unknown
// window except on rank 0) without any other rank's data; only its window
// -- the last 32 KiB of the rank before's text -- is missing, and it arrives
// through the caller's point-to-point chain: rank p resolves its own last
// 32 KiB (member_part_tail) once it has its window and passes them on.
// member_part_finish then resolves the rest of the text in parallel and
// gives the CRC-32 of the rank's text; the caller combines the ranks' CRCs
// and checks them and the total size against the gzip trailer.

struct MemberPart {
    const uint8_t *src = nullptr;
    int64_t len = 0, d0 = 0, dend = 0;
    std::vector<int64_t> st;      // this part's span starts (bits)
    Placement P;
    bool decoded = false;
};

MemberPart *member_part_open(const uint8_t *src, int64_t len, int part, int parts, int threads,
                             int64_t *info)
{
    const int64_t d0 = gzip_header_end(src, len);
    if (d0 < 0) return nullptr;
    std::unique_ptr<MemberPart> m(new MemberPart());
    m->src = src;
    m->len = len;
    m->d0 = d0;
    m->dend = len - 8;
    const int64_t a = d0 + (m->dend - d0) * part / parts, b = d0 + (m->dend - d0) * (part + 1) / parts;
    const int64_t span_min = span_min_bytes();
    const int T = (int)std::max<int64_t>(1, std::min<int64_t>(threads, (b - a) / span_min));
    // span 0: rank 0 starts at the stream's start; every other rank at its
    // range's first block start (searched with the others, on a thread)
    int64_t first = part == 0 ? d0 * 8 : -1;
    std::vector<int64_t> found((size_t)T, -1);
    if (!threads_run(T, [&](int t) {
            if (t == 0 && part == 0) { found[0] = d0 * 8; return; }
            found[(size_t)t] = find_block(src, m->dend, a + (b - a) * t / T, a + (b - a) * (t + 1) / T);
        }))
        return nullptr;
    first = found[0];
    if (first >= 0)
        for (int64_t f : found) if (f >= 0) m->st.push_back(f);
    info[0] = first;                               // -1: no block start in the range
    info[1] = m->dend * 8;
    info[2] = rd32(src + len - 8);                 // the trailer's CRC-32 and size
    info[3] = rd32(src + len - 4);
    info[4] = (int64_t)m->st.size();
    return m.release();
}

int member_part_decode(MemberPart *m, int64_t end_bit, bool windowed, int threads)
{
    if (m->st.empty() || end_bit <= m->st.back() || end_bit > m->dend * 8) return -1;
    Placement &P = m->P;
    P.windowed = windowed;
    P.K = (int)m->st.size();
    if (!decode_spans(m->src, m->len, m->dend, m->st, end_bit, windowed, threads, P.p1, P.p2, P.skip,
                      false))
        return -1;
    if (!plan(P)) return -1;
    if (P.total() < (size_t)WIN) return -1;        // the next rank's window lies in this text
    if (windowed || P.K > 1) find_dirty(P, threads);
    m->decoded = true;
    return 0;
}

template <class Buf>
int member_part_place(MemberPart *m, Buf &out, int threads)
{
    if (!m->decoded) return -1;
    const bool ok = place_all(m->P, out, threads, nullptr, nullptr);
    free_later(m->P.p1, m->P.p2);
    return ok ? 0 : -1;
}

namespace {

// plane-2 bytes of [i0, i1) resolved from the window
bool resolve(MemberPart *m, char *o, const char *window, size_t i0, size_t i1)
{
    const Placement &P = m->P;
    if (!P.windowed) return true;
    const uint16_t *T = windows().at_of.data();
    const char *o2 = P.o2.data();
    for (int k = 0; k < P.K; ++k) {          // only dirty prefixes hold plane 2
        const size_t a = std::max(i0, P.off[(size_t)k]);
        const size_t b = std::min(i1, P.off[(size_t)k] + P.dirty[(size_t)k]);
        for (size_t i = a; i < b;) {
            if (i + 8 <= b) {
                uint64_t x, y;
                memcpy(&x, o + i, 8);
                memcpy(&y, o2 + i, 8);
                if (x == y) { i += 8; continue; }
            }
            const size_t e = std::min(i + 8, b);
            for (; i < e; ++i) {
                const int a1 = (uint8_t)o[i], a2 = (uint8_t)o2[i];
                if (a1 == a2) continue;
                const int idx = T[a1 << 8 | a2];
                if (idx == 0xffff) return false;
                o[i] = window[idx];
            }
        }
    }
    return true;
}

}  // namespace

template <class Buf>
int member_part_tail(MemberPart *m, Buf &out, const char *window, char *tail)
{
    const size_t n = m->P.total();
    if (n < (size_t)WIN || out.size() != n) return -1;
    if (m->P.windowed && !window) return -1;
    if (!resolve(m, &out[0], window, n - WIN, n)) return -1;
    memcpy(tail, &out[0] + n - WIN, WIN);
    return 0;
}

template <class Buf>
int member_part_finish(MemberPart *m, Buf &out, const char *window, int threads, uint32_t *crc_out)
{
    const size_t n = m->P.total();
    if (out.size() != n || (m->P.windowed && !window)) return -1;
    const size_t tail = n - WIN;               // resolved by member_part_tail
    const size_t np = std::max<size_t>(1, n >> 22);
    std::vector<uint32_t> crc(np, 0);
    std::atomic<int> bad(0);
    std::atomic<size_t> next(0);
    char *o = &out[0];
    threads_run((int)std::min<size_t>(np, (size_t)threads), [&](int) {
        for (size_t j; (j = next.fetch_add(1)) < np;) {
            const size_t a = n * j / np, b = j + 1 < np ? n * (j + 1) / np : n;
            if (!resolve(m, o, window, a, std::min(b, tail))) bad = 1;
            crc[j] = crc32_update(0, o + a, b - a);
        }
    });
    m->P.o2.release();
    if (bad) return -1;
    uint32_t all = 0;
    for (size_t j = 0; j < np; ++j) {
        const size_t a = n * j / np, b = j + 1 < np ? n * (j + 1) / np : n;
        all = crc32_join(all, crc[j], (int64_t)(b - a));
    }
    *crc_out = all;
    return 0;
}

void member_part_free(MemberPart *m) { delete m; }

template int member_part_place<TextBuf>(MemberPart *, TextBuf &, int);
template int member_part_tail<TextBuf>(MemberPart *, TextBuf &, const char *, char *);
template int member_part_finish<TextBuf>(MemberPart *, TextBuf &, const char *, int, uint32_t *);

}  // namespace mh
