// mh_censor.hip -- censor_fastq.censor (micall/core/censor_fastq.py:32-102)
// on gfx950, behind mh_censor_fastq / mh_censor_output:
//   host      gunzip (multi-member): libdeflate on the whole file when the
//             system has it, else streaming zlib (a producer thread inflates
//             ~32 MB chunks while the whole records of the chunks already
//             there are censored); records split in parallel,
//             tile + read direction from each header exactly as :59-63 parse
//             them, bad (tile, cycle) set from the caller
//   k_censor  one wave64 per read: the bases / qualities of bad cycles
//             become 'N' / '#' in place, the trailing run of bad cycles is
//             dropped (the reference only flushes pending Ns before a good
//             cycle, :66-74, :78-90), and every quality score is summed for
//             the summary (:80-82) -- per-block sums, one atomic per block
//   host      records rewritten (header and '+' lines verbatim), optional
//             gzip as independent deflate members compressed in parallel
#include <zlib.h>

#include <algorithm>
#include <chrono>
#include <condition_variable>
#include <deque>
#include <mutex>
#include <cstring>
#include <functional>
#include <string>
#include <thread>
#include <unordered_map>
#include <vector>

#include "mh_gunzip.h"
#include "mh_internal.h"

namespace mh {

int s2a_threads();   // mh_s2a_host.cpp: host worker count

struct CensorState {
    std::string text;                       // the FASTQ (censored in place)
    // per record: spans into text
    std::vector<int64_t> h0, s0, o0, q0;    // header, seq, '+' line, qual starts
    std::vector<int32_t> hl, sl, ol, ql;    // line lengths incl. their newline (h, o) /
                                            // stripped lengths (s, q)
    std::vector<int32_t> tile, sign;        // tile id (-1: no bad cycle) / +1, -1
    std::vector<int32_t> keep;              // 2 per record: kept seq / qual length
    int64_t base_count = 0, score_sum = 0;
    int64_t rec_base = 0;                   // records before this piece (messages)
    std::string out;
    double t_host_in = 0, t_device = 0, t_host_out = 0;
    // device buffers, grown on demand and kept between pieces and calls
    uint8_t *d_text = nullptr;
    int64_t *d_s0 = nullptr, *d_q0 = nullptr;
    int32_t *d_sl = nullptr, *d_ql = nullptr, *d_tile = nullptr, *d_sign = nullptr, *d_keep = nullptr;
    uint32_t *d_bad = nullptr;
    unsigned long long *d_sums = nullptr;
    int64_t cap_text = 0, cap_rec = 0, cap_bad = 0;
};

static void censor_free_device(CensorState &C)
{
    hipFree(C.d_text); hipFree(C.d_s0); hipFree(C.d_q0); hipFree(C.d_sl); hipFree(C.d_ql);
    hipFree(C.d_tile); hipFree(C.d_sign); hipFree(C.d_keep); hipFree(C.d_bad); hipFree(C.d_sums);
    C.d_text = nullptr; C.d_s0 = C.d_q0 = nullptr;
    C.d_sl = C.d_ql = C.d_tile = C.d_sign = C.d_keep = nullptr;
    C.d_bad = nullptr; C.d_sums = nullptr;
    C.cap_text = C.cap_rec = C.cap_bad = 0;
}

static void cz_parallel(int nt, const std::function<void(int)> &fn)
{
    if (nt <= 1) { fn(0); return; }
    std::vector<std::thread> th;
    for (int t = 1; t < nt; ++t) th.emplace_back(fn, t);
    fn(0);
    for (auto &x : th) x.join();
}

void censor_free(Ctx &c)
{
    if (c.censor) censor_free_device(*c.censor);
    delete c.censor;
    c.censor = nullptr;
}

// ---------------------------------------------------------------------------
// device
// ---------------------------------------------------------------------------
struct CensorArgs {
    uint8_t *text;
    const int64_t *s0, *q0;
    const int32_t *sl, *ql, *tile, *sign;
    int64_t n;
    const uint32_t *bad;     // per bad tile: bitmap over cycles -maxc .. maxc
    int maxc, words;         // words per tile bitmap
    int32_t *keep;
    unsigned long long *sums;   // [0] score sum (two's complement), [1] bases
};

__device__ __forceinline__ bool censor_bad(const CensorArgs &A, int t, int cyc)
{
    if (t < 0 || cyc < -A.maxc || cyc > A.maxc) return false;
    const int b = cyc + A.maxc;
    return (A.bad[(int64_t)t * A.words + (b >> 5)] >> (b & 31)) & 1u;
}

__global__ __launch_bounds__(256) void k_censor(CensorArgs A)
{
    __shared__ long long part_sum[4];
    __shared__ long long part_n[4];
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    long long ssum = 0, nb = 0;
    for (int64_t r = (int64_t)blockIdx.x * 4 + wv; r < A.n; r += (int64_t)gridDim.x * 4) {
        const int t = A.tile[r], sg = A.sign[r];
        // bases
        int last = 0;
        uint8_t *s = A.text + A.s0[r];
        for (int i = lane; i < A.sl[r]; i += 64) {
            if (censor_bad(A, t, sg * (i + 1))) s[i] = 'N';
            else last = i + 1;
        }
        for (int o = 32; o > 0; o >>= 1) last = max(last, __shfl_xor(last, o, 64));
        const int keep_s = last;
        // qualities (summed before censoring)
        last = 0;
        uint8_t *q = A.text + A.q0[r];
        for (int i = lane; i < A.ql[r]; i += 64) {
            ssum += (long long)q[i] - 33;
            if (censor_bad(A, t, sg * (i + 1))) q[i] = '#';
            else last = i + 1;
        }
        nb += A.ql[r] > lane ? (A.ql[r] - lane + 63) / 64 : 0;
        for (int o = 32; o > 0; o >>= 1) last = max(last, __shfl_xor(last, o, 64));
        if (lane == 0) {
            A.keep[2 * r] = keep_s;
            A.keep[2 * r + 1] = last;
        }
    }
    for (int o = 32; o > 0; o >>= 1) {
        ssum += __shfl_xor(ssum, o, 64);
        nb += __shfl_xor(nb, o, 64);
    }
    if (lane == 0) { part_sum[wv] = ssum; part_n[wv] = nb; }
    __syncthreads();
    if (threadIdx.x == 0) {
        long long a = 0, b = 0;
        for (int w = 0; w < (int)(blockDim.x >> 6); ++w) { a += part_sum[w]; b += part_n[w]; }
        if (a) atomicAdd(&A.sums[0], (unsigned long long)a);
        if (b) atomicAdd(&A.sums[1], (unsigned long long)b);
    }
}

// ---------------------------------------------------------------------------
// host
// ---------------------------------------------------------------------------
// gzip of `in` as independent members of `block` bytes, compressed in parallel
static int gzip_parallel(const std::string &in, std::string &out, int level)
{
    const int64_t block = 8 << 20;
    const int64_t nblk = std::max<int64_t>(1, ((int64_t)in.size() + block - 1) / block);
    std::vector<std::string> parts((size_t)nblk);
    std::vector<int> err((size_t)nblk, 0);
    const int nt = (int)std::min<int64_t>(s2a_threads(), nblk);
    cz_parallel(nt, [&](int t) {
        for (int64_t b = t; b < nblk; b += nt) {
            const int64_t a = b * block, e = std::min<int64_t>((int64_t)in.size(), a + block);
            if (gzip_member(in.data() + a, (size_t)(e - a), parts[b], level)) err[b] = 1;
        }
    });
    for (int e : err) if (e) { set_error("censor: deflate failed"); return -2; }
    size_t total = 0;
    for (auto &p : parts) total += p.size();
    out.clear();
    out.reserve(total);
    for (auto &p : parts) out += p;
    return 0;
}

static inline bool py_space(unsigned char c)
{
    return c == ' ' || (c >= 9 && c <= 13) || (c >= 0x1c && c <= 0x1f);
}

// records of the FASTQ text: 4 lines each (itertools.zip_longest, :57)
static int split_records(CensorState &C, const std::unordered_map<std::string, int> &tiles)
{
    const std::string &T = C.text;
    const int64_t n = (int64_t)T.size();
    // line starts, in parallel chunks
    const int nt = s2a_threads();
    std::vector<std::vector<int64_t>> ls(nt);
    cz_parallel(nt, [&](int t) {
        const int64_t a = n * t / nt, b = n * (t + 1) / nt;
        for (int64_t i = a; i < b; ++i)
            if (T[i] == '\n' && i + 1 < n) ls[t].push_back(i + 1);
    });
    std::vector<int64_t> starts;
    if (n > 0) starts.push_back(0);
    for (auto &v : ls) starts.insert(starts.end(), v.begin(), v.end());
    const int64_t nl = (int64_t)starts.size();
    if (nl % 4) {
        set_error("censor: FASTQ has %lld lines, not a multiple of 4",
                  (long long)(nl + 4 * C.rec_base));
        return -3;
    }
    const int64_t nr = nl / 4;
    C.h0.resize(nr); C.s0.resize(nr); C.o0.resize(nr); C.q0.resize(nr);
    C.hl.resize(nr); C.sl.resize(nr); C.ol.resize(nr); C.ql.resize(nr);
    C.tile.resize(nr); C.sign.resize(nr);
    std::vector<int> bad(nt, 0);
    std::vector<int64_t> bad_rec(nt, -1);
    auto line_end = [&](int64_t k) { return k + 1 < nl ? starts[k + 1] : n; };   // after '\n'
    cz_parallel(nt, [&](int t) {
        for (int64_t r = nr * t / nt; r < nr * (t + 1) / nt; ++r) {
            const int64_t k = 4 * r;
            const int64_t ha = starts[k], he = line_end(k);
            C.h0[r] = ha; C.hl[r] = (int32_t)(he - ha);
            C.o0[r] = starts[k + 2]; C.ol[r] = (int32_t)(line_end(k + 2) - starts[k + 2]);
            auto stripped = [&](int64_t a, int64_t e) {
                while (e > a && py_space((unsigned char)T[e - 1])) --e;
                return (int32_t)(e - a);
            };
            C.s0[r] = starts[k + 1]; C.sl[r] = stripped(starts[k + 1], line_end(k + 1));
            C.q0[r] = starts[k + 3]; C.ql[r] = stripped(starts[k + 3], line_end(k + 3));
            // ident.split(' ') -> fields[0].split(':')[4] (tile),
            // fields[1].split(':')[0] (read direction); the line keeps its '\n'
            const char *h = T.data() + ha;
            const int64_t hn = he - ha;
            int64_t sp = 0;
            while (sp < hn && h[sp] != ' ') ++sp;
            if (sp >= hn) { bad[t] = 1; bad_rec[t] = r; break; }
            int64_t f = 0, colon = 0;
            while (f < sp && colon < 4) { if (h[f] == ':') ++colon; ++f; }
            if (colon < 4) { bad[t] = 2; bad_rec[t] = r; break; }
            int64_t g = f;
            while (g < sp && h[g] != ':') ++g;
            const std::string tl(h + f, (size_t)(g - f));
            int64_t d = sp + 1, de = d;
            while (de < hn && h[de] != ' ' && h[de] != ':') ++de;
            const bool fwd = de - d == 1 && h[d] == '1';
            C.sign[r] = fwd ? 1 : -1;
            auto it = tiles.find(tl);
            C.tile[r] = it == tiles.end() ? -1 : it->second;
        }
    });
    for (int t = 0; t < nt; ++t)
        if (bad[t]) {
            set_error(bad[t] == 1 ? "censor: header of record %lld has no space (ValueError)"
                                  : "censor: header of record %lld has no tile field (IndexError)",
                      (long long)(bad_rec[t] + 1 + C.rec_base));
            return -3;
        }
    return 0;
}

static int censor_run(Ctx &c, CensorState &C, CensorState &D, int n_bad,
                      const char *const *tiles, const int32_t *cycles)
{
    const int64_t nr = (int64_t)C.h0.size();
    C.keep.assign(2 * (size_t)nr, 0);
    C.base_count = C.score_sum = 0;
    if (nr == 0) return 0;
    // bad-cycle bitmaps per bad tile id, over the cycles of this piece's reads
    std::unordered_map<std::string, int> tid;
    for (int k = 0; k < n_bad; ++k) tid.emplace(tiles[k], (int)tid.size());
    int maxc = 1;
    for (int64_t r = 0; r < nr; ++r) maxc = std::max(maxc, std::max(C.sl[r], C.ql[r]));
    const int words = (2 * maxc + 1 + 31) / 32;
    std::vector<uint32_t> bm((size_t)std::max(1, (int)tid.size()) * words, 0u);
    for (int k = 0; k < n_bad; ++k) {
        const int c0 = cycles[k];
        if (c0 < -maxc || c0 > maxc) continue;
        const int b = c0 + maxc;
        bm[(size_t)tid[tiles[k]] * words + (b >> 5)] |= 1u << (b & 31);
    }
    hipStream_t s = c.stream;
    int st = 0;
    auto H = [&](hipError_t e, const char *what) {
        if (e != hipSuccess && !st) st = hip_fail(e, what);
        return st == 0;
    };
    if ((int64_t)C.text.size() + 1 > D.cap_text) {
        hipFree(D.d_text);
        D.d_text = nullptr;
        D.cap_text = (int64_t)C.text.size() + 1;
        H(hipMalloc(&D.d_text, D.cap_text), "hipMalloc text");
    }
    if (nr > D.cap_rec) {
        hipFree(D.d_s0); hipFree(D.d_q0); hipFree(D.d_sl); hipFree(D.d_ql);
        hipFree(D.d_tile); hipFree(D.d_sign); hipFree(D.d_keep);
        D.cap_rec = nr;
        H(hipMalloc(&D.d_s0, 8 * nr), "hipMalloc");
        H(hipMalloc(&D.d_q0, 8 * nr), "hipMalloc");
        H(hipMalloc(&D.d_sl, 4 * nr), "hipMalloc");
        H(hipMalloc(&D.d_ql, 4 * nr), "hipMalloc");
        H(hipMalloc(&D.d_tile, 4 * nr), "hipMalloc");
        H(hipMalloc(&D.d_sign, 4 * nr), "hipMalloc");
        H(hipMalloc(&D.d_keep, 8 * nr), "hipMalloc");
    }
    if ((int64_t)bm.size() > D.cap_bad) {
        hipFree(D.d_bad);
        D.cap_bad = (int64_t)bm.size();
        H(hipMalloc(&D.d_bad, 4 * bm.size()), "hipMalloc");
    }
    if (!D.d_sums) H(hipMalloc(&D.d_sums, 16), "hipMalloc");
    if (st) { censor_free_device(D); return st; }
    H(hipMemcpyAsync(D.d_text, C.text.data(), C.text.size(), hipMemcpyHostToDevice, s), "H2D");
    H(hipMemcpyAsync(D.d_s0, C.s0.data(), 8 * nr, hipMemcpyHostToDevice, s), "H2D");
    H(hipMemcpyAsync(D.d_q0, C.q0.data(), 8 * nr, hipMemcpyHostToDevice, s), "H2D");
    H(hipMemcpyAsync(D.d_sl, C.sl.data(), 4 * nr, hipMemcpyHostToDevice, s), "H2D");
    H(hipMemcpyAsync(D.d_ql, C.ql.data(), 4 * nr, hipMemcpyHostToDevice, s), "H2D");
    H(hipMemcpyAsync(D.d_tile, C.tile.data(), 4 * nr, hipMemcpyHostToDevice, s), "H2D");
    H(hipMemcpyAsync(D.d_sign, C.sign.data(), 4 * nr, hipMemcpyHostToDevice, s), "H2D");
    H(hipMemcpyAsync(D.d_bad, bm.data(), 4 * bm.size(), hipMemcpyHostToDevice, s), "H2D");
    H(hipMemsetAsync(D.d_sums, 0, 16, s), "memset");
    CensorArgs a{D.d_text, D.d_s0, D.d_q0, D.d_sl, D.d_ql, D.d_tile, D.d_sign, nr, D.d_bad, maxc,
                 words, D.d_keep, D.d_sums};
    int64_t blocks = (nr + 3) / 4;
    if (blocks > 256 * 64) blocks = 256 * 64;
    if (!st) {
        const int pk = prof_begin(c, "k_censor");
        hipLaunchKernelGGL(k_censor, dim3((unsigned)blocks), dim3(256), 0, s, a);
        prof_end(c, pk);
        H(hipGetLastError(), "k_censor");
    }
    unsigned long long sums[2] = {0, 0};
    H(hipMemcpyAsync(&C.text[0], D.d_text, C.text.size(), hipMemcpyDeviceToHost, s), "D2H");
    H(hipMemcpyAsync(C.keep.data(), D.d_keep, 8 * nr, hipMemcpyDeviceToHost, s), "D2H");
    H(hipMemcpyAsync(sums, D.d_sums, 16, hipMemcpyDeviceToHost, s), "D2H");
    H(hipStreamSynchronize(s), "sync");
    if (st) return st;
    prof_flush(c);
    C.score_sum = (long long)sums[0];
    C.base_count = (long long)sums[1];
    return 0;
}

static void censor_write(CensorState &C)
{
    const int64_t nr = (int64_t)C.h0.size();
    const int nt = s2a_threads();
    std::vector<std::string> piece(nt);
    cz_parallel(nt, [&](int t) {
        std::string &o = piece[t];
        for (int64_t r = nr * t / nt; r < nr * (t + 1) / nt; ++r) {
            o.append(C.text, (size_t)C.h0[r], (size_t)C.hl[r]);
            o.append(C.text, (size_t)C.s0[r], (size_t)C.keep[2 * r]);
            o.push_back('\n');
            o.append(C.text, (size_t)C.o0[r], (size_t)C.ol[r]);
            o.append(C.text, (size_t)C.q0[r], (size_t)C.keep[2 * r + 1]);
            o.push_back('\n');
        }
    });
    size_t total = 0;
    for (auto &p : piece) total += p.size();
    C.out.clear();
    C.out.reserve(total);
    for (auto &p : piece) C.out += p;
}

// One piece of whole records: split, censor on the device, rewrite, deflate;
// the output and the sums go to C.
static int censor_piece(Ctx &c, CensorState &C, std::string &&text,
                        const std::unordered_map<std::string, int> &tid, int n_bad,
                        const char *const *tiles, const int32_t *cycles, int dst_gzip)
{
    CensorState P;
    P.text.swap(text);
    P.rec_base = C.rec_base;
    if (int st = split_records(P, tid)) return st;
    C.rec_base += (int64_t)P.h0.size();
    auto t0 = std::chrono::steady_clock::now();
    if (int st = censor_run(c, P, C, n_bad, tiles, cycles)) return st;
    C.t_device += std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    censor_write(P);
    std::string().swap(P.text);
    if (dst_gzip) {
        std::string z;
        if (int st = gzip_parallel(P.out, z, 1)) return st;
        C.out += z;
    } else {
        C.out += P.out;
    }
    C.base_count += P.base_count;
    C.score_sum += P.score_sum;
    return 0;
}

// Streaming inflate: a producer thread inflates the gzip input (multi-member)
// into ~32 MB chunks while the caller censors the records of the chunks
// already there (serial inflate is this stage's bound).
struct InflateQueue {
    std::mutex m;
    std::condition_variable cv;
    std::deque<std::string> q;
    bool done = false;
    int err = 0;
    std::string msg;
};

static void inflate_producer(const uint8_t *src, int64_t len, InflateQueue &Q)
{
    const size_t chunk = 32u << 20;
    auto push = [&](std::string &&piece) {
        std::unique_lock<std::mutex> lk(Q.m);
        Q.cv.wait(lk, [&] { return Q.q.size() < 4; });
        Q.q.push_back(std::move(piece));
        Q.cv.notify_all();
    };
    auto finish = [&](int err, const char *msg) {
        std::lock_guard<std::mutex> lk(Q.m);
        Q.err = err;
        if (msg) Q.msg = msg;
        Q.done = true;
        Q.cv.notify_all();
    };
    if (len == 0) { finish(0, nullptr); return; }
    z_stream z{};
    if (inflateInit2(&z, 15 + 32) != Z_OK) { finish(1, "censor: zlib init"); return; }
    std::string cur;
    cur.reserve(chunk + (4u << 20));
    std::vector<char> buf(4u << 20);
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
        z.next_out = (Bytef *)buf.data();
        z.avail_out = (uInt)buf.size();
        const int st = inflate(&z, Z_NO_FLUSH);
        cur.append(buf.data(), buf.size() - z.avail_out);
        if (cur.size() >= chunk) {
            push(std::move(cur));
            cur = std::string();
            cur.reserve(chunk + (4u << 20));
        }
        if (st == Z_STREAM_END) {
            ended = true;
            if (z.avail_in == 0 && pos >= len) break;
            inflateReset(&z);          // GzipFile reads concatenated members
            ended = false;
            continue;
        }
        if (st != Z_OK && !(st == Z_BUF_ERROR && z.avail_in == 0)) {
            inflateEnd(&z);
            finish(1, "censor: not a valid gzip stream");
            return;
        }
    }
    inflateEnd(&z);
    if (!ended) { finish(1, "censor: truncated gzip stream"); return; }
    if (!cur.empty()) push(std::move(cur));
    finish(0, nullptr);
}

// end of the last whole record (4 lines) in t, from its start
static size_t last_record_end(const std::string &t)
{
    size_t cut = 0, at = 0;
    int lines = 0;
    for (;;) {
        const void *nl = memchr(t.data() + at, '\n', t.size() - at);
        if (!nl) break;
        at = (size_t)((const char *)nl - t.data()) + 1;
        if (++lines == 4) { lines = 0; cut = at; }
    }
    return cut;
}

}  // namespace mh

using namespace mh;

extern "C" int mh_censor_fastq(mh_ctx *ctx, const uint8_t *src, int64_t len, int src_gzip,
                               int n_bad, const char *const *tiles, const int32_t *cycles,
                               int dst_gzip, int64_t *base_count, int64_t *score_sum)
{
    if (!ctx || (len && !src) || len < 0 || n_bad < 0 || (n_bad && (!tiles || !cycles))) return -3;
    Ctx &c = *ctx_of(ctx);
    MH_HIP(hipSetDevice(c.device));
    if (!c.censor) c.censor = new CensorState();
    CensorState &C = *c.censor;
    C.out.clear();
    C.base_count = C.score_sum = 0;
    C.rec_base = 0;
    C.t_host_in = C.t_device = C.t_host_out = 0;
    std::unordered_map<std::string, int> tid;
    for (int k = 0; k < n_bad; ++k) tid.emplace(tiles[k], (int)tid.size());
    auto t0 = std::chrono::steady_clock::now();
    int pieces = 0;
    if (!src_gzip) {
        std::string text((const char *)src, (size_t)len);
        if (len) {
            if (int st = censor_piece(c, C, std::move(text), tid, n_bad, tiles, cycles, dst_gzip))
                return st;
            ++pieces;
        }
    } else if (gunzip_fast_available()) {
        // libdeflate decodes the whole file faster than the streaming zlib
        // producer below can overlap it with the rest
        std::string text, why;
        if (gunzip_buffer(src, len, text, why)) {
            set_error("censor: %s", why.c_str());
            return -3;
        }
        C.t_host_in = std::chrono::duration<double, std::milli>(
                          std::chrono::steady_clock::now() - t0).count();
        if (!text.empty()) {
            if (int st = censor_piece(c, C, std::move(text), tid, n_bad, tiles, cycles, dst_gzip))
                return st;
            ++pieces;
        }
    } else {
        InflateQueue Q;
        std::thread producer(inflate_producer, src, len, std::ref(Q));
        std::string carry;
        int st = 0;
        for (;;) {
            std::string chunk;
            bool last = false;
            {
                std::unique_lock<std::mutex> lk(Q.m);
                Q.cv.wait(lk, [&] { return !Q.q.empty() || Q.done; });
                if (!Q.q.empty()) {
                    chunk = std::move(Q.q.front());
                    Q.q.pop_front();
                    Q.cv.notify_all();
                } else {
                    last = true;
                    if (Q.err) {
                        set_error("%s", Q.msg.c_str());
                        st = -3;
                    }
                }
            }
            if (st) break;
            if (last) {
                C.t_host_in = std::chrono::duration<double, std::milli>(
                                  std::chrono::steady_clock::now() - t0).count();
                // a trailing partial record (or one without its last newline)
                if (!carry.empty()) {
                    st = censor_piece(c, C, std::move(carry), tid, n_bad, tiles, cycles, dst_gzip);
                    ++pieces;
                }
                break;
            }
            carry += chunk;
            std::string().swap(chunk);
            const size_t cut = last_record_end(carry);
            if (cut == 0) continue;
            std::string rest(carry, cut);
            carry.resize(cut);
            st = censor_piece(c, C, std::move(carry), tid, n_bad, tiles, cycles, dst_gzip);
            ++pieces;
            carry.swap(rest);
            if (st) break;
        }
        if (st) {
            // drain the producer before leaving
            {
                std::unique_lock<std::mutex> lk(Q.m);
                Q.q.clear();
                Q.cv.notify_all();
            }
            for (;;) {
                std::unique_lock<std::mutex> lk(Q.m);
                if (Q.done) break;
                Q.cv.wait(lk, [&] { return !Q.q.empty() || Q.done; });
                Q.q.clear();
                Q.cv.notify_all();
            }
            producer.join();
            C.out.clear();
            return st;
        }
        producer.join();
    }
    if (!pieces && dst_gzip) {
        // an empty FASTQ still makes one (empty) gzip member
        if (int st = gzip_parallel(std::string(), C.out, 1)) return st;
    }
    const double total = std::chrono::duration<double, std::milli>(
                             std::chrono::steady_clock::now() - t0).count();
    if (!src_gzip) C.t_host_in = 0;
    if (!C.t_host_in) C.t_host_in = 0;
    C.t_host_out = total - C.t_host_in;
    if (base_count) *base_count = C.base_count;
    if (score_sum) *score_sum = C.score_sum;
    return 0;
}

extern "C" int mh_censor_output(mh_ctx *ctx, char *buf, size_t cap, size_t *used)
{
    if (!ctx || !used) return -3;
    Ctx &c = *ctx_of(ctx);
    if (!c.censor) { set_error("mh_censor_output: no censor results"); return -3; }
    CensorState &C = *c.censor;
    *used = C.out.size();
    if (!buf) return 0;
    if (cap < C.out.size()) { set_error("mh_censor_output: buffer too small"); return -2; }
    memcpy(buf, C.out.data(), C.out.size());
    std::string().swap(C.out);
    return 0;
}

extern "C" int mh_censor_timing(mh_ctx *ctx, double *ms3)
{
    if (!ctx || !ms3) return -3;
    Ctx &c = *ctx_of(ctx);
    if (!c.censor) { set_error("mh_censor_timing: no censor results"); return -3; }
    ms3[0] = c.censor->t_host_in;
    ms3[1] = c.censor->t_device;
    ms3[2] = c.censor->t_host_out;
    return 0;
}
