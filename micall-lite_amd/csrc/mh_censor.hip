// mh_censor.hip -- censor_fastq.censor (micall/core/censor_fastq.py:32-102)
// on gfx950, behind mh_censor_fastq / mh_censor_staged / mh_censor_output /
// mh_censor_write:
//   host      the FASTQ text: gunzipped from a buffer (libdeflate, else
//             zlib) or taken from a staged FASTQ (mh_fastq_open_part: the
//             file mmap'd, its gzip members inflated in parallel), into a
//             buffer that is not zero-filled; line starts found in parallel
//             (memchr, two passes: counts, then positions); records parsed
//             in parallel, tile + read direction from each header exactly as
//             :59-63 parse them, bad (tile, cycle) set from the caller
//   k_censor  one wave64 per read: the bases / qualities of bad cycles
//             become 'N' / '#' in place, the trailing run of bad cycles is
//             dropped (the reference only flushes pending Ns before a good
//             cycle, :66-74, :78-90), and every quality score is summed for
//             the summary (:80-82) -- per-block sums, one atomic per block
//   host      records rewritten (header and '+' lines verbatim) and, for
//             gzip output, compressed, in blocks of ~8 MB of records on
//             every host thread (one gzip member per block: the member
//             boundaries depend on the input only, not on the thread count);
//             the output is written with pwrite (mh_censor_write) or copied
//             out (mh_censor_output)
#include <sys/types.h>
#include <unistd.h>
#include <zlib.h>

#include <algorithm>
#include <atomic>
#include <cerrno>
#include <chrono>
#include <cstring>
#include <exception>
#include <functional>
#include <memory>
#include <mutex>
#include <string>
#include <string_view>
#include <system_error>
#include <thread>
#include <unordered_map>
#include <vector>

#include "mh_fastq.h"
#include "mh_gunzip.h"
#include "mh_internal.h"

namespace mh {

int s2a_threads();   // mh_s2a_host.cpp: host worker count

struct CensorState {
    TextBuf text;                           // the FASTQ (censored in place)
    // per record: line starts (header, seq, '+', qual); the header line is
    // [h0, s0), the '+' line [o0, q0), both with their newline
    std::vector<int64_t> h0, s0, o0, q0;
    std::vector<int32_t> sl, ql;            // seq / qual lengths, trailing whitespace stripped
    std::vector<int32_t> tile, sign;        // tile id (-1: no bad cycle) / +1, -1
    std::vector<int32_t> keep;              // 2 per record: kept seq / qual length
    int64_t base_count = 0, score_sum = 0;
    TextBuf out;                            // the censored file (gzip members or text)
    // set: the blocks are written to sink_fd from sink_pos as they are made
    // (mh_censor_staged_write) instead of collected in out
    int sink_fd = -1;
    int64_t sink_pos = 0;
    int sink_err = 0;
    double t_host_in = 0, t_device = 0, t_host_out = 0;
    // device buffers, grown on demand and kept between calls
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

// fn(t) on nt threads; the first exception a worker throws (an allocation
// failure) is rethrown here once every worker has ended
static void cz_parallel(int nt, const std::function<void(int)> &fn)
{
    if (nt <= 1) { fn(0); return; }
    std::exception_ptr err;
    std::mutex mu;
    auto guarded = [&](int t) {
        try {
            fn(t);
        } catch (...) {
            std::lock_guard<std::mutex> lk(mu);
            if (!err) err = std::current_exception();
        }
    };
    std::vector<std::thread> th;
    try {
        for (int t = 1; t < nt; ++t) th.emplace_back(guarded, t);
    } catch (const std::system_error &) {   // no more threads: the rest run here
        for (int t = (int)th.size() + 1; t < nt; ++t) guarded(t);
    }
    guarded(0);
    for (auto &x : th) x.join();
    if (err) std::rethrow_exception(err);
}

void censor_free(Ctx &c)
{
    if (c.censor) censor_free_device(*c.censor);
    delete c.censor;
    c.censor = nullptr;
}

static double ms_since(std::chrono::steady_clock::time_point t0)
{
    return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
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
static inline bool py_space(unsigned char c)
{
    return c == ' ' || (c >= 9 && c <= 13) || (c >= 0x1c && c <= 0x1f);
}

using TileMap = std::unordered_map<std::string_view, int>;

// records of the FASTQ text: 4 lines each (itertools.zip_longest, :57)
static int split_records(CensorState &C, const TileMap &tiles)
{
    const char *T = C.text.data();
    const int64_t n = (int64_t)C.text.size();
    const int nt = std::max(1, std::min<int>(s2a_threads(), (int)(n >> 20) + 1));
    // newlines per chunk, then every line start at its place: 0, and the byte
    // after every newline that is not the text's last byte
    std::vector<int64_t> cnt((size_t)nt + 1, 0);
    auto chunk = [&](int t, int64_t &a, int64_t &b) { a = n * t / nt; b = n * (t + 1) / nt; };
    cz_parallel(nt, [&](int t) {
        int64_t a, b, k = 0;
        chunk(t, a, b);
        for (const char *p = T + a, *e = T + b; p < e;) {
            const char *q = (const char *)memchr(p, '\n', (size_t)(e - p));
            if (!q) break;
            ++k;
            p = q + 1;
        }
        cnt[(size_t)t + 1] = k;
    });
    for (int t = 0; t < nt; ++t) cnt[(size_t)t + 1] += cnt[(size_t)t];
    const int64_t nl = n == 0 ? 0 : 1 + cnt[(size_t)nt] - (T[n - 1] == '\n' ? 1 : 0);
    if (nl % 4) {
        set_error("censor: FASTQ has %lld lines, not a multiple of 4", (long long)nl);
        return -3;
    }
    std::unique_ptr<int64_t[]> starts(new int64_t[(size_t)std::max<int64_t>(nl, 1)]);
    if (nl) starts[0] = 0;
    cz_parallel(nt, [&](int t) {
        int64_t a, b, k = 1 + cnt[(size_t)t];
        chunk(t, a, b);
        for (const char *p = T + a, *e = T + b; p < e;) {
            const char *q = (const char *)memchr(p, '\n', (size_t)(e - p));
            if (!q) break;
            const int64_t at = (int64_t)(q - T) + 1;
            if (at < n) starts[(size_t)k++] = at;
            p = q + 1;
        }
    });
    const int64_t nr = nl / 4;
    C.h0.resize(nr); C.s0.resize(nr); C.o0.resize(nr); C.q0.resize(nr);
    C.sl.resize(nr); C.ql.resize(nr); C.tile.resize(nr); C.sign.resize(nr);
    const int rt = std::max(1, std::min<int>(nt, (int)(nr >> 12) + 1));
    std::vector<int> bad((size_t)rt, 0);
    std::vector<int64_t> bad_rec((size_t)rt, -1);
    auto line_end = [&](int64_t k) { return k + 1 < nl ? starts[(size_t)k + 1] : n; };   // after '\n'
    auto stripped = [&](int64_t a, int64_t e) {
        while (e > a && py_space((unsigned char)T[e - 1])) --e;
        return (int32_t)(e - a);
    };
    cz_parallel(rt, [&](int t) {
        for (int64_t r = nr * t / rt; r < nr * (t + 1) / rt; ++r) {
            const int64_t k = 4 * r;
            const int64_t ha = starts[(size_t)k], he = starts[(size_t)k + 1];
            C.h0[r] = ha;
            C.s0[r] = he;
            C.o0[r] = starts[(size_t)k + 2];
            C.q0[r] = starts[(size_t)k + 3];
            C.sl[r] = stripped(he, C.o0[r]);
            C.ql[r] = stripped(C.q0[r], line_end(k + 3));
            // ident.split(' ') -> fields[0].split(':')[4] (tile),
            // fields[1].split(':')[0] (read direction); the line keeps its '\n'
            const char *h = T + ha;
            const int64_t hn = he - ha;
            const char *spp = (const char *)memchr(h, ' ', (size_t)hn);
            if (!spp) { bad[(size_t)t] = 1; bad_rec[(size_t)t] = r; break; }
            const int64_t sp = spp - h;
            int64_t f = 0, colon = 0;
            while (f < sp && colon < 4) { if (h[f] == ':') ++colon; ++f; }
            if (colon < 4) { bad[(size_t)t] = 2; bad_rec[(size_t)t] = r; break; }
            int64_t g = f;
            while (g < sp && h[g] != ':') ++g;
            int64_t d = sp + 1, de = d;
            while (de < hn && h[de] != ' ' && h[de] != ':') ++de;
            C.sign[r] = (de - d == 1 && h[d] == '1') ? 1 : -1;
            auto it = tiles.find(std::string_view(h + f, (size_t)(g - f)));
            C.tile[r] = it == tiles.end() ? -1 : it->second;
        }
    });
    for (int t = 0; t < rt; ++t)
        if (bad[(size_t)t]) {
            set_error(bad[(size_t)t] == 1 ? "censor: header of record %lld has no space (ValueError)"
                                          : "censor: header of record %lld has no tile field (IndexError)",
                      (long long)(bad_rec[(size_t)t] + 1));
            return -3;
        }
    return 0;
}

// k_censor over the records: the text up, censored in place, down again
static int censor_run(Ctx &c, CensorState &C, const TileMap &tid, int n_bad, const char *const *tiles,
                      const int32_t *cycles)
{
    const int64_t nr = (int64_t)C.h0.size();
    C.keep.assign(2 * (size_t)nr, 0);
    C.base_count = C.score_sum = 0;
    if (nr == 0) return 0;
    // bad-cycle bitmaps per bad tile id, over the cycles of the reads
    int maxc = 1;
    for (int64_t r = 0; r < nr; ++r) maxc = std::max(maxc, std::max(C.sl[r], C.ql[r]));
    const int words = (2 * maxc + 1 + 31) / 32;
    std::vector<uint32_t> bm((size_t)std::max(1, (int)tid.size()) * words, 0u);
    for (int k = 0; k < n_bad; ++k) {
        const int c0 = cycles[k];
        if (c0 < -maxc || c0 > maxc) continue;
        const int b = c0 + maxc;
        bm[(size_t)tid.at(std::string_view(tiles[k])) * words + (b >> 5)] |= 1u << (b & 31);
    }
    hipStream_t s = c.stream;
    int st = 0;
    auto H = [&](hipError_t e, const char *what) {
        if (e != hipSuccess && !st) st = hip_fail(e, what);
        return st == 0;
    };
    CensorState &D = C;
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
    H(hipMemcpyAsync(C.text.data(), D.d_text, C.text.size(), hipMemcpyDeviceToHost, s), "D2H");
    H(hipMemcpyAsync(C.keep.data(), D.d_keep, 8 * nr, hipMemcpyDeviceToHost, s), "D2H");
    H(hipMemcpyAsync(sums, D.d_sums, 16, hipMemcpyDeviceToHost, s), "D2H");
    H(hipStreamSynchronize(s), "sync");
    if (st) return st;
    prof_flush(c);
    C.score_sum = (long long)sums[0];
    C.base_count = (long long)sums[1];
    return 0;
}

// The censored records, rewritten (header and '+' lines verbatim, seq and
// qual cut to their kept length, each line ending in '\n') and, for gzip,
// deflated, in blocks of records of about CENSOR_BLOCK input bytes, one gzip
// member per block; the blocks are made by every host thread in turn and
// placed into C.out by their precomputed offsets.
constexpr int64_t CENSOR_BLOCK = (int64_t)8 << 20;

static int censor_emit(CensorState &C, int dst_gzip)
{
    const int64_t nr = (int64_t)C.h0.size();
    const int64_t n = (int64_t)C.text.size();
    std::vector<int64_t> bstart{0};
    for (int64_t r = 0, base = 0; r < nr; ++r) {
        if (C.h0[r] - base >= CENSOR_BLOCK) { bstart.push_back(r); base = C.h0[r]; }
    }
    if (nr > 0) bstart.push_back(nr);
    const int64_t nb = (int64_t)bstart.size() - 1;
    if (nb <= 0) {
        C.out.clear();
        if (dst_gzip) {   // an empty FASTQ still makes one (empty) gzip member
            if (gzip_member("", 0, C.out, 1)) { set_error("censor: deflate failed"); return -2; }
        }
        if (C.sink_fd >= 0 && C.out.size()) {
            const ssize_t w = pwrite(C.sink_fd, C.out.data(), C.out.size(), (off_t)C.sink_pos);
            if (w != (ssize_t)C.out.size()) {
                set_error("censor: write failed (%s)", strerror(errno ? errno : EIO));
                return -4;
            }
            C.sink_pos += w;
            C.out.clear();
        }
        return 0;
    }
    std::vector<TextBuf> part((size_t)nb);
    std::atomic<int64_t> next(0);
    std::atomic<int> err(0);
    const char *T = C.text.data();
    const bool stream = C.sink_fd >= 0;
    // streamed: thread 0 writes the blocks in order as the others finish them
    const int nt = std::max(stream ? 2 : 1, std::min<int>(s2a_threads(), (int)nb + (stream ? 1 : 0)));
    std::unique_ptr<std::atomic<int>[]> done(new std::atomic<int>[(size_t)nb]);
    for (int64_t b = 0; b < nb; ++b) done[b].store(0);
    std::atomic<int> dead(0);   // a block maker failed: the writer stops waiting
    auto write_blocks = [&]() {
        for (int64_t b = 0; b < nb; ++b) {
            while (!done[b].load(std::memory_order_acquire) && !dead) std::this_thread::yield();
            if (dead || err) return;
            const char *p = part[(size_t)b].data();
            size_t left = part[(size_t)b].size();
            while (left > 0) {
                const ssize_t w = pwrite(C.sink_fd, p, left, (off_t)C.sink_pos);
                if (w <= 0) { C.sink_err = errno ? errno : EIO; dead = 1; return; }
                p += w; left -= (size_t)w; C.sink_pos += w;
            }
            part[(size_t)b].release();
        }
    };
    cz_parallel(nt, [&](int t) {
        if (stream && t == 0) { write_blocks(); return; }
        TextBuf raw;
        struct Dead {   // a throw out of a block maker releases the writer
            std::atomic<int> &d;
            bool ok = false;
            ~Dead() { if (!ok) d = 1; }
        } guard{dead};
        for (int64_t b; !dead && (b = next.fetch_add(1)) < nb;) {
            const int64_t r0 = bstart[(size_t)b], r1 = bstart[(size_t)b + 1];
            const int64_t in_end = r1 < nr ? C.h0[r1] : n;
            TextBuf &dst = dst_gzip ? raw : part[(size_t)b];
            dst.resize((size_t)(in_end - C.h0[r0] + 2 * (r1 - r0)));
            char *o = dst.data();
            for (int64_t r = r0; r < r1; ++r) {
                const size_t hl = (size_t)(C.s0[r] - C.h0[r]), pl = (size_t)(C.q0[r] - C.o0[r]);
                const size_t ks = (size_t)C.keep[2 * r], kq = (size_t)C.keep[2 * r + 1];
                memcpy(o, T + C.h0[r], hl); o += hl;
                memcpy(o, T + C.s0[r], ks); o += ks;
                *o++ = '\n';
                memcpy(o, T + C.o0[r], pl); o += pl;
                memcpy(o, T + C.q0[r], kq); o += kq;
                *o++ = '\n';
            }
            dst.resize((size_t)(o - dst.data()));
            if (dst_gzip && gzip_member(raw.data(), raw.size(), part[(size_t)b], 1)) { err = 1; dead = 1; }
            done[b].store(1, std::memory_order_release);
        }
        guard.ok = true;
    });
    if (err) { set_error("censor: deflate failed"); return -2; }
    if (stream) {
        if (C.sink_err) { set_error("censor: write failed (%s)", strerror(C.sink_err)); return -4; }
        return 0;
    }
    std::vector<size_t> off((size_t)nb + 1, 0);
    for (int64_t b = 0; b < nb; ++b) off[(size_t)b + 1] = off[(size_t)b] + part[(size_t)b].size();
    C.out.resize(off[(size_t)nb]);
    next = 0;
    cz_parallel(nt, [&](int) {
        for (int64_t b; (b = next.fetch_add(1)) < nb;) {
            memcpy(C.out.data() + off[(size_t)b], part[(size_t)b].data(), part[(size_t)b].size());
            part[(size_t)b].release();
        }
    });
    return 0;
}

// one FASTQ text (moved into C.text) through split, k_censor and the rewrite
static int censor_text(Ctx &c, CensorState &C, int n_bad, const char *const *tiles,
                       const int32_t *cycles, int dst_gzip, std::chrono::steady_clock::time_point t0)
{
    TileMap tid;
    for (int k = 0; k < n_bad; ++k) tid.emplace(std::string_view(tiles[k]), (int)tid.size());
    if (int st = split_records(C, tid)) return st;
    C.t_host_in = ms_since(t0);
    const auto t1 = std::chrono::steady_clock::now();
    if (int st = censor_run(c, C, tid, n_bad, tiles, cycles)) return st;
    C.t_device = ms_since(t1);
    const auto t2 = std::chrono::steady_clock::now();
    const int st = censor_emit(C, dst_gzip);
    C.t_host_out = ms_since(t2);
    // the text and record tables are not needed past the call: freed on a
    // detached thread (a GB-sized free is tens of ms)
    auto *old = new TextBuf();
    old->swap(C.text);
    std::thread([old]() { delete old; }).detach();
    return st;
}

// censor_text with an allocation failure (here or in a worker) as status -2
static int censor_text_guarded(Ctx &c, CensorState &C, int n_bad, const char *const *tiles,
                               const int32_t *cycles, int dst_gzip,
                               std::chrono::steady_clock::time_point t0)
{
    try {
        return censor_text(c, C, n_bad, tiles, cycles, dst_gzip, t0);
    } catch (const std::exception &e) {
        set_error("censor: out of memory (%s)", e.what());
        return -2;
    }
}

static bool censor_args_ok(mh_ctx *ctx, int n_bad, const char *const *tiles, const int32_t *cycles)
{
    return ctx && n_bad >= 0 && (!n_bad || (tiles && cycles));
}

}  // namespace mh

using namespace mh;

extern "C" int mh_censor_fastq(mh_ctx *ctx, const uint8_t *src, int64_t len, int src_gzip,
                               int n_bad, const char *const *tiles, const int32_t *cycles,
                               int dst_gzip, int64_t *base_count, int64_t *score_sum)
{
    if (!censor_args_ok(ctx, n_bad, tiles, cycles) || (len && !src) || len < 0) return -3;
    Ctx &c = *ctx_of(ctx);
    MH_HIP(hipSetDevice(c.device));
    if (!c.censor) c.censor = new CensorState();
    CensorState &C = *c.censor;
    C.out.clear();
    C.base_count = C.score_sum = 0;
    C.t_host_in = C.t_device = C.t_host_out = 0;
    const auto t0 = std::chrono::steady_clock::now();
    if (src_gzip) {
        std::string why;
        if (gunzip_buffer(src, len, C.text, why)) {
            set_error("censor: %s", why.c_str());
            return -3;
        }
    } else {
        try {
            C.text.assign((const char *)src, (size_t)len);
        } catch (const std::exception &) {
            set_error("censor: out of memory");
            return -2;
        }
    }
    if (int st = censor_text_guarded(c, C, n_bad, tiles, cycles, dst_gzip, t0)) { C.out.clear(); return st; }
    if (base_count) *base_count = C.base_count;
    if (score_sum) *score_sum = C.score_sum;
    return 0;
}

extern "C" int mh_censor_staged(mh_ctx *ctx, mh_fastq *fq, int n_bad, const char *const *tiles,
                                const int32_t *cycles, int dst_gzip, int64_t *out_bytes,
                                int64_t *base_count, int64_t *score_sum)
{
    if (!censor_args_ok(ctx, n_bad, tiles, cycles) || !fq) return -3;
    Ctx &c = *ctx_of(ctx);
    MH_HIP(hipSetDevice(c.device));
    if (!c.censor) c.censor = new CensorState();
    CensorState &C = *c.censor;
    C.out.clear();
    C.base_count = C.score_sum = 0;
    C.t_host_in = C.t_device = C.t_host_out = 0;
    const auto t0 = std::chrono::steady_clock::now();
    TextBuf text = take_fastq_text(fq);
    C.text.swap(text);
    if (int st = censor_text_guarded(c, C, n_bad, tiles, cycles, dst_gzip, t0)) { C.out.clear(); return st; }
    if (out_bytes) *out_bytes = (int64_t)C.out.size();
    if (base_count) *base_count = C.base_count;
    if (score_sum) *score_sum = C.score_sum;
    return 0;
}

extern "C" int mh_censor_staged_write(mh_ctx *ctx, mh_fastq *fq, int n_bad, const char *const *tiles,
                                      const int32_t *cycles, int dst_gzip, int fd, int64_t offset,
                                      int64_t *written, int64_t *base_count, int64_t *score_sum)
{
    if (!censor_args_ok(ctx, n_bad, tiles, cycles) || !fq || fd < 0 || offset < 0) return -3;
    Ctx &c = *ctx_of(ctx);
    MH_HIP(hipSetDevice(c.device));
    if (!c.censor) c.censor = new CensorState();
    CensorState &C = *c.censor;
    C.out.clear();
    C.base_count = C.score_sum = 0;
    C.t_host_in = C.t_device = C.t_host_out = 0;
    C.sink_fd = fd;
    C.sink_pos = offset;
    C.sink_err = 0;
    const auto t0 = std::chrono::steady_clock::now();
    TextBuf text = take_fastq_text(fq);
    C.text.swap(text);
    const int st = censor_text_guarded(c, C, n_bad, tiles, cycles, dst_gzip, t0);
    C.sink_fd = -1;
    if (st) return st;
    if (written) *written = C.sink_pos - offset;
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
    if (C.out.size()) memcpy(buf, C.out.data(), C.out.size());
    C.out.release();
    return 0;
}

extern "C" int mh_censor_write(mh_ctx *ctx, int fd, int64_t offset, int64_t *written)
{
    if (!ctx || fd < 0 || offset < 0) return -3;
    Ctx &c = *ctx_of(ctx);
    if (!c.censor) { set_error("mh_censor_write: no censor results"); return -3; }
    CensorState &C = *c.censor;
    const char *p = C.out.data();
    size_t left = C.out.size();
    int64_t pos = offset;
    while (left > 0) {
        const ssize_t w = pwrite(fd, p, left, (off_t)pos);
        if (w <= 0) {
            set_error("mh_censor_write: write failed (%s)", strerror(errno ? errno : EIO));
            return -4;
        }
        p += w; left -= (size_t)w; pos += w;
    }
    if (written) *written = pos - offset;
    C.out.release();
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
