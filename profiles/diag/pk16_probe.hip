// profiles/diag/pk16_probe.hip -- would k_dp's row recurrence be faster with
// two extensions' cells packed as int16 in each lane (VERDICT r03, next round
// item 5: v_pk_add_i16 / v_pk_max_i16, one v_mov_b32_dpp per lane move)?
//
// Two DP cores over the same synthetic local-mode extensions (251 rows, the
// library's nibble score encoding, bowtie2's +-15 band = 31 live lanes of a
// 32-lane half), timed and cross-checked:
//   k_row32  the r03 k_dp row (dp_row_gap<LOCAL>, mh_map.hip): one cell per
//            lane, two extensions per wave, row values shifted by exD * lane
//            with a +2^20 bias, 4 traceback sign bits per cell packed 8 rows
//            per u32 in LDS, best cell as (H << 10 | 1023 - row) max
//   k_row16  the same recurrence on int16 pairs: lane half 0 holds extension
//            w and half 1 extension w + 2, so a wave runs four; every lane
//            move is a v_mov_b32_dpp of both halves, arithmetic v_pk_*_i16
//            (saturating where a dead-lane constant is added); the sign bits
//            of both halves go to two accumulators (8 rows each), the best
//            cell as packed (H, row) updated with a bit-select
// Both write every extension's best (score, row, lane) and, in the check
// pass, every cell's traceback nibble in one canonical layout; the host
// compares them.  Timing: hipEvents around each kernel, best of several
// launches, ns per cell = time / (extensions * rows * 32).
//   hipcc --offload-arch=gfx950 -O3 -o pk16_probe pk16_probe.hip && ./pk16_probe [extensions]
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#define CHECK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e_)); exit(1); } } while (0)

constexpr int M = 251, ROWS = 256, GBAR = 4, XC = 16, HB = 15;
constexpr int OEI = 13, EXI = 3, OED = 13, EXD = 3;
constexpr int BIAS32 = 1 << 20;
constexpr int BIAS16 = 1 << 13;
constexpr int HUGE_NEG = -(1 << 24);

template <int CTRL>
__device__ __forceinline__ int dppz(int v) { return __builtin_amdgcn_update_dpp(0, v, CTRL, 0xF, 0xF, true); }
constexpr int ROW_SHR1 = 0x111, ROW_SHR2 = 0x112, ROW_SHR4 = 0x114, ROW_SHR8 = 0x118,
              WAVE_SHL1 = 0x130, WAVE_SHR1 = 0x138;
__device__ __forceinline__ int imax(int a, int b) { return a > b ? a : b; }

// extension e: tab[e][row] (score nibbles of the read base against ref codes
// 0..4 at 4 * code), refw[e][x] (ref code * 4 of diagonal d0 + x)
struct Ext {
    const uint32_t *tab;    // [n][ROWS]
    const uint8_t *refw;    // [n][ROWS + 64]
    int n;
};

// ------------------------------------------------------------------ int32 rows
__device__ __forceinline__ int scan_max32(int x)
{
    x = imax(x, dppz<ROW_SHR1>(x));
    x = imax(x, dppz<ROW_SHR2>(x));
    x = imax(x, dppz<ROW_SHR4>(x));
    x = imax(x, dppz<ROW_SHR8>(x));
    asm volatile("s_nop 1\n\tv_max_i32_dpp %0, %0, %0 row_bcast:15 row_mask:0xa bank_mask:0xf\n\ts_nop 1"
                 : "+v"(x));
    return x;
}

__device__ __forceinline__ uint32_t push_sign(uint32_t acc, int d) { return __builtin_amdgcn_alignbit(acc, (uint32_t)d, 31u); }

struct K32 { int mexI, dIE, cF, floor; };

__device__ __forceinline__ void row32(uint32_t tbv, int rc, int &Hp, int &Ep, uint32_t &bestKey, int ci,
                                      const K32 &K, uint32_t &acc)
{
    const int nib = (int)__builtin_amdgcn_ubfe(tbv, (uint32_t)rc, 4);
    const int Hd = Hp + nib - 8;
    const int hc = Hp + K.dIE;
    const int q = imax(Ep, hc);
    const int E = dppz<WAVE_SHL1>(q) + K.mexI;
    acc = push_sign(acc, hc - Ep);
    int H1 = imax(Hd, E);
    H1 = imax(H1, K.floor);
    const int P = scan_max32(H1);
    const int F = dppz<WAVE_SHR1>(P) + K.cF;
    const int H = imax(H1, F);
    acc = push_sign(acc, H1 - P);
    acc = push_sign(acc, Hd - H);
    acc = push_sign(acc, E - H);
    const uint32_t key = ((uint32_t)H << 10) | (uint32_t)ci;
    bestKey = bestKey > key ? bestKey : key;
    Hp = H;
    Ep = E;
}

template <bool CHECKBITS>
__global__ __launch_bounds__(256) void k_row32(Ext X, int *best, uint8_t *nibs)
{
    __shared__ uint32_t bits[4][(ROWS / 8) * 64];
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const int h = lane >> 5, kl = lane & 31;
    const bool live = kl >= XC - HB && kl <= XC + HB;
    K32 K;
    K.mexI = (live && kl < XC + HB) ? -(EXI + EXD) : HUGE_NEG;
    K.dIE = EXI - OEI;
    K.cF = live ? -(OED - EXD) : HUGE_NEG;
    K.floor = live ? BIAS32 + EXD * lane : 0;
    for (int pair = blockIdx.x * 4 + wv; 2 * pair + 1 < X.n; pair += gridDim.x * 4) {
        const int e = 2 * pair + h;
        const uint32_t *tab = X.tab + (size_t)e * ROWS;
        const uint8_t *refw = X.refw + (size_t)e * (ROWS + 64) + kl;
        int Hp = K.floor, Ep = 0;
        uint32_t bestKey = 0;
        for (int i0 = 0; i0 < M; i0 += 8) {
            uint32_t acc = 0;
#pragma unroll
            for (int t = 0; t < 8; ++t) {
                const int i = i0 + t;
                const uint32_t tbv = tab[i];
                const int rc = refw[i];
                if (i >= M) acc <<= 4;
                else if (i >= GBAR && i < M - GBAR) row32(tbv, rc, Hp, Ep, bestKey, 1023 - i, K, acc);
                else {   // no gap window: diagonal only
                    int H = Hp + (int)__builtin_amdgcn_ubfe(tbv, (uint32_t)rc, 4) - 8;
                    H = imax(H, K.floor);
                    const uint32_t key = ((uint32_t)H << 10) | (uint32_t)(1023 - i);
                    bestKey = bestKey > key ? bestKey : key;
                    acc <<= 4;
                    Hp = H;
                    Ep = 0;
                }
            }
            bits[wv][(i0 >> 3) * 64 + lane] = acc;
            if (CHECKBITS) {
                for (int t = 0; t < 8 && i0 + t < M; ++t)
                    nibs[((size_t)e * ROWS + i0 + t) * 32 + kl] = (uint8_t)((acc >> (4 * (7 - t))) & 15);
            }
        }
        best[e * 64 + kl * 2] = live ? (int)(bestKey >> 10) - BIAS32 - EXD * lane : -1;
        best[e * 64 + kl * 2 + 1] = 1023 - (int)(bestKey & 1023u);
        if (lane == 0 && bits[wv][lane] == 0xdeadbeef) best[0] = 0;   // keep the stores
    }
}

// ------------------------------------------------------------------ int16 pairs
typedef short s16x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ s16x2 as2(uint32_t v) { return __builtin_bit_cast(s16x2, v); }
__device__ __forceinline__ uint32_t as1(s16x2 v) { return __builtin_bit_cast(uint32_t, v); }
// plain vector ops (the compiler schedules them): v_pk_add_u16 / v_pk_max_i16 /
// v_pk_add_i16 clamp / v_pk_sub_i16 clamp
__device__ __forceinline__ uint32_t pk_add(uint32_t a, uint32_t b) { return as1(as2(a) + as2(b)); }
__device__ __forceinline__ uint32_t pk_add_sat(uint32_t a, uint32_t b)
{
    return as1(__builtin_elementwise_add_sat(as2(a), as2(b)));
}
__device__ __forceinline__ uint32_t pk_sub_sat(uint32_t a, uint32_t b)
{
    return as1(__builtin_elementwise_sub_sat(as2(a), as2(b)));
}
__device__ __forceinline__ uint32_t pk_max(uint32_t a, uint32_t b)
{
    return as1(__builtin_elementwise_max(as2(a), as2(b)));
}
__device__ __forceinline__ uint32_t pk_sign(uint32_t a) { return as1(as2(a) >> (s16x2)(15)); }
template <int CTRL>
__device__ __forceinline__ uint32_t mvz(uint32_t v) { return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, CTRL, 0xF, 0xF, true); }

__device__ __forceinline__ uint32_t scan_max16(uint32_t x)
{
    x = pk_max(x, mvz<ROW_SHR1>(x));
    x = pk_max(x, mvz<ROW_SHR2>(x));
    x = pk_max(x, mvz<ROW_SHR4>(x));
    x = pk_max(x, mvz<ROW_SHR8>(x));
    // rows 1 and 3 take lane 15 of rows 0 and 2; rows 0 and 2 keep x
    const uint32_t b = (uint32_t)__builtin_amdgcn_update_dpp((int)x, (int)x, 0x142, 0xA, 0xF, false);
    return pk_max(x, b);
}

// sign bits of both halves: hi half into accH, lo half into accL
__device__ __forceinline__ void push2(uint32_t &accH, uint32_t &accL, uint32_t d)
{
    accH = __builtin_amdgcn_alignbit(accH, d, 31u);
    accL = __builtin_amdgcn_alignbit(accL, d << 16, 31u);
}

struct K16 { uint32_t mexI, dIE, cF, floor, m8; };

__device__ __forceinline__ void row16(uint32_t nib, uint32_t &Hp, uint32_t &Ep, uint32_t &bestH,
                                      uint32_t &bestR, uint32_t row2, const K16 &K, uint32_t &accH,
                                      uint32_t &accL)
{
    const uint32_t Hd = pk_add(pk_add(Hp, nib), K.m8);
    const uint32_t hc = pk_add(Hp, K.dIE);
    const uint32_t q = pk_max(Ep, hc);
    const uint32_t E = pk_add_sat(mvz<WAVE_SHL1>(q), K.mexI);
    push2(accH, accL, pk_sub_sat(hc, Ep));
    uint32_t H1 = pk_max(Hd, E);
    H1 = pk_max(H1, K.floor);
    const uint32_t P = scan_max16(H1);
    const uint32_t F = pk_add_sat(mvz<WAVE_SHR1>(P), K.cF);
    const uint32_t H = pk_max(H1, F);
    push2(accH, accL, pk_sub_sat(H1, P));
    push2(accH, accL, pk_sub_sat(Hd, H));
    push2(accH, accL, pk_sub_sat(E, H));
    // best cell: a strictly larger H takes this row (the first row keeps a tie)
    const uint32_t gt = pk_sub_sat(bestH, H);             // < 0 where H > bestH
    const uint32_t msk = pk_sign(gt);
    bestR = (row2 & msk) | (bestR & ~msk);
    bestH = pk_max(bestH, H);
    Hp = H;
    Ep = E;
}

__device__ __forceinline__ uint32_t pack2(int lo, int hi) { return ((uint32_t)hi << 16) | ((uint32_t)lo & 0xFFFFu); }

template <bool CHECKBITS>
__global__ __launch_bounds__(256) void k_row16(Ext X, int *best, uint8_t *nibs)
{
    __shared__ uint32_t bits[4][(ROWS / 8) * 64 * 2];
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const int h = lane >> 5, kl = lane & 31;
    const bool live = kl >= XC - HB && kl <= XC + HB;
    const int mexI = (live && kl < XC + HB) ? -(EXI + EXD) : -32768;
    const int cF = live ? -(OED - EXD) : -32768;
    const int floor = live ? BIAS16 + EXD * kl : 0;
    K16 K;
    K.mexI = pack2(mexI, mexI);
    K.dIE = pack2(EXI - OEI, EXI - OEI);
    K.cF = pack2(cF, cF);
    K.floor = pack2(floor, floor);
    K.m8 = pack2(-8, -8);
    // a wave runs extensions 4q + h (lo halves) and 4q + 2 + h (hi halves)
    for (int quad = blockIdx.x * 4 + wv; 4 * quad + 3 < X.n; quad += gridDim.x * 4) {
        const int eA = 4 * quad + h, eB = 4 * quad + 2 + h;
        const uint32_t *tabA = X.tab + (size_t)eA * ROWS, *tabB = X.tab + (size_t)eB * ROWS;
        const uint8_t *refA = X.refw + (size_t)eA * (ROWS + 64) + kl;
        const uint8_t *refB = X.refw + (size_t)eB * (ROWS + 64) + kl;
        uint32_t Hp = K.floor, Ep = 0, bestH = 0, bestR = 0;
        for (int i0 = 0; i0 < M; i0 += 8) {
            uint32_t accH = 0, accL = 0;
#pragma unroll
            for (int t = 0; t < 8; ++t) {
                const int i = i0 + t;
                const uint32_t nA = __builtin_amdgcn_ubfe(tabA[i], (uint32_t)refA[i], 4);
                const uint32_t nB = __builtin_amdgcn_ubfe(tabB[i], (uint32_t)refB[i], 4);
                const uint32_t nib = (nB << 16) | nA;
                const uint32_t row2 = pack2(1023 - i, 1023 - i);
                if (i >= M) { accH <<= 4; accL <<= 4; }
                else if (i >= GBAR && i < M - GBAR) {
                    row16(nib, Hp, Ep, bestH, bestR, row2, K, accH, accL);
                } else {
                    uint32_t H = pk_max(pk_add(pk_add(Hp, nib), K.m8), K.floor);
                    const uint32_t gt = pk_sub_sat(bestH, H);
                    const uint32_t msk = pk_sign(gt);
                    bestR = (row2 & msk) | (bestR & ~msk);
                    bestH = pk_max(bestH, H);
                    accH <<= 4;
                    accL <<= 4;
                    Hp = H;
                    Ep = 0;
                }
            }
            bits[wv][(i0 >> 3) * 128 + 2 * lane] = accL;
            bits[wv][(i0 >> 3) * 128 + 2 * lane + 1] = accH;
            if (CHECKBITS) {
                for (int t = 0; t < 8 && i0 + t < M; ++t) {
                    nibs[((size_t)eA * ROWS + i0 + t) * 32 + kl] = (uint8_t)((accL >> (4 * (7 - t))) & 15);
                    nibs[((size_t)eB * ROWS + i0 + t) * 32 + kl] = (uint8_t)((accH >> (4 * (7 - t))) & 15);
                }
            }
        }
        const int bA = (int)(int16_t)(bestH & 0xFFFF), bB = (int)(int16_t)(bestH >> 16);
        best[eA * 64 + kl * 2] = live ? bA - BIAS16 - EXD * kl : -1;
        best[eA * 64 + kl * 2 + 1] = 1023 - (int)(bestR & 0xFFFF);
        best[eB * 64 + kl * 2] = live ? bB - BIAS16 - EXD * kl : -1;
        best[eB * 64 + kl * 2 + 1] = 1023 - (int)(bestR >> 16);
        if (lane == 0 && bits[wv][lane] == 0xdeadbeef) best[0] = 0;
    }
}

// ------------------------------------------------------------------ host
static uint32_t lcg(uint64_t &s) { s = s * 6364136223846793005ull + 1442695040888963407ull; return (uint32_t)(s >> 33); }

int main(int argc, char **argv)
{
    const int n = argc > 1 ? atoi(argv[1]) : 400000;
    std::vector<uint32_t> tab((size_t)n * ROWS);
    std::vector<uint8_t> refw((size_t)n * (ROWS + 64));
    uint64_t s = 12345;
    for (int e = 0; e < n; ++e) {
        // a reference window and a read drawn from it at diagonal XC with
        // ~10 % substitutions and a few indels (scores like a remap pass)
        uint8_t ref[ROWS + 64];
        for (int x = 0; x < ROWS + 64; ++x) ref[x] = (uint8_t)(lcg(s) & 3);
        int off = XC;
        for (int i = 0; i < ROWS; ++i) {
            const uint32_t r = lcg(s) % 1000;
            if (r < 3 && off < XC + 10) ++off;
            else if (r < 6 && off > XC - 10) --off;
            int b = ref[i + off];
            if (lcg(s) % 100 < 10) b = (b + 1 + lcg(s) % 3) & 3;
            const int q = 2 + (int)(lcg(s) % 39);
            const int mm = 2 + ((q < 40 ? q : 40) * 205 >> 11);
            uint32_t w = 0;
            for (int c = 0; c < 5; ++c) {
                const int sc = c == 4 ? -1 : (c == b ? 2 : -mm);
                w |= (uint32_t)(sc + 8) << (4 * c);
            }
            tab[(size_t)e * ROWS + i] = w;
        }
        for (int x = 0; x < ROWS + 64; ++x) refw[(size_t)e * (ROWS + 64) + x] = (uint8_t)(ref[x] * 4);
    }
    uint32_t *dtab;
    uint8_t *drefw, *dn32, *dn16;
    int *db32, *db16;
    CHECK(hipMalloc(&dtab, tab.size() * 4));
    CHECK(hipMalloc(&drefw, refw.size()));
    CHECK(hipMalloc(&db32, (size_t)n * 64 * 4));
    CHECK(hipMalloc(&db16, (size_t)n * 64 * 4));
    const int ncheck = n < 4096 ? n : 4096;
    CHECK(hipMalloc(&dn32, (size_t)ncheck * ROWS * 32));
    CHECK(hipMalloc(&dn16, (size_t)ncheck * ROWS * 32));
    CHECK(hipMemcpy(dtab, tab.data(), tab.size() * 4, hipMemcpyHostToDevice));
    CHECK(hipMemcpy(drefw, refw.data(), refw.size(), hipMemcpyHostToDevice));
    // check pass on the first extensions: best cells and every traceback nibble
    {
        Ext X{dtab, drefw, ncheck};
        CHECK(hipMemset(dn32, 0, (size_t)ncheck * ROWS * 32));
        CHECK(hipMemset(dn16, 0, (size_t)ncheck * ROWS * 32));
        hipLaunchKernelGGL(k_row32<true>, dim3(256), dim3(256), 0, 0, X, db32, dn32);
        hipLaunchKernelGGL(k_row16<true>, dim3(256), dim3(256), 0, 0, X, db16, dn16);
        CHECK(hipDeviceSynchronize());
        std::vector<int> b32((size_t)ncheck * 64), b16((size_t)ncheck * 64);
        std::vector<uint8_t> n32((size_t)ncheck * ROWS * 32), n16(n32.size());
        CHECK(hipMemcpy(b32.data(), db32, b32.size() * 4, hipMemcpyDeviceToHost));
        CHECK(hipMemcpy(b16.data(), db16, b16.size() * 4, hipMemcpyDeviceToHost));
        CHECK(hipMemcpy(n32.data(), dn32, n32.size(), hipMemcpyDeviceToHost));
        CHECK(hipMemcpy(n16.data(), dn16, n16.size(), hipMemcpyDeviceToHost));
        long bad_best = 0, bad_nib = 0;
        for (size_t k = 0; k < b32.size(); k += 2)
            if (b32[k] >= 0 && (b32[k] != b16[k] || b32[k + 1] != b16[k + 1])) ++bad_best;
        for (int e = 0; e < ncheck; ++e)
            for (int i = 0; i < M; ++i)
                for (int k = XC - HB; k <= XC + HB; ++k) {
                    const size_t at = ((size_t)e * ROWS + i) * 32 + k;
                    if (n32[at] != n16[at]) ++bad_nib;
                }
        printf("{\"check_extensions\": %d, \"best_mismatches\": %ld, \"nibble_mismatches\": %ld}\n", ncheck,
               bad_best, bad_nib);
    }
    Ext X{dtab, drefw, n};
    hipEvent_t a, b;
    CHECK(hipEventCreate(&a));
    CHECK(hipEventCreate(&b));
    int dev;
    hipDeviceProp_t prop;
    CHECK(hipGetDevice(&dev));
    CHECK(hipGetDeviceProperties(&prop, dev));
    const int grid = prop.multiProcessorCount * 8;
    float t32 = 1e30f, t16 = 1e30f;
    for (int rep = 0; rep < 5; ++rep) {
        float ms;
        CHECK(hipEventRecord(a));
        hipLaunchKernelGGL(k_row32<false>, dim3(grid), dim3(256), 0, 0, X, db32, nullptr);
        CHECK(hipEventRecord(b));
        CHECK(hipEventSynchronize(b));
        CHECK(hipEventElapsedTime(&ms, a, b));
        t32 = ms < t32 ? ms : t32;
        CHECK(hipEventRecord(a));
        hipLaunchKernelGGL(k_row16<false>, dim3(grid), dim3(256), 0, 0, X, db16, nullptr);
        CHECK(hipEventRecord(b));
        CHECK(hipEventSynchronize(b));
        CHECK(hipEventElapsedTime(&ms, a, b));
        t16 = ms < t16 ? ms : t16;
    }
    const double cells = (double)n * M * 31;
    printf("{\"extensions\": %d, \"rows\": %d, \"grid\": %d, \"k_row32_ms\": %.3f, \"k_row16_ms\": %.3f, "
           "\"row32_gcups\": %.1f, \"row16_gcups\": %.1f, \"speedup\": %.3f}\n",
           n, M, grid, t32, t16, cells / (t32 * 1e-3) / 1e9, cells / (t16 * 1e-3) / 1e9, t32 / t16);
    return 0;
}
