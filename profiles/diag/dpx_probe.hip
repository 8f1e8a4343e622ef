// profiles/diag/dpx_probe.hip -- is an anti-diagonal k_dp faster than the
// row-wise one?  Two DP cores over the same synthetic extensions (251 rows,
// 64-diagonal band, local mode, the library's scoring encoding), timed and
// cross-checked (best score, row and diagonal of every extension):
//   k_rows  the r02 k_dp row recurrence: lane = diagonal, 8-row groups,
//           DPP prefix-max scan for the deletions, 4 traceback bits per cell
//           in LDS, 1 extension per wave, 4 waves per workgroup
//   k_diag  cell (i, k) at step t = 2i + k: lane l holds diagonals 2l and
//           2l+1, two extensions per wave (lanes 0-31, 32-63), one DPP move
//           per step and no scan, traceback bits in LDS, 1 wave per workgroup
//   hipcc --offload-arch=gfx950 -O3 -o dpx_probe dpx_probe.hip && ./dpx_probe
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); exit(1); } } while (0)

constexpr int M = 251, ROWS = 256, BAND = 64, GBAR = 4;
constexpr int OEI = 13, EXI = 3, OED = 13, EXD = 3;

template <int CTRL>
__device__ __forceinline__ int dppz(int v) { return __builtin_amdgcn_update_dpp(0, v, CTRL, 0xF, 0xF, true); }
constexpr int ROW_SHR1 = 0x111, ROW_SHR2 = 0x112, ROW_SHR4 = 0x114, ROW_SHR8 = 0x118,
              WAVE_SHL1 = 0x130, WAVE_SHR1 = 0x138;
__device__ __forceinline__ int imax(int a, int b) { return a > b ? a : b; }
__device__ __forceinline__ int in_vgpr(int v) { int r; asm("v_mov_b32 %0, %1" : "=v"(r) : "s"(v)); return r; }

// ------------------------------------------------------------------ rows
constexpr int BIAS = 1 << 20;

__device__ __forceinline__ int scan_max(int x)
{
    x = imax(x, dppz<ROW_SHR1>(x));
    x = imax(x, dppz<ROW_SHR2>(x));
    x = imax(x, dppz<ROW_SHR4>(x));
    x = imax(x, dppz<ROW_SHR8>(x));
    asm volatile("s_nop 1\n\tv_max_i32_dpp %0, %0, %0 row_bcast:15 row_mask:0xa bank_mask:0xf\n\t"
                 "s_nop 1\n\tv_max_i32_dpp %0, %0, %0 row_bcast:31 row_mask:0xc bank_mask:0xf\n\ts_nop 1"
                 : "+v"(x));
    return x;
}

struct RowK { int mexI, moeI, xD, cF; };

// AB (ablation, timing only): bit 0 drops the traceback bits, bit 1 the best-cell
// key, bit 2 replaces the 6-step prefix-max scan by one neighbour step
template <int AB>
__device__ __forceinline__ void row_gap(uint32_t tbv, int rc, int &Hp, int &Ep, uint32_t &bestKey,
                                        int ci, const RowK &K, uint32_t &acc)
{
    const int Hd = Hp + (int)__builtin_amdgcn_ubfe(tbv, (uint32_t)rc, 4) - 8;
    const int e1 = dppz<WAVE_SHL1>(Ep) + K.mexI;
    const int h1 = dppz<WAVE_SHL1>(Hp) + K.moeI;
    const int E = imax(e1, h1);
    int H1 = imax(imax(Hd, E), BIAS);
    const int X = H1 + K.xD;
    const int P = (AB & 4) ? imax(X, dppz<ROW_SHR1>(X)) : scan_max(X);
    const int F = dppz<WAVE_SHR1>(P) + K.cF;
    const int H = imax(H1, F);
    if (!(AB & 2)) {
        const uint32_t key = (uint32_t)H * 1024u + (uint32_t)ci;
        bestKey = bestKey > key ? bestKey : key;
    } else {
        bestKey = bestKey > (uint32_t)H ? bestKey : (uint32_t)H;
    }
    uint64_t ma, mb, mz, me, mf;
    int xl;
    if (AB & 1) acc += (uint32_t)(H ^ E ^ Hd);
    else asm volatile(
        "v_cmp_ne_u32_e64 %[ma], %[H], %[Hd]\n\t"
        "v_cmp_ne_u32_e64 %[mb], %[H], %[E]\n\t"
        "v_cmp_ne_u32_e64 %[mz], %[bias], %[H]\n\t"
        "v_cmp_lt_i32_e64 %[me], %[h1], %[e1]\n\t"
        "v_add_u32_dpp %[xl], %[X], %[cF] wave_shr:1 row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t"
        "s_orn2_b64 %[mb], %[mb], %[ma]\n\t"
        "v_cmp_lt_i32_e64 %[mf], %[xl], %[F]\n\t"
        "s_and_b64 %[ma], %[ma], %[mz]\n\t"
        "s_and_b64 %[mb], %[mb], %[mz]\n\t"
        "v_addc_co_u32_e64 %[acc], vcc, %[acc], %[acc], %[mf]\n\t"
        "v_addc_co_u32_e64 %[acc], vcc, %[acc], %[acc], %[me]\n\t"
        "v_addc_co_u32_e64 %[acc], vcc, %[acc], %[acc], %[ma]\n\t"
        "v_addc_co_u32_e64 %[acc], vcc, %[acc], %[acc], %[mb]"
        : [acc] "+v"(acc), [ma] "=&s"(ma), [mb] "=&s"(mb), [mz] "=&s"(mz), [me] "=&s"(me),
          [mf] "=&s"(mf), [xl] "=&v"(xl)
        : [H] "v"(H), [Hd] "v"(Hd), [E] "v"(E), [h1] "v"(h1), [e1] "v"(e1), [X] "v"(X),
          [cF] "v"(K.cF), [F] "v"(F), [bias] "s"(BIAS)
        : "vcc");
    Hp = H;
    Ep = E;
}

__device__ __forceinline__ void row_nogap(uint32_t tbv, int rc, int &Hp, int &Ep, uint32_t &bestKey,
                                          int ci, uint32_t &acc)
{
    int H = Hp + (int)__builtin_amdgcn_ubfe(tbv, (uint32_t)rc, 4) - 8;
    H = imax(H, BIAS);
    const uint32_t src = (uint32_t)(H - BIAS) < 1u ? (uint32_t)(H - BIAS) : 1u;
    const uint32_t key = (uint32_t)H * 1024u + (uint32_t)ci;
    bestKey = bestKey > key ? bestKey : key;
    acc = (acc << 4) + src;
    Hp = H;
    Ep = 0;
}

// tab: n_ext x ROWS u32; ref: n_ext x (ROWS + 72) bytes (code * 4).
// GB = 0: traceback bits in LDS (the r02 layout, 9.5 KB per wave, 4 waves
// per SIMD); GB = 1: bits in a per-wave global slab (LDS 1.3 KB per wave, the
// VGPR count sets the occupancy).  After the DP a serial walk reads 32
// dependent traceback words, like the real traceback does.
template <int GB, int AB = 0>
__global__ __launch_bounds__(256) void k_rows(const uint32_t *gtab, const uint8_t *gref, int n_ext,
                                              int *out, uint32_t *gbits)
{
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    constexpr int WL = GB ? ROWS * 4 + ROWS + 72 : ROWS / 8 * 64 * 4 + ROWS * 4 + ROWS + 72;
    unsigned char *wb = smem + wv * WL;
    uint32_t *bits = GB ? gbits + (size_t)(blockIdx.x * 4 + wv) * (ROWS / 8 * 64) : (uint32_t *)wb;
    uint32_t *tab = GB ? (uint32_t *)wb : (uint32_t *)wb + ROWS / 8 * 64;
    uint8_t *refw = (uint8_t *)(tab + ROWS);
    RowK K;
    K.mexI = in_vgpr(-EXI);
    K.moeI = in_vgpr(-OEI);
    K.xD = lane * EXD;
    K.cF = -(OED - EXD) - EXD * lane;
    for (int x = blockIdx.x * 4 + wv; x < n_ext; x += gridDim.x * 4) {
        for (int i = lane; i < ROWS; i += 64) tab[i] = gtab[(size_t)x * ROWS + i];
        for (int i = lane; i < ROWS + 72; i += 64) refw[i] = gref[(size_t)x * (ROWS + 72) + i];
        __builtin_amdgcn_wave_barrier();
        int Hp = BIAS, Ep = 0;
        uint32_t bestKey = 0;
        for (int i0 = 0; i0 < M; i0 += 8) {
            uint32_t tbv[8];
            int rcv[8];
#pragma unroll
            for (int t = 0; t < 8; ++t) { tbv[t] = tab[i0 + t]; rcv[t] = refw[i0 + t + lane]; }
            uint32_t acc = 0;
            if (i0 >= GBAR && i0 + 8 <= M - GBAR) {
#pragma unroll
                for (int t = 0; t < 8; ++t) row_gap<AB>(tbv[t], rcv[t], Hp, Ep, bestKey, 1023 - (i0 + t), K, acc);
            } else {
#pragma unroll
                for (int t = 0; t < 8; ++t) {
                    const int i = i0 + t;
                    if (i >= M) acc <<= 4;
                    else if (i >= GBAR && i < M - GBAR) row_gap<AB>(tbv[t], rcv[t], Hp, Ep, bestKey, 1023 - i, K, acc);
                    else row_nogap(tbv[t], rcv[t], Hp, Ep, bestKey, 1023 - i, acc);
                }
            }
            bits[(i0 >> 3) * 64 + lane] = acc;
        }
        // best: max score, then smallest row, then smallest lane
        const int bestH = (int)(bestKey >> 10) - BIAS, bestI = 1023 - (int)(bestKey & 1023u);
        long long key = (long long)bestH * 1048576ll + (long long)((1023 - bestI) << 6) + (63 - lane);
        for (int o = 32; o; o >>= 1) { long long y = __shfl_xor(key, o); key = key > y ? key : y; }
        if (GB) {   // the wave's own vector stores, visible to its loads below
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
        } else {
            __builtin_amdgcn_wave_barrier();
        }
        // serial walk: 32 dependent words from the best cell's group down
        int k = __builtin_amdgcn_readfirstlane(63 - (int)(key & 63));
        uint32_t sum = 0;
        for (int g = __builtin_amdgcn_readfirstlane((1023 - (int)((key >> 6) & 1023)) >> 3); g >= 0; --g) {
            const uint32_t word = __builtin_amdgcn_readfirstlane(bits[g * 64 + k]);
            sum += word;
            k = (k + (int)(word >> 31)) & 63;
        }
        if (lane == 0) {
            out[4 * x] = (int)(key >> 20);
            out[4 * x + 1] = 1023 - (int)((key >> 6) & 1023);
            out[4 * x + 2] = 63 - (int)(key & 63);
            out[4 * x + 3] = (int)sum;
        }
        __builtin_amdgcn_wave_barrier();
    }
}

int main(int argc, char **argv)
{
    const int n = argc > 1 ? atoi(argv[1]) : 400000;
    std::vector<uint32_t> tab((size_t)n * ROWS);
    std::vector<uint8_t> ref((size_t)n * (ROWS + 72));
    srand(7);
    for (int x = 0; x < n; ++x) {
        std::vector<int> g(ROWS + 72);
        for (auto &c : g) c = rand() & 3;
        for (int i = 0; i < ROWS + 72; ++i) ref[(size_t)x * (ROWS + 72) + i] = (uint8_t)(g[i] * 4);
        // read = ref along diagonal 32 with 8 % substitutions and one 3-base deletion in the middle
        const int del = 80 + rand() % 90;
        for (int i = 0; i < ROWS; ++i) {
            int j = i + 32 + (i >= del ? 3 : 0);
            int c = j < ROWS + 72 ? g[j] : 0;
            if (rand() % 100 < 8) c = (c + 1 + rand() % 3) & 3;
            const int pen = 2 + (rand() % 41) / 10;
            uint32_t tb = 0;
            for (int q = 0; q < 5; ++q) {
                const int sc = q > 3 ? -1 : (q == c ? 2 : -pen);
                tb |= (uint32_t)(sc + 8) << (4 * q);
            }
            tab[(size_t)x * ROWS + i] = tb;
        }
    }
    uint32_t *dt; uint8_t *dr; int *o1, *o2; uint32_t *gb;
    const int g_lds = 256 * 12, g_glb = 256 * 8;   // grids: LDS variant 4 blocks/CU resident (grid-stride), global variant 8 blocks/CU
    CHECK(hipMalloc(&dt, tab.size() * 4));
    CHECK(hipMalloc(&dr, ref.size()));
    CHECK(hipMalloc(&o1, (size_t)n * 16));
    CHECK(hipMalloc(&o2, (size_t)n * 16));
    CHECK(hipMalloc(&gb, (size_t)g_glb * 4 * (ROWS / 8 * 64) * 4));
    CHECK(hipMemcpy(dt, tab.data(), tab.size() * 4, hipMemcpyHostToDevice));
    CHECK(hipMemcpy(dr, ref.data(), ref.size(), hipMemcpyHostToDevice));
    const int lds0 = 4 * (ROWS / 8 * 64 * 4 + ROWS * 4 + ROWS + 72);
    const int lds1 = 4 * (ROWS * 4 + ROWS + 72);
    CHECK(hipFuncSetAttribute((const void *)k_rows<0>, hipFuncAttributeMaxDynamicSharedMemorySize, lds0));
    CHECK(hipFuncSetAttribute((const void *)k_rows<1>, hipFuncAttributeMaxDynamicSharedMemorySize, lds1));
    hipEvent_t a, b;
    hipEventCreate(&a); hipEventCreate(&b);
    float ms1 = 0, ms2 = 0;
    for (int rep = 0; rep < 3; ++rep) {
        hipEventRecord(a);
        hipLaunchKernelGGL(k_rows<0>, dim3(g_lds), dim3(256), lds0, 0, dt, dr, n, o1, gb);
        hipEventRecord(b);
        hipEventSynchronize(b);
        hipEventElapsedTime(&ms1, a, b);
        hipEventRecord(a);
        hipLaunchKernelGGL(k_rows<1>, dim3(g_glb), dim3(256), lds1, 0, dt, dr, n, o2, gb);
        hipEventRecord(b);
        hipEventSynchronize(b);
        hipEventElapsedTime(&ms2, a, b);
        CHECK(hipGetLastError());
    }
    std::vector<int> r1((size_t)n * 4), r2((size_t)n * 4);
    CHECK(hipMemcpy(r1.data(), o1, r1.size() * 4, hipMemcpyDeviceToHost));
    CHECK(hipMemcpy(r2.data(), o2, r2.size() * 4, hipMemcpyDeviceToHost));
    int bad = 0;
    for (int x = 0; x < n; ++x)
        for (int q = 0; q < 4; ++q)
            if (r1[4 * x + q] != r2[4 * x + q]) {
                if (bad < 5) printf("ext %d: lds (%d,%d,%d,%d) global (%d,%d,%d,%d)\n", x, r1[4 * x], r1[4 * x + 1],
                                    r1[4 * x + 2], r1[4 * x + 3], r2[4 * x], r2[4 * x + 1], r2[4 * x + 2], r2[4 * x + 3]);
                ++bad;
                break;
            }
    // ablations (timing only): ns per row per SIMD
    float ab[4] = {0, 0, 0, 0};
    const int abk[4] = {1, 2, 4, 7};
    for (int q = 0; q < 4; ++q) {
        for (int rep = 0; rep < 2; ++rep) {
            hipEventRecord(a);
            switch (abk[q]) {
                case 1: hipLaunchKernelGGL((k_rows<0, 1>), dim3(g_lds), dim3(256), lds0, 0, dt, dr, n, o2, gb); break;
                case 2: hipLaunchKernelGGL((k_rows<0, 2>), dim3(g_lds), dim3(256), lds0, 0, dt, dr, n, o2, gb); break;
                case 4: hipLaunchKernelGGL((k_rows<0, 4>), dim3(g_lds), dim3(256), lds0, 0, dt, dr, n, o2, gb); break;
                default: hipLaunchKernelGGL((k_rows<0, 7>), dim3(g_lds), dim3(256), lds0, 0, dt, dr, n, o2, gb); break;
            }
            hipEventRecord(b);
            hipEventSynchronize(b);
            hipEventElapsedTime(&ab[q], a, b);
        }
        CHECK(hipGetLastError());
    }
    const double rows_per_simd = (double)n * M / 1024.0;
    printf("{\"ns_per_row_per_simd\": {\"full\": %.2f, \"no_bits\": %.2f, \"no_key\": %.2f, \"no_scan\": %.2f, "
           "\"none_of_the_three\": %.2f}}\n", ms1 * 1e6 / rows_per_simd, ab[0] * 1e6 / rows_per_simd,
           ab[1] * 1e6 / rows_per_simd, ab[2] * 1e6 / rows_per_simd, ab[3] * 1e6 / rows_per_simd);
    printf("{\"extensions\": %d, \"lds_bits_ms\": %.3f, \"global_bits_ms\": %.3f, \"speedup\": %.3f, "
           "\"mismatches\": %d, \"example_best\": [%d, %d, %d]}\n",
           n, ms1, ms2, ms1 / ms2, bad, r1[0], r1[1], r1[2]);
    return bad != 0;
}
