// profiles/diag/issue_probe.hip -- SIMD issue cost of the instruction kinds
// of k_dp's row recurrence, with the chip full (8 waves per SIMD) and with one
// wave per SIMD.  Each wave runs ITER x 8 independent instructions of one
// kind (8 round-robin chains, so no DPP read is near the write it reads);
// cycles come from s_memtime around the loop.  Output: JSON, one entry per
// kind: cycles per instruction per SIMD (all waves of the SIMD together) and
// per wave.
//   hipcc --offload-arch=gfx950 -O3 -o issue_probe issue_probe.hip && ./issue_probe
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); exit(1); } } while (0)

constexpr int ITER = 2048;

#define R8(body) body(0) body(1) body(2) body(3) body(4) body(5) body(6) body(7)

template <int KIND>
__global__ __launch_bounds__(256) void k_issue(int *out, long long *cyc, int seed)
{
    int v0 = threadIdx.x + seed, v1 = v0 * 3, v2 = v0 ^ 5, v3 = v0 + 7, v4 = v0 * 11, v5 = v0 ^ 9,
        v6 = v0 + 13, v7 = v0 * 17;
    int w = v0 | 1;
    uint32_t a = 0;
    __shared__ int pad[256];   // LDS the ds_read kind reads (address 0)
    if (KIND == 16) {
        pad[threadIdx.x] = 0;
        __syncthreads();
    }
    const long long t0 = __builtin_amdgcn_s_memtime();
    for (int it = 0; it < ITER; ++it) {
        if (KIND == 0) {   // VOP2 add
#define B(i) asm volatile("v_add_u32 %0, %0, %1" : "+v"(v##i) : "v"(w));
            R8(B)
#undef B
        } else if (KIND == 1) {   // v_max_i32_dpp row_shr:1 (scan step)
#define B(i) asm volatile("v_max_i32_dpp %0, %0, %0 row_shr:1 row_mask:0xf bank_mask:0xf bound_ctrl:1" : "+v"(v##i));
            R8(B)
#undef B
        } else if (KIND == 2) {   // v_add_u32_dpp wave_shr:1 (E / F moves)
#define B(i) asm volatile("v_add_u32_dpp %0, %0, %1 wave_shr:1 row_mask:0xf bank_mask:0xf bound_ctrl:1" : "+v"(v##i) : "v"(w));
            R8(B)
#undef B
        } else if (KIND == 3) {   // v_max_i32_dpp row_bcast:15 (cross-row scan step)
#define B(i) asm volatile("v_max_i32_dpp %0, %0, %0 row_bcast:15 row_mask:0xa bank_mask:0xf" : "+v"(v##i));
            R8(B)
#undef B
        } else if (KIND == 4) {   // v_cmp_e64 into an SGPR pair
            uint64_t m;
#define B(i) asm volatile("v_cmp_ne_u32_e64 %0, %1, %2" : "=s"(m) : "v"(v##i), "v"(w)); a += (uint32_t)(m >> 0 & 0);
            R8(B)
#undef B
        } else if (KIND == 5) {   // v_addc_co_u32_e64 with an SGPR carry-in (traceback bit append)
            uint64_t m = (uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane(w) * 0x100000001ull;
#define B(i) asm volatile("v_addc_co_u32_e64 %0, vcc, %0, %0, %1" : "+v"(v##i) : "s"(m) : "vcc");
            R8(B)
#undef B
        } else if (KIND == 6) {   // VOP3 3-operand integer op
#define B(i) asm volatile("v_lshl_add_u32 %0, %0, 2, %1" : "+v"(v##i) : "v"(w));
            R8(B)
#undef B
        } else if (KIND == 7) {   // v_max3_i32
#define B(i) asm volatile("v_max3_i32 %0, %0, %1, %1" : "+v"(v##i) : "v"(w));
            R8(B)
#undef B
        } else if (KIND == 10) {   // VOPC e32 into VCC
#define B(i) asm volatile("v_cmp_ne_u32_e32 vcc, %0, %1" : : "v"(v##i), "v"(w) : "vcc");
            R8(B)
#undef B
        } else if (KIND == 11) {   // VOP2 v_addc_co_u32_e32 (carry in / out in VCC)
#define B(i) asm volatile("v_addc_co_u32_e32 %0, vcc, %0, %0, vcc" : "+v"(v##i) : : "vcc");
            R8(B)
#undef B
        } else if (KIND == 12) {   // v_alignbit_b32 (VOP3: shift a sign bit into an accumulator)
#define B(i) asm volatile("v_alignbit_b32 %0, %0, %1, 31" : "+v"(v##i) : "v"(w));
            R8(B)
#undef B
        } else if (KIND == 13) {   // v_cndmask_b32_e32 (VCC select)
#define B(i) asm volatile("v_cndmask_b32_e32 %0, %0, %1, vcc" : "+v"(v##i) : "v"(w) : "vcc");
            R8(B)
#undef B
        } else if (KIND == 14) {   // VOPC e32 + VOP2 addc e32 pairs (one bit appended per pair)
#define B(i) asm volatile("v_cmp_lt_i32_e32 vcc, %0, %1\n\tv_addc_co_u32_e32 %0, vcc, %0, %0, vcc" : "+v"(v##i) : "v"(w) : "vcc");
            R8(B)
#undef B
        } else if (KIND == 15) {   // VOPC e32 + s_mov_b64 of VCC (mask kept for SALU logic)
            uint64_t m;
#define B(i) asm volatile("v_cmp_lt_i32_e32 vcc, %1, %2\n\ts_mov_b64 %0, vcc" : "=s"(m) : "v"(v##i), "v"(w) : "vcc"); a += 0 * (uint32_t)m;
            R8(B)
#undef B
        } else if (KIND == 16) {   // ds_read_b32 interleaved with VOP2 adds (LDS pipe beside the VALU)
#define B(i) asm volatile("ds_read_b32 %0, %1\n\tv_add_u32 %0, %0, %2" : "+v"(v##i) : "v"(0), "v"(w));
            R8(B)
#undef B
            asm volatile("s_waitcnt lgkmcnt(0)");
        } else if (KIND == 8) {   // dependent chain of v_add_u32 (latency, 1 chain)
#define B(i) asm volatile("v_add_u32 %0, %0, %1" : "+v"(v0) : "v"(w));
            R8(B)
#undef B
        } else if (KIND == 9) {   // dependent DPP chain: VALU write -> DPP read, s_nop 1 between
#define B(i) asm volatile("s_nop 1\n\tv_max_i32_dpp %0, %0, %0 row_shr:1 row_mask:0xf bank_mask:0xf bound_ctrl:1" : "+v"(v0));
            R8(B)
#undef B
        }
    }
    const long long t1 = __builtin_amdgcn_s_memtime();
    out[blockIdx.x * blockDim.x + threadIdx.x] = v0 + v1 + v2 + v3 + v4 + v5 + v6 + v7 + (int)a;
    if ((threadIdx.x & 63) == 0) cyc[blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6)] = t1 - t0;
}

template <int KIND>
static void run(const char *name, int blocks, int *dout, long long *dcyc, long long *hcyc, bool last)
{
    hipEvent_t ea, eb;
    CHECK(hipEventCreate(&ea));
    CHECK(hipEventCreate(&eb));
    CHECK(hipEventRecord(ea));
    hipLaunchKernelGGL(k_issue<KIND>, dim3(blocks), dim3(256), 0, 0, dout, dcyc, 1);
    CHECK(hipEventRecord(eb));
    CHECK(hipDeviceSynchronize());
    float ms = 0;
    CHECK(hipEventElapsedTime(&ms, ea, eb));
    const int waves = blocks * 4;
    CHECK(hipMemcpy(hcyc, dcyc, waves * sizeof(long long), hipMemcpyDeviceToHost));
    double s = 0;
    for (int i = 0; i < waves; ++i) s += (double)hcyc[i];
    const double per_wave = s / waves / (ITER * 8.0);
    // waves resident per SIMD: blocks * 4 waves spread over 256 CUs x 4 SIMDs
    const double wps = waves / 1024.0;
    printf("    \"%s\": {\"waves_per_simd\": %.0f, \"cyc_per_inst_per_wave\": %.2f, \"cyc_per_inst_per_simd\": %.2f, "
           "\"ns_per_inst_per_simd_wall\": %.3f}%s\n",
           name, wps, per_wave, per_wave / wps, ms * 1e6 / (wps * ITER * 8.0), last ? "" : ",");
}

int main()
{
    int *dout;
    long long *dcyc, *hcyc;
    CHECK(hipMalloc(&dout, 2048 * 256 * 4));
    CHECK(hipMalloc(&dcyc, 2048 * 4 * 8));
    hcyc = (long long *)malloc(2048 * 4 * 8);
    hipLaunchKernelGGL(k_issue<0>, dim3(2048), dim3(256), 0, 0, dout, dcyc, 1);   // warm up
    CHECK(hipDeviceSynchronize());
    printf("{\"note\": \"s_memtime cycles; 8 waves/SIMD = 2048 blocks of 4 waves, 1 wave/SIMD = 256 blocks\",\n");
    for (int pass = 0; pass < 2; ++pass) {
        const int blocks = pass ? 256 : 2048;
        printf("  \"%s\": {\n", pass ? "one_wave_per_simd" : "full_chip");
        run<0>("v_add_u32", blocks, dout, dcyc, hcyc, false);
        run<1>("v_max_i32_dpp_row_shr", blocks, dout, dcyc, hcyc, false);
        run<2>("v_add_u32_dpp_wave_shr", blocks, dout, dcyc, hcyc, false);
        run<3>("v_max_i32_dpp_row_bcast", blocks, dout, dcyc, hcyc, false);
        run<4>("v_cmp_ne_u32_e64_sgpr", blocks, dout, dcyc, hcyc, false);
        run<5>("v_addc_co_u32_e64_sgpr_carry", blocks, dout, dcyc, hcyc, false);
        run<6>("v_lshl_add_u32", blocks, dout, dcyc, hcyc, false);
        run<7>("v_max3_i32", blocks, dout, dcyc, hcyc, false);
        run<8>("dependent_v_add_u32", blocks, dout, dcyc, hcyc, false);
        run<9>("dependent_dpp_with_nop", blocks, dout, dcyc, hcyc, false);
        run<10>("v_cmp_ne_u32_e32_vcc", blocks, dout, dcyc, hcyc, false);
        run<11>("v_addc_co_u32_e32_vcc", blocks, dout, dcyc, hcyc, false);
        run<12>("v_alignbit_b32", blocks, dout, dcyc, hcyc, false);
        run<13>("v_cndmask_b32_e32", blocks, dout, dcyc, hcyc, false);
        run<14>("pair_vopc_e32_addc_e32", blocks, dout, dcyc, hcyc, false);
        run<15>("pair_vopc_e32_s_mov_b64", blocks, dout, dcyc, hcyc, false);
        run<16>("pair_ds_read_b32_v_add", blocks, dout, dcyc, hcyc, true);
        printf("  }%s\n", pass ? "" : ",");
    }
    printf("}\n");
    return 0;
}
