// profiles/diag/valu_rate.hip -- issue cost of the instruction forms k_dp's row
// recurrence is made of, on gfx950: plain VALU, DPP row_shr / row_bcast /
// wave_shl, VOP3 compare + cndmask.  Four independent chains per wave (no DPP
// hazard wait states needed), 1 or 4 waves per SIMD; prints SIMD cycles per
// wave-instruction from s_memtime over the loop.
//   hipcc --offload-arch=gfx950 -O2 -o valu_rate valu_rate.hip && ./valu_rate
#include <hip/hip_runtime.h>
#include <cstdio>

#define REP8(x) x x x x x x x x
#define K(name, body)                                                              \
__global__ void name(long long *cyc, int iters, int *sink)                         \
{                                                                                  \
    int a = threadIdx.x, b = a + 1, c = a + 2, d = a + 3;                          \
    long long t0 = __builtin_readcyclecounter();                                   \
    for (int it = 0; it < iters; ++it) {                                           \
        REP8(body)                                                                 \
    }                                                                              \
    long long t1 = __builtin_readcyclecounter();                                   \
    if (threadIdx.x % 64 == 0) cyc[blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64] = t1 - t0; \
    if (a + b + c + d == 12345) sink[0] = 1;                                        \
}
// 4 instructions per body, 8 bodies per iteration -> 32 per iteration
K(k_max, asm volatile("v_max_i32 %0, %0, %1\n v_max_i32 %1, %1, %2\n v_max_i32 %2, %2, %3\n v_max_i32 %3, %3, %0" : "+v"(a), "+v"(b), "+v"(c), "+v"(d));)
K(k_add3, asm volatile("v_add3_u32 %0, %0, %1, 8\n v_add3_u32 %1, %1, %2, 8\n v_add3_u32 %2, %2, %3, 8\n v_add3_u32 %3, %3, %0, 8" : "+v"(a), "+v"(b), "+v"(c), "+v"(d));)
K(k_dpp_shr, asm volatile("v_max_i32_dpp %0, %1, %0 row_shr:1 bound_ctrl:1\n v_max_i32_dpp %1, %2, %1 row_shr:1 bound_ctrl:1\n v_max_i32_dpp %2, %3, %2 row_shr:1 bound_ctrl:1\n v_max_i32_dpp %3, %0, %3 row_shr:1 bound_ctrl:1" : "+v"(a), "+v"(b), "+v"(c), "+v"(d));)
K(k_dpp_bcast, asm volatile("v_max_i32_dpp %0, %1, %0 row_bcast:15 row_mask:0xa\n v_max_i32_dpp %1, %2, %1 row_bcast:15 row_mask:0xa\n v_max_i32_dpp %2, %3, %2 row_bcast:31 row_mask:0xc\n v_max_i32_dpp %3, %0, %3 row_bcast:31 row_mask:0xc" : "+v"(a), "+v"(b), "+v"(c), "+v"(d));)
K(k_dpp_wshl, asm volatile("v_add_u32_dpp %0, %1, %0 wave_shl:1 bound_ctrl:1\n v_add_u32_dpp %1, %2, %1 wave_shl:1 bound_ctrl:1\n v_add_u32_dpp %2, %3, %2 wave_shr:1 bound_ctrl:1\n v_add_u32_dpp %3, %0, %3 wave_shr:1 bound_ctrl:1" : "+v"(a), "+v"(b), "+v"(c), "+v"(d));)
K(k_cmp_cnd, asm volatile("v_cmp_lt_i32_e64 s[40:41], %0, %1\n v_cndmask_b32_e64 %2, 0, -1, s[40:41]\n v_cmp_ne_u32_e64 s[42:43], %3, %1\n v_cndmask_b32_e64 %0, 1, 2, s[42:43]" : "+v"(a), "+v"(b), "+v"(c), "+v"(d) :: "s40", "s41", "s42", "s43");)
// one dependent chain (each instruction needs the previous result): latency
K(k_chain, asm volatile("v_max_i32 %0, %0, %1\n v_add_u32 %0, %0, %2\n v_max_i32 %0, %0, %3\n v_add_u32 %0, %0, %1" : "+v"(a), "+v"(b), "+v"(c), "+v"(d));)

// a dependent DPP scan chain as k_dp's row has it: every step reads the
// previous step's result, so 2 wait states (s_nop 1) separate them
K(k_scan_nop, asm volatile("v_max_i32_dpp %0, %0, %0 row_shr:1 bound_ctrl:1\n s_nop 1\n v_max_i32_dpp %0, %0, %0 row_shr:2 bound_ctrl:1\n s_nop 1\n v_max_i32_dpp %0, %0, %0 row_shr:4 bound_ctrl:1\n s_nop 1\n v_max_i32_dpp %0, %0, %0 row_shr:8 bound_ctrl:1\n s_nop 1" : "+v"(a), "+v"(b), "+v"(c), "+v"(d));)
// the same chain with two independent VALU ops in every wait slot pair
K(k_scan_fill, asm volatile("v_max_i32_dpp %0, %0, %0 row_shr:1 bound_ctrl:1\n v_add_u32 %1, %1, %2\n v_add_u32 %3, %3, %2\n v_max_i32_dpp %0, %0, %0 row_shr:2 bound_ctrl:1\n v_add_u32 %1, %1, %2\n v_add_u32 %3, %3, %2\n v_max_i32_dpp %0, %0, %0 row_shr:4 bound_ctrl:1\n v_add_u32 %1, %1, %2\n v_add_u32 %3, %3, %2\n v_max_i32_dpp %0, %0, %0 row_shr:8 bound_ctrl:1\n v_add_u32 %1, %1, %2\n v_add_u32 %3, %3, %2" : "+v"(a), "+v"(b), "+v"(c), "+v"(d));)

typedef void (*KF)(long long *, int, int *);

int main()
{
    struct { const char *n; KF f; } ks[] = {{"v_max_i32", k_max}, {"v_add3_u32", k_add3},
        {"v_max_i32_dpp row_shr", k_dpp_shr}, {"v_max_i32_dpp row_bcast", k_dpp_bcast},
        {"v_add_u32_dpp wave_shl/shr", k_dpp_wshl}, {"v_cmp_e64 + v_cndmask_e64", k_cmp_cnd},
        {"dependent chain max/add", k_chain},
        {"scan chain + s_nop 1 (4 VALU, per 4)", k_scan_nop}, {"scan chain filled (12 VALU, per 4)", k_scan_fill}};
    hipDeviceProp_t p;
    hipGetDeviceProperties(&p, 0);
    const int cus = p.multiProcessorCount, iters = 4096;
    long long *cyc; int *sink;
    hipMalloc(&cyc, sizeof(long long) * cus * 64);
    hipMalloc(&sink, 4);
    long long *h = new long long[cus * 64];
    for (int wps = 1; wps <= 4; wps *= 2) {          // waves per SIMD
        for (auto &k : ks) {
            const int waves = 4 * wps;               // per CU: one block of 4*wps waves
            hipLaunchKernelGGL(k.f, dim3(cus), dim3(64 * waves), 0, 0, cyc, 16, sink);
            hipLaunchKernelGGL(k.f, dim3(cus), dim3(64 * waves), 0, 0, cyc, iters, sink);
            hipMemcpy(h, cyc, sizeof(long long) * cus * waves, hipMemcpyDeviceToHost);
            double s = 0;
            for (int i = 0; i < cus * waves; ++i) s += (double)h[i];
            s /= cus * waves;
            const double per_wave_instr = s / (iters * 32.0);
            printf("waves/SIMD %d  %-28s  wave cycles/instr %6.2f  SIMD cycles/instr %6.2f\n",
                   wps, k.n, per_wave_instr, per_wave_instr / wps);
        }
    }
    return 0;
}
