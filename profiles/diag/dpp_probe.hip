// Probe: prefix max over a wave64 with row_shr steps and the two cross-row
// steps done (a) with row masks 0xA / 0xC (current k_dp form) and (b) with
// full row masks and bound_ctrl (zero fill), against a serial reference.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>

template <int CTRL, int RM, bool BC>
__device__ int dpp(int old, int v) { return __builtin_amdgcn_update_dpp(old, v, CTRL, RM, 0xF, BC); }
__device__ int imax(int a, int b) { return a > b ? a : b; }

__global__ void k(const int *in, int *outa, int *outb, int *raw15, int *raw31)
{
    const int t = blockIdx.x * 64 + threadIdx.x;
    int x = in[t];
    x = imax(x, dpp<0x111, 0xF, true>(0, x));
    x = imax(x, dpp<0x112, 0xF, true>(0, x));
    x = imax(x, dpp<0x114, 0xF, true>(0, x));
    x = imax(x, dpp<0x118, 0xF, true>(0, x));
    int a = imax(x, dpp<0x142, 0xA, false>(x, x));
    a = imax(a, dpp<0x143, 0xC, false>(a, a));
    int b = imax(x, dpp<0x142, 0xF, true>(0, x));
    b = imax(b, dpp<0x143, 0xF, true>(0, b));
    outa[t] = a;
    outb[t] = b;
    raw15[t] = dpp<0x142, 0xF, true>(0, x);
    raw31[t] = dpp<0x143, 0xF, true>(0, x);
}

int main()
{
    const int W = 4096, N = W * 64;
    std::vector<int> h(N), a(N), b(N), r15(N), r31(N);
    srand(7);
    for (int i = 0; i < N; ++i) h[i] = 1 + rand() % 100000;
    int *d, *da, *db, *d15, *d31;
    hipMalloc(&d, N * 4); hipMalloc(&da, N * 4); hipMalloc(&db, N * 4);
    hipMalloc(&d15, N * 4); hipMalloc(&d31, N * 4);
    hipMemcpy(d, h.data(), N * 4, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(k, dim3(W), dim3(64), 0, 0, d, da, db, d15, d31);
    hipMemcpy(a.data(), da, N * 4, hipMemcpyDeviceToHost);
    hipMemcpy(b.data(), db, N * 4, hipMemcpyDeviceToHost);
    hipMemcpy(r15.data(), d15, N * 4, hipMemcpyDeviceToHost);
    hipMemcpy(r31.data(), d31, N * 4, hipMemcpyDeviceToHost);
    long bad_a = 0, bad_b = 0;
    for (int w = 0; w < W; ++w) {
        int m = 0;
        for (int l = 0; l < 64; ++l) {
            m = h[w * 64 + l] > m ? h[w * 64 + l] : m;
            bad_a += a[w * 64 + l] != m;
            bad_b += b[w * 64 + l] != m;
        }
    }
    printf("mismatches: masked form %ld, full-mask bound_ctrl form %ld (of %d)\n", bad_a, bad_b, N);
    printf("raw bcast15 (bound_ctrl, full mask) lanes 0,15,16,31,32,48: %d %d %d %d %d %d\n", r15[0], r15[15], r15[16], r15[31], r15[32], r15[48]);
    printf("raw bcast31 (bound_ctrl, full mask) lanes 0,16,31,32,48,63: %d %d %d %d %d %d\n", r31[0], r31[16], r31[31], r31[32], r31[48], r31[63]);
    return 0;
}
