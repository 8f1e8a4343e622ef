// profiles/diag/h2d_probe.hip -- host-to-device copy rates on the box for a
// GB-sized buffer in pageable memory (as the FASTQ loader and sam2aln upload
// it): one hipMemcpyAsync, the same split over N threads each with its own
// stream, and from pinned memory (hipHostMalloc) for reference.
//   hipcc --offload-arch=gfx950 -O3 -o h2d_probe h2d_probe.hip -lpthread && ./h2d_probe [MiB]
#include <hip/hip_runtime.h>
#include <sys/mman.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <thread>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)

static double now() { return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count(); }

int main(int argc, char **argv)
{
    const size_t mib = argc > 1 ? (size_t)atol(argv[1]) : 1024;
    const size_t n = mib << 20;
    char *host = (char *)mmap(nullptr, n, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS, -1, 0);
    madvise(host, n, MADV_HUGEPAGE);
    memset(host, 7, n);
    char *dev = nullptr;
    CK(hipMalloc(&dev, n));
    hipStream_t s0;
    CK(hipStreamCreate(&s0));
    for (int rep = 0; rep < 3; ++rep) {
        double t = now();
        CK(hipMemcpyAsync(dev, host, n, hipMemcpyHostToDevice, s0));
        CK(hipStreamSynchronize(s0));
        const double one = now() - t;
        double tt[3];
        const int nts[3] = {4, 8, 16};
        for (int k = 0; k < 3; ++k) {
            const int nt = nts[k];
            std::vector<hipStream_t> st(nt);
            for (auto &x : st) hipStreamCreate(&x);
            t = now();
            std::vector<std::thread> th;
            for (int i = 0; i < nt; ++i)
                th.emplace_back([&, i]() {
                    const size_t a = n * i / nt, b = n * (i + 1) / nt;
                    hipMemcpyAsync(dev + a, host + a, b - a, hipMemcpyHostToDevice, st[i]);
                    hipStreamSynchronize(st[i]);
                });
            for (auto &x : th) x.join();
            tt[k] = now() - t;
            for (auto &x : st) hipStreamDestroy(x);
        }
        printf("{\"rep\": %d, \"MiB\": %zu, \"one_s\": %.4f, \"t4_s\": %.4f, \"t8_s\": %.4f, \"t16_s\": %.4f}\n",
               rep, mib, one, tt[0], tt[1], tt[2]);
    }
    char *pin = nullptr;
    double t = now();
    CK(hipHostMalloc((void **)&pin, n, 0));
    const double pin_alloc = now() - t;
    memcpy(pin, host, n);
    t = now();
    CK(hipMemcpyAsync(dev, pin, n, hipMemcpyHostToDevice, s0));
    CK(hipStreamSynchronize(s0));
    printf("{\"pinned_alloc_s\": %.4f, \"pinned_copy_s\": %.4f}\n", pin_alloc, now() - t);
    t = now();
    CK(hipHostRegister(host, n, 0));
    const double reg = now() - t;
    t = now();
    CK(hipMemcpyAsync(dev, host, n, hipMemcpyHostToDevice, s0));
    CK(hipStreamSynchronize(s0));
    printf("{\"register_s\": %.4f, \"registered_copy_s\": %.4f}\n", reg, now() - t);
    return 0;
}
