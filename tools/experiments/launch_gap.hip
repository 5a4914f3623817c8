// launch_gap.hip -- idle time between dependent kernels on one stream for each way of timing
// them (experiment, not the product): 200 small kernels back to back,
//   plain       k<<<...>>>
//   ext-null    hipExtLaunchKernelGGL without events
//   ext-events  hipExtLaunchKernelGGL with a start + stop event per kernel
//   record      hipEventRecord before and after every kernel
//   record-nf   the same with hipEventDisableSystemFence events
//   hipcc --offload-arch=gfx950 -O3 tools/experiments/launch_gap.hip -o launch_gap
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

#include <vector>

#define CK(x)                                                                            \
    do {                                                                                 \
        hipError_t e = (x);                                                              \
        if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); exit(1); } \
    } while (0)

__global__ void k_spin(unsigned *p, unsigned n) {
    unsigned v = p[blockIdx.x * blockDim.x + threadIdx.x];
    for (unsigned i = 0; i < n; ++i) v = v * 1664525u + 1013904223u;
    p[blockIdx.x * blockDim.x + threadIdx.x] = v;
}

int main() {
    const int K = 200, G = 1024, B = 256;
    const unsigned work = 2000;  // a few us per kernel
    unsigned *p;
    CK(hipMalloc(&p, G * B * 4));
    CK(hipMemset(p, 0, G * B * 4));
    hipStream_t s;
    CK(hipStreamCreate(&s));
    std::vector<hipEvent_t> ev(2 * K), evnf(2 * K);
    for (auto &x : ev) CK(hipEventCreate(&x));
    for (auto &x : evnf) CK(hipEventCreateWithFlags(&x, hipEventDisableSystemFence));
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    auto time = [&](const char *name, auto body) {
        float best = 1e30f;
        for (int r = 0; r < 5; ++r) {
            CK(hipStreamSynchronize(s));
            CK(hipEventRecord(a, s));
            body();
            CK(hipEventRecord(b, s));
            CK(hipEventSynchronize(b));
            float ms;
            CK(hipEventElapsedTime(&ms, a, b));
            if (ms < best) best = ms;
        }
        printf("%-12s %8.2f us per kernel\n", name, best * 1e3f / K);
        fflush(stdout);
    };
    time("plain", [&] { for (int i = 0; i < K; ++i) k_spin<<<G, B, 0, s>>>(p, work); });
    time("ext-null", [&] {
        for (int i = 0; i < K; ++i)
            hipExtLaunchKernelGGL(k_spin, dim3(G), dim3(B), 0, s, nullptr, nullptr, 0, p, work);
    });
    time("ext-stop", [&] {
        for (int i = 0; i < K; ++i)
            hipExtLaunchKernelGGL(k_spin, dim3(G), dim3(B), 0, s, nullptr, ev[2 * i + 1], 0, p,
                                  work);
    });
    time("ext-events", [&] {
        for (int i = 0; i < K; ++i)
            hipExtLaunchKernelGGL(k_spin, dim3(G), dim3(B), 0, s, ev[2 * i], ev[2 * i + 1], 0, p,
                                  work);
    });
    time("record", [&] {
        for (int i = 0; i < K; ++i) {
            CK(hipEventRecord(ev[2 * i], s));
            k_spin<<<G, B, 0, s>>>(p, work);
            CK(hipEventRecord(ev[2 * i + 1], s));
        }
    });
    time("record-nf", [&] {
        for (int i = 0; i < K; ++i) {
            CK(hipEventRecord(evnf[2 * i], s));
            k_spin<<<G, B, 0, s>>>(p, work);
            CK(hipEventRecord(evnf[2 * i + 1], s));
        }
    });
    time("plain", [&] { for (int i = 0; i < K; ++i) k_spin<<<G, B, 0, s>>>(p, work); });
    return 0;
}
