// kernel_boundary.hip -- the idle time between two dependent kernels on one stream
// (experiment, not the product; run under rocprofv3 --kernel-trace and read the gaps with
// tools/boundary_gaps.py).  The sort's timeline shows ~4.5 us between every pair of kernels
// (profiles/r05_v35_sort_timeline.txt); this asks whether that gap depends on what the first
// kernel wrote (a write-back of dirty L2 lines at the kernel's end) or on how the pair is
// launched:
//   tiny      a 1-block kernel after a 1-block kernel
//   wN        a 1-block kernel after a kernel that wrote N MiB (streaming stores)
//   wN-nt     the same with nontemporal stores
//   graph     the w1024 pair captured in a hipGraph and replayed
//   then 256 MiB writers back to back (20 each): plain launches; hipExtLaunchKernel with a stop
//   event per kernel (device-scope events, as libgsort's timed launches); with default
//   (system-scope) stop events; with start + stop events
//   hipcc --offload-arch=gfx950 -O3 tools/experiments/kernel_boundary.hip -o /tmp/kernel_boundary
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

#define CK(x)                                                                            \
    do {                                                                                 \
        hipError_t e = (x);                                                              \
        if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); exit(1); } \
    } while (0)

__global__ void k_tiny(unsigned *p) { if (threadIdx.x == 0) p[0] += 1; }

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
template <bool NT>
__global__ __launch_bounds__(256) void k_write(u32x4 *p, size_t n16) {
    for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < n16; i += (size_t)gridDim.x * 256) {
        u32x4 v = {(unsigned)i, 1u, 2u, 3u};
        if (NT) __builtin_nontemporal_store(v, p + i); else p[i] = v;
    }
}

int main() {
    const size_t maxb = (size_t)1 << 30;
    u32x4 *buf;
    unsigned *t;
    CK(hipMalloc(&buf, maxb));
    CK(hipMalloc(&t, 256));
    hipStream_t s;
    CK(hipStreamCreate(&s));
    const int R = 20;
    for (int r = 0; r < R; ++r) { k_tiny<<<1, 64, 0, s>>>(t); k_tiny<<<1, 64, 0, s>>>(t); }
    CK(hipStreamSynchronize(s));
    for (size_t mib : {1, 16, 64, 256, 1024}) {
        const size_t n16 = mib * (1 << 20) / 16;
        for (int r = 0; r < R; ++r) {
            k_write<false><<<2048, 256, 0, s>>>(buf, n16);
            k_tiny<<<1, 64, 0, s>>>(t);
        }
        CK(hipStreamSynchronize(s));
        for (int r = 0; r < R; ++r) {
            k_write<true><<<2048, 256, 0, s>>>(buf, n16);
            k_tiny<<<1, 64, 0, s>>>(t);
        }
        CK(hipStreamSynchronize(s));
    }
    // graph replay of the 1 GiB pair
    hipGraph_t g;
    hipGraphExec_t ge;
    CK(hipStreamBeginCapture(s, hipStreamCaptureModeGlobal));
    for (int r = 0; r < 4; ++r) {
        k_write<false><<<2048, 256, 0, s>>>(buf, maxb / 16);
        k_tiny<<<1, 64, 0, s>>>(t);
    }
    CK(hipStreamEndCapture(s, &g));
    CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
    for (int r = 0; r < 5; ++r) CK(hipGraphLaunch(ge, s));
    CK(hipStreamSynchronize(s));
    const size_t n256 = (size_t)256 * (1 << 20) / 16;
    hipEvent_t evd[64], evs[64];
    for (int i = 0; i < 64; ++i) {
        CK(hipEventCreateWithFlags(&evd[i], hipEventDisableSystemFence));
        CK(hipEventCreateWithFlags(&evs[i], 0));
    }
    for (int r = 0; r < R; ++r) k_write<false><<<2048, 256, 0, s>>>(buf, n256);
    CK(hipStreamSynchronize(s));
    for (int r = 0; r < R; ++r)
        hipExtLaunchKernelGGL(k_write<false>, dim3(2048), dim3(256), 0, s, nullptr, evd[r], 0, buf, n256);
    CK(hipStreamSynchronize(s));
    for (int r = 0; r < R; ++r)
        hipExtLaunchKernelGGL(k_write<false>, dim3(2048), dim3(256), 0, s, nullptr, evs[r], 0, buf, n256);
    CK(hipStreamSynchronize(s));
    for (int r = 0; r < R; ++r)
        hipExtLaunchKernelGGL(k_write<false>, dim3(2048), dim3(256), 0, s, evd[2 * r], evd[2 * r + 1], 0, buf, n256);
    CK(hipStreamSynchronize(s));
    printf("done\n");
    return 0;
}
