// kexp10.hip -- what a read + write pass of 2^lg keys can reach (development tool): tile copies
// in the K3u geometry (one 8192-key tile per 1024-thread workgroup) with dword or 16-B accesses
// on either side, nontemporal stores, and hipMemcpyAsync D2D for comparison.
//   run: kexp10 [log2n=28] [rounds=7]
#include <stdio.h>
#include <stdlib.h>

#include <algorithm>
#include <vector>

#include <hip/hip_runtime.h>

#define CK(x)                                                                         \
    do {                                                                              \
        hipError_t e = (x);                                                           \
        if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); exit(1); } \
    } while (0)

namespace {
constexpr int TILE = 8192;

// LOADV / STOREV: 16-B accesses (thread owns keys 4*tid.. of each 4096-key half) else dwords
template <bool LOADV, bool STOREV, bool NT>
__global__ __launch_bounds__(1024) void k_tcopy(const uint32_t *__restrict__ in,
                                                uint32_t *__restrict__ out) {
    const uint64_t t0 = (uint64_t)blockIdx.x * TILE;
    const int tid = threadIdx.x;
    uint32_t k[8];
    if (LOADV) {
        const uint4 *p = reinterpret_cast<const uint4 *>(in + t0);
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            const uint4 q = p[h * 1024 + tid];
            k[4 * h] = q.x; k[4 * h + 1] = q.y; k[4 * h + 2] = q.z; k[4 * h + 3] = q.w;
        }
    } else {
        // the same key -> register map as LOADV so both store forms are comparable
#pragma unroll
        for (int h = 0; h < 2; ++h)
#pragma unroll
            for (int j = 0; j < 4; ++j) k[4 * h + j] = in[t0 + h * 4096 + 4 * tid + j];
    }
    if (STOREV) {
        uint4 *p = reinterpret_cast<uint4 *>(out + t0);
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            const uint4 q = make_uint4(k[4 * h], k[4 * h + 1], k[4 * h + 2], k[4 * h + 3]);
            typedef unsigned int v4u __attribute__((ext_vector_type(4)));
            if (NT) {
                const v4u qv = {q.x, q.y, q.z, q.w};
                __builtin_nontemporal_store(qv, reinterpret_cast<v4u *>(&p[h * 1024 + tid]));
            } else {
                p[h * 1024 + tid] = q;
            }
        }
    } else {
#pragma unroll
        for (int h = 0; h < 2; ++h)
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                uint32_t *d = &out[t0 + h * 4096 + 4 * tid + j];
                if (NT) __builtin_nontemporal_store(k[4 * h + j], d);
                else *d = k[4 * h + j];
            }
    }
}

// coalesced dword version (lane-contiguous), as the product kernels load today
template <bool NT>
__global__ __launch_bounds__(1024) void k_tcopy_lane(const uint32_t *__restrict__ in,
                                                     uint32_t *__restrict__ out) {
    const uint64_t t0 = (uint64_t)blockIdx.x * TILE;
    uint32_t k[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) k[i] = in[t0 + i * 1024 + threadIdx.x];
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        if (NT) __builtin_nontemporal_store(k[i], &out[t0 + i * 1024 + threadIdx.x]);
        else out[t0 + i * 1024 + threadIdx.x] = k[i];
    }
}
}  // namespace

int main(int argc, char **argv) {
    const int lg = argc > 1 ? atoi(argv[1]) : 28;
    const int rounds = argc > 2 ? atoi(argv[2]) : 7;
    const uint64_t n = 1ull << lg;
    uint32_t *in, *out;
    CK(hipMalloc(&in, n * 4));
    CK(hipMalloc(&out, n * 4));
    CK(hipMemset(in, 1, n * 4));
    hipStream_t s;
    CK(hipStreamCreate(&s));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    const char *names[] = {"lane_dword",       "lane_dword_nt",   "vec_load_vec_store",
                           "vec_load_dword_store", "dword_load_vec_store", "vec_vec_nt",
                           "hipMemcpyAsync_D2D"};
    for (int v = 0; v < 7; ++v) {
        std::vector<float> t;
        for (int r = 0; r < rounds; ++r) {
            CK(hipEventRecord(e0, s));
            const int g = (int)(n / TILE);
            switch (v) {
                case 0: k_tcopy_lane<false><<<g, 1024, 0, s>>>(in, out); break;
                case 1: k_tcopy_lane<true><<<g, 1024, 0, s>>>(in, out); break;
                case 2: k_tcopy<true, true, false><<<g, 1024, 0, s>>>(in, out); break;
                case 3: k_tcopy<true, false, false><<<g, 1024, 0, s>>>(in, out); break;
                case 4: k_tcopy<false, true, false><<<g, 1024, 0, s>>>(in, out); break;
                case 5: k_tcopy<true, true, true><<<g, 1024, 0, s>>>(in, out); break;
                case 6: CK(hipMemcpyAsync(out, in, n * 4, hipMemcpyDeviceToDevice, s)); break;
            }
            CK(hipEventRecord(e1, s));
            CK(hipEventSynchronize(e1));
            float m;
            CK(hipEventElapsedTime(&m, e0, e1));
            t.push_back(m);
        }
        std::sort(t.begin(), t.end());
        const float m = t[t.size() / 2];
        printf("{\"variant\": \"%s\", \"ms\": %.4f, \"GBps\": %.1f}\n", names[v], m,
               n * 8.0 / (m * 1e-3) / 1e9);
    }
    return 0;
}
