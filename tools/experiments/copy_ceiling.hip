// copy_ceiling.hip -- what a read + write pass over HBM reaches on MI355X (experiment, not the
// product): streaming-copy variants over 1 GiB (the bench's 2^28 int32 keys), best-of-reps
// time per variant.  The product's gsort_copy_ceiling uses the winner.
//   hipcc --offload-arch=gfx950 -O3 tools/experiments/copy_ceiling.hip -o /tmp/copy_ceiling
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#include <algorithm>
#include <vector>

typedef unsigned int v4u __attribute__((ext_vector_type(4)));
#define uint4 v4u

#define CK(x)                                                                        \
    do {                                                                             \
        hipError_t e_ = (x);                                                         \
        if (e_ != hipSuccess) {                                                      \
            fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));                  \
            exit(2);                                                                 \
        }                                                                            \
    } while (0)

// grid-strided, U uint4 per thread in flight, optional nontemporal load/store
template <int U, bool NTL, bool NTS>
__global__ __launch_bounds__(256) void k_strided(const uint4 *__restrict__ in,
                                                 uint4 *__restrict__ out, uint64_t n16) {
    const uint64_t stride = (uint64_t)gridDim.x * 256;
    uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    for (; i + (U - 1) * stride < n16; i += U * stride) {
        uint4 v[U];
#pragma unroll
        for (int u = 0; u < U; ++u)
            v[u] = NTL ? __builtin_nontemporal_load(in + i + u * stride) : in[i + u * stride];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            if (NTS) __builtin_nontemporal_store(v[u], out + i + u * stride);
            else out[i + u * stride] = v[u];
        }
    }
    for (; i < n16; i += stride) out[i] = in[i];
}

// one block per contiguous chunk of CH uint4 (block-contiguous, U in flight per thread)
template <int U, int B, bool NTS>
__global__ __launch_bounds__(B) void k_chunk(const uint4 *__restrict__ in,
                                             uint4 *__restrict__ out, uint64_t n16) {
    constexpr uint64_t CH = (uint64_t)U * B;
    const uint64_t base = (uint64_t)blockIdx.x * CH;
    uint4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
        const uint64_t j = base + u * B + threadIdx.x;
        if (j < n16) v[u] = in[j];
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
        const uint64_t j = base + u * B + threadIdx.x;
        if (j < n16) {
            if (NTS) __builtin_nontemporal_store(v[u], out + j);
            else out[j] = v[u];
        }
    }
}

int main(int argc, char **argv) {
    const size_t bytes = (argc > 1 ? strtoull(argv[1], nullptr, 0) : (1ull << 30));
    const int reps = 12;
    const uint64_t n16 = bytes / 16;
    uint4 *a, *b;
    CK(hipMalloc(&a, bytes));
    CK(hipMalloc(&b, bytes));
    CK(hipMemset(a, 1, bytes));
    CK(hipMemset(b, 2, bytes));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    auto time = [&](const char *name, auto launch) {
        std::vector<float> t;
        for (int r = 0; r < reps + 2; ++r) {
            CK(hipEventRecord(e0, 0));
            launch();
            CK(hipEventRecord(e1, 0));
            CK(hipEventSynchronize(e1));
            float ms;
            CK(hipEventElapsedTime(&ms, e0, e1));
            if (r >= 2) t.push_back(ms);
        }
        std::sort(t.begin(), t.end());
        printf("%-40s min %.4f ms (%.0f GB/s)  median %.4f ms (%.0f GB/s)\n", name, t[0],
               2.0 * bytes / (t[0] * 1e-3) / 1e9, t[t.size() / 2],
               2.0 * bytes / (t[t.size() / 2] * 1e-3) / 1e9);
    };
    char nm[128];
    for (unsigned g : {1024u, 2048u, 4096u, 8192u, 16384u, 32768u}) {
        snprintf(nm, sizeof nm, "strided U4 g%u", g);
        time(nm, [&] { k_strided<4, false, false><<<g, 256>>>(a, b, n16); });
        snprintf(nm, sizeof nm, "strided U8 g%u", g);
        time(nm, [&] { k_strided<8, false, false><<<g, 256>>>(a, b, n16); });
        snprintf(nm, sizeof nm, "strided U4 nt-store g%u", g);
        time(nm, [&] { k_strided<4, false, true><<<g, 256>>>(a, b, n16); });
        snprintf(nm, sizeof nm, "strided U4 nt-load+store g%u", g);
        time(nm, [&] { k_strided<4, true, true><<<g, 256>>>(a, b, n16); });
    }
    {
        const unsigned g = (unsigned)((n16 + 4 * 256 - 1) / (4 * 256));
        time("chunk U4 B256", [&] { k_chunk<4, 256, false><<<g, 256>>>(a, b, n16); });
        time("chunk U4 B256 nt-store", [&] { k_chunk<4, 256, true><<<g, 256>>>(a, b, n16); });
    }
    {
        const unsigned g = (unsigned)((n16 + 8 * 256 - 1) / (8 * 256));
        time("chunk U8 B256", [&] { k_chunk<8, 256, false><<<g, 256>>>(a, b, n16); });
        time("chunk U8 B256 nt-store", [&] { k_chunk<8, 256, true><<<g, 256>>>(a, b, n16); });
    }
    {
        const unsigned g = (unsigned)((n16 + 2 * 1024 - 1) / (2 * 1024));
        time("chunk U2 B1024", [&] { k_chunk<2, 1024, false><<<g, 1024>>>(a, b, n16); });
    }
    time("hipMemcpyAsync D2D", [&] { CK(hipMemcpyAsync(b, a, bytes, hipMemcpyDeviceToDevice, 0)); });
    // read-only reference: the same bytes read, no write
    return 0;
}
