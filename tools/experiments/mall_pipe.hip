// mall_pipe.hip -- does the 256 MiB Infinity Cache absorb a pass's intermediate buffer?
// (experiment, not the product).  The local sort writes and re-reads an intermediate array
// between level 2 (K3a) and the bucket sorts (K11).  If that array is a small ring reused chunk
// by chunk, its lines may be re-read and overwritten while still on-die, so HBM sees only the
// first read and the last write.  Measured here with streaming copies over 1 GiB:
//   direct   src -> dst                                  (one read + write pass)
//   via HBM  src -> tmp (1 GiB) -> dst                   (two passes)
//   ring C   per chunk c: src[c] -> ring[c % 2], ring[c % 2] -> dst[c]
//   hipcc --offload-arch=gfx950 -O3 tools/experiments/mall_pipe.hip -o /tmp/mall_pipe
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#include <algorithm>
#include <vector>

typedef unsigned int v4u __attribute__((ext_vector_type(4)));

#define CK(x)                                                               \
    do {                                                                    \
        hipError_t e_ = (x);                                                \
        if (e_ != hipSuccess) {                                             \
            fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));         \
            exit(2);                                                        \
        }                                                                   \
    } while (0)

// one block per contiguous 16 KiB chunk (4 uint4 per thread in flight)
template <bool NTS>
__global__ __launch_bounds__(256) void k_chunk(const v4u *__restrict__ in, v4u *__restrict__ out,
                                               uint64_t n16) {
    const uint64_t base = (uint64_t)blockIdx.x * 1024;
    v4u v[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
        const uint64_t j = base + u * 256 + threadIdx.x;
        if (j < n16) v[u] = in[j];
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
        const uint64_t j = base + u * 256 + threadIdx.x;
        if (j < n16) {
            if (NTS) __builtin_nontemporal_store(v[u], out + j);
            else out[j] = v[u];
        }
    }
}

__global__ __launch_bounds__(256) void k_read(const v4u *__restrict__ in, uint64_t n16,
                                              unsigned *sink) {
    const uint64_t base = (uint64_t)blockIdx.x * 1024;
    unsigned acc = 0;
#pragma unroll
    for (int u = 0; u < 4; ++u) {
        const uint64_t j = base + u * 256 + threadIdx.x;
        if (j < n16) { v4u v = in[j]; acc ^= v.x ^ v.y ^ v.z ^ v.w; }
    }
    if (acc == 0x12345678u) sink[0] = acc;
}

static void copy(const void *a, void *b, size_t bytes, bool nts, hipStream_t s) {
    const uint64_t n16 = bytes / 16;
    const unsigned g = (unsigned)((n16 + 1023) / 1024);
    if (nts) k_chunk<true><<<g, 256, 0, s>>>((const v4u *)a, (v4u *)b, n16);
    else k_chunk<false><<<g, 256, 0, s>>>((const v4u *)a, (v4u *)b, n16);
}

int main(int argc, char **argv) {
    const size_t bytes = argc > 1 ? strtoull(argv[1], nullptr, 0) : (1ull << 30);
    const int reps = 10;
    char *src, *dst, *tmp;
    unsigned *sink;
    CK(hipMalloc(&src, bytes));
    CK(hipMalloc(&dst, bytes));
    CK(hipMalloc(&tmp, bytes));
    CK(hipMalloc(&sink, 64));
    CK(hipMemset(src, 1, bytes));
    CK(hipMemset(dst, 2, bytes));
    CK(hipMemset(tmp, 3, bytes));
    hipStream_t s;
    CK(hipStreamCreate(&s));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    auto time = [&](const char *name, auto launch) {
        std::vector<float> t;
        for (int r = 0; r < reps + 2; ++r) {
            CK(hipEventRecord(e0, s));
            launch();
            CK(hipEventRecord(e1, s));
            CK(hipEventSynchronize(e1));
            float ms;
            CK(hipEventElapsedTime(&ms, e0, e1));
            if (r >= 2) t.push_back(ms);
        }
        std::sort(t.begin(), t.end());
        printf("%-44s min %.4f  median %.4f ms  (%.0f GB/s of src+dst at median)\n", name, t[0],
               t[t.size() / 2], 2.0 * bytes / (t[t.size() / 2] * 1e-3) / 1e9);
        fflush(stdout);
    };
    time("read only", [&] {
        k_read<<<(unsigned)((bytes / 16 + 1023) / 1024), 256, 0, s>>>((const v4u *)src, bytes / 16, sink);
    });
    time("direct src->dst", [&] { copy(src, dst, bytes, false, s); });
    time("direct src->dst nt", [&] { copy(src, dst, bytes, true, s); });
    time("via HBM src->tmp->dst", [&] {
        copy(src, tmp, bytes, false, s);
        copy(tmp, dst, bytes, false, s);
    });
    char nm[96];
    for (size_t mib : {8, 16, 32, 64, 96, 128}) {
        const size_t C = mib << 20;
        for (int mode = 0; mode < 3; ++mode) {
            // mode 0: plain stores everywhere; 1: nt store of dst; 2: nt store of ring and dst
            snprintf(nm, sizeof nm, "ring %zu MiB x2 %s", mib,
                     mode == 0 ? "plain" : mode == 1 ? "dst-nt" : "all-nt");
            time(nm, [&] {
                for (size_t off = 0, c = 0; off < bytes; off += C, ++c) {
                    const size_t len = std::min(C, bytes - off);
                    char *ring = tmp + (c & 1) * C;
                    copy(src + off, ring, len, mode == 2, s);
                    copy(ring, dst + off, len, mode >= 1, s);
                }
            });
        }
        // no reuse: chunked through the whole 1 GiB tmp (every chunk a fresh range)
        snprintf(nm, sizeof nm, "chunked %zu MiB, fresh tmp", mib);
        time(nm, [&] {
            for (size_t off = 0; off < bytes; off += C) {
                const size_t len = std::min(C, bytes - off);
                copy(src + off, tmp + off, len, false, s);
                copy(tmp + off, dst + off, len, false, s);
            }
        });
    }
    return 0;
}
