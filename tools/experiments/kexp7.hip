// kexp7.hip -- Infinity Cache (256 MiB) reuse experiment for the count -> partition pair
// (development tool).  Level 3 of the MSD sort reads the input twice (K1 counts, then K3u);
// done in C chunks of n/C keys, the K3u of a chunk re-reads what its K1 just read.  Times the
// whole pair and each kernel class for C = 1, 2, 4, 8, 16 (caches flushed before every rep).
//   run: kexp7 [log2n=28] [rounds=5]
#include <stdio.h>
#include <stdlib.h>

#include <algorithm>
#include <vector>

#include "../csrc/gsort_kernels.hip"

using namespace gsort;

#define CK(x)                                                                         \
    do {                                                                              \
        hipError_t e = (x);                                                           \
        if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); exit(1); } \
    } while (0)

namespace {
// idealised K3u writes: tile t's key idx = b*32 + j goes to bucket b's run of tile t
__global__ __launch_bounds__(1024) void k_runs(const uint32_t *__restrict__ in,
                                               uint32_t *__restrict__ out, uint64_t n) {
    const uint64_t t = blockIdx.x, per_bucket = n / 256;
    uint32_t k[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) k[i] = in[t * 8192 + i * 1024 + threadIdx.x];
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        const uint32_t idx = i * 1024 + threadIdx.x;
        out[(idx >> 5) * per_bucket + t * 32 + (idx & 31)] = k[i];
    }
}
__global__ __launch_bounds__(1024) void k_tilecopy(const uint32_t *__restrict__ in,
                                                   uint32_t *__restrict__ out) {
    const uint64_t t = blockIdx.x;
    uint32_t k[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) k[i] = in[t * 8192 + i * 1024 + threadIdx.x];
#pragma unroll
    for (int i = 0; i < 8; ++i) out[t * 8192 + i * 1024 + threadIdx.x] = k[i];
}
}  // namespace

int main(int argc, char **argv) {
    const int lg = argc > 1 ? atoi(argv[1]) : 28;
    const int rounds = argc > 2 ? atoi(argv[2]) : 5;
    const uint64_t n = 1ull << lg;
    uint32_t *in, *out, *tc, *flush;
    uint64_t *gsum, *small;
    CK(hipMalloc(&in, n * 4));
    CK(hipMalloc(&out, n * 4));
    CK(hipMalloc(&tc, sweep_tiles(n) * kRadix * 4));
    CK(hipMalloc(&gsum, scan_groups(n) * kRadix * 8));
    CK(hipMalloc(&small, 2 * kRadix * 8));
    const size_t flush_bytes = 768ull << 20;
    CK(hipMalloc(&flush, flush_bytes));
    hipStream_t s;
    CK(hipStreamCreate(&s));
    CK(launch_generate(0, 42, 0, n, (int32_t *)in, s));
    std::vector<hipEvent_t> ev(64);
    for (auto &evt : ev) CK(hipEventCreate(&evt));
    for (int v = 0; v < 3; ++v) {
        std::vector<float> t;
        for (int r = 0; r < rounds; ++r) {
            CK(hipMemsetAsync(flush, r & 255, flush_bytes, s));
            CK(hipEventRecord(ev[0], s));
            if (v == 0) CK(launch_copy(in, out, n, s));
            else if (v == 1) k_tilecopy<<<n / 8192, 1024, 0, s>>>(in, out);
            else k_runs<<<n / 8192, 1024, 0, s>>>(in, out, n);
            CK(hipEventRecord(ev[1], s));
            CK(hipEventSynchronize(ev[1]));
            float x;
            CK(hipEventElapsedTime(&x, ev[0], ev[1]));
            t.push_back(x);
        }
        std::sort(t.begin(), t.end());
        const char *nm[] = {"k_copy", "tilecopy_1024x8", "runs_of_32"};
        printf("{\"calib\": \"%s\", \"ms\": %.4f, \"GBps\": %.1f}\n", nm[v], t[t.size() / 2],
               n * 8.0 / (t[t.size() / 2] * 1e-3) / 1e9);
    }
    for (int C : {1, 4, 16}) {
        const uint64_t m = n / C;
        std::vector<float> tot, tk1, tk3;
        for (int r = 0; r < rounds; ++r) {
            CK(hipMemsetAsync(flush, r & 255, flush_bytes, s));
            CK(hipEventRecord(ev[0], s));
            for (int c = 0; c < C; ++c) {
                const uint32_t *src = in + c * m;
                CK(launch_tile_counts1(src, m, 24, true, tc, s));
                CK(launch_scan_tiles(tc, m, gsum, small, small + kRadix, s));
                CK(hipEventRecord(ev[1 + 2 * (c % 31)], s));
                CK(launch_partition(src, out + c * m, m, 24, tc, gsum, small + kRadix, true, s));
                CK(hipEventRecord(ev[2 + 2 * (c % 31)], s));
                if (C > 16) CK(hipEventSynchronize(ev[2 + 2 * (c % 31)]));
            }
            CK(hipEventRecord(ev[63], s));
            CK(hipEventSynchronize(ev[63]));
            float all;
            CK(hipEventElapsedTime(&all, ev[0], ev[63]));
            tot.push_back(all);
            if (C <= 16) {
                float k3 = 0;
                for (int c = 0; c < C; ++c) {
                    float x;
                    CK(hipEventElapsedTime(&x, ev[1 + 2 * c], ev[2 + 2 * c]));
                    k3 += x;
                }
                tk3.push_back(k3);
                tk1.push_back(all - k3);
            }
        }
        auto med = [](std::vector<float> v) {
            if (v.empty()) return -1.0f;
            std::sort(v.begin(), v.end());
            return v[v.size() / 2];
        };
        printf("{\"chunks\": %d, \"chunk_MiB\": %.0f, \"ms_pair\": %.4f, \"ms_count_scan\": %.4f, "
               "\"ms_partition\": %.4f}\n",
               C, m * 4.0 / (1 << 20), med(tot), med(tk1), med(tk3));
    }
    return 0;
}
