// kexp6.hip -- K3u tile-size experiment (development tool): 8192- vs 16384-key tiles for the
// unstable partition (count with one block per tile, the product K2 scans, kexp2's k3u).
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
template <int BLOCK, int TILE>
__global__ __launch_bounds__(BLOCK) void k1t(const uint32_t *__restrict__ in, int shift,
                                             uint32_t *__restrict__ tcounts) {
    constexpr int PER = TILE / BLOCK;
    __shared__ uint32_t h[kRadix];
    const int tid = threadIdx.x;
    for (int i = tid; i < kRadix; i += BLOCK) h[i] = 0;
    const uint32_t *src = in + (uint64_t)blockIdx.x * TILE;
    uint32_t k[PER];
#pragma unroll
    for (int i = 0; i < PER; ++i) k[i] = src[i * BLOCK + tid];
    __syncthreads();
#pragma unroll
    for (int i = 0; i < PER; ++i) atomicAdd(&h[(k[i] >> shift) & 255u], 1u);
    __syncthreads();
    for (int b = tid; b < kRadix; b += BLOCK) tcounts[(uint64_t)blockIdx.x * kRadix + b] = h[b];
}

template <int BLOCK, int ITEMS>
__global__ __launch_bounds__(BLOCK) void k3t(const uint32_t *__restrict__ in,
                                             uint32_t *__restrict__ out, uint64_t n, int shift,
                                             const uint32_t *__restrict__ toff,
                                             const unsigned long long *__restrict__ gpfx,
                                             const unsigned long long *__restrict__ bases) {
    constexpr int TILE = BLOCK * ITEMS;
    __shared__ uint32_t s_keys[TILE];
    __shared__ uint32_t s_cur[kRadix];
    __shared__ uint32_t *s_dst[kRadix];
    __shared__ uint32_t s_wsum[kRadix / 64];
    const uint32_t tile = xcd_tile(blockIdx.x, gridDim.x);
    const uint64_t t0 = (uint64_t)tile * TILE;
    const uint32_t len = (uint32_t)(n - t0 < (uint64_t)TILE ? n - t0 : (uint64_t)TILE);
    uint32_t *dst_base = nullptr;
    if (threadIdx.x < kRadix)
        dst_base = out + bases[threadIdx.x] +
                   gpfx[(uint64_t)(tile / kScanGroup) * kRadix + threadIdx.x] +
                   toff[(uint64_t)tile * kRadix + threadIdx.x];
    partition_tile<BLOCK, ITEMS, false, false>(in, t0, len, shift, dst_base, s_keys, s_cur, s_dst,
                                               s_wsum);
}

template <int BLOCK, int ITEMS>
float run(const uint32_t *in, uint32_t *out, uint64_t n, int shift, uint32_t *tc,
          unsigned long long *gs, unsigned long long *tot, unsigned long long *bases, hipStream_t s,
          float *t_count) {
    constexpr int TILE = BLOCK * ITEMS;
    const uint32_t nt = (uint32_t)(n / TILE), ng = (nt + kScanGroup - 1) / kScanGroup;
    hipEvent_t e0, e1, e2;
    CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1)); CK(hipEventCreate(&e2));
    CK(hipEventRecord(e0, s));
    k1t<512, TILE><<<nt, 512, 0, s>>>(in, shift, tc);
    k_scan_tiles<<<ng, kRadix, 0, s>>>(tc, nt, gs);
    k_scan_groups<<<kRadix, 1024, 0, s>>>(gs, ng, tot);
    k_scan_digits<<<1, kRadix, 0, s>>>(tot, bases);
    CK(hipEventRecord(e1, s));
    k3t<BLOCK, ITEMS><<<nt, BLOCK, 0, s>>>(in, out, n, shift, tc, gs, bases);
    CK(hipEventRecord(e2, s));
    CK(hipEventSynchronize(e2));
    float a, b;
    CK(hipEventElapsedTime(&a, e0, e1));
    CK(hipEventElapsedTime(&b, e1, e2));
    *t_count = a;
    return b;
}
}  // namespace

int main(int argc, char **argv) {
    const int lg = argc > 1 ? atoi(argv[1]) : 28;
    const int rounds = argc > 2 ? atoi(argv[2]) : 7;
    const uint64_t n = 1ull << lg;
    uint32_t *in, *out, *tc;
    unsigned long long *gs, *tot, *bases;
    CK(hipMalloc(&in, n * 4));
    CK(hipMalloc(&out, n * 4));
    CK(hipMalloc(&tc, (n / 4096) * kRadix * 4));
    CK(hipMalloc(&gs, (n / 4096 / kScanGroup + 1) * kRadix * 8));
    CK(hipMalloc(&tot, kRadix * 8));
    CK(hipMalloc(&bases, kRadix * 8));
    hipStream_t s;
    CK(hipStreamCreate(&s));
    CK(launch_generate(0, 42, 0, n, (int32_t *)in, s));
    CK(hipStreamSynchronize(s));
    std::vector<uint32_t> h_in(n), h_out(n);
    CK(hipMemcpy(h_in.data(), in, n * 4, hipMemcpyDeviceToHost));
    const int shift = 24;
    struct R { const char *name; std::vector<float> c, p; };
    std::vector<R> rs = {{"tile8192_b1024_i8"}, {"tile16384_b1024_i16"}, {"tile16384_b512_i32"},
                         {"tile4096_b512_i8"}};
    for (int r = 0; r < rounds; ++r) {
        for (size_t v = 0; v < rs.size(); ++v) {
            float tcnt, tp;
            if (v == 0) tp = run<1024, 8>(in, out, n, shift, tc, gs, tot, bases, s, &tcnt);
            if (v == 1) tp = run<1024, 16>(in, out, n, shift, tc, gs, tot, bases, s, &tcnt);
            if (v == 2) tp = run<512, 32>(in, out, n, shift, tc, gs, tot, bases, s, &tcnt);
            if (v == 3) tp = run<512, 8>(in, out, n, shift, tc, gs, tot, bases, s, &tcnt);
            rs[v].c.push_back(tcnt);
            rs[v].p.push_back(tp);
            if (r == 0) {
                CK(hipMemcpy(h_out.data(), out, n * 4, hipMemcpyDeviceToHost));
                uint64_t bad = 0;
                for (uint64_t i = 1; i < n; ++i)
                    if ((h_out[i] >> shift) < (h_out[i - 1] >> shift)) ++bad;
                std::vector<uint32_t> a(h_in), b(h_out);
                std::sort(a.begin(), a.end());
                std::sort(b.begin(), b.end());
                if (bad || a != b) { printf("FAIL %s\n", rs[v].name); return 1; }
            }
        }
    }
    for (auto &x : rs) {
        std::sort(x.c.begin(), x.c.end());
        std::sort(x.p.begin(), x.p.end());
        printf("{\"variant\": \"%s\", \"count_scan_ms\": %.4f, \"partition_ms\": %.4f}\n", x.name,
               x.c[x.c.size() / 2], x.p[x.p.size() / 2]);
    }
    return 0;
}
