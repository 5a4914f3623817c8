// kexp4.hip -- tile-count (K1 / K1s) kernel experiments (development tool).
// All variants write tcounts[tile][256] for kSweepTile-key tiles of 2^lg keys and are checked
// against the product K1.
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
// one block per tile; dword loads block-strided (VEC=false) or uint4 loads (VEC=true);
// SUB > 1: SUB interleaved sub-histograms (bin*SUB + lane%SUB) to spread same-bin lanes
template <int BLOCK, bool VEC, int SUB>
__global__ __launch_bounds__(BLOCK) void k1x(const uint32_t *__restrict__ in, int shift,
                                             uint32_t *__restrict__ tcounts) {
    constexpr int PER = kSweepTile / BLOCK;
    __shared__ uint32_t h[kRadix * SUB];
    const int tid = threadIdx.x;
    for (int i = tid; i < kRadix * SUB; i += BLOCK) h[i] = 0;
    const uint32_t t = blockIdx.x;
    const uint32_t *src = in + (uint64_t)t * kSweepTile;
    uint32_t k[PER];
    if (VEC) {
        const uint4 *p = reinterpret_cast<const uint4 *>(src);
#pragma unroll
        for (int j = 0; j < PER / 4; ++j) {
            const uint4 q = p[j * BLOCK + tid];
            k[4 * j] = q.x; k[4 * j + 1] = q.y; k[4 * j + 2] = q.z; k[4 * j + 3] = q.w;
        }
    } else {
#pragma unroll
        for (int i = 0; i < PER; ++i) k[i] = src[i * BLOCK + tid];
    }
    __syncthreads();
    const uint32_t sub = SUB > 1 ? (tid % SUB) : 0;
#pragma unroll
    for (int i = 0; i < PER; ++i) atomicAdd(&h[((k[i] >> shift) & 255u) * SUB + sub], 1u);
    __syncthreads();
    for (int b = tid; b < kRadix; b += BLOCK) {
        uint32_t c = 0;
#pragma unroll
        for (int j = 0; j < SUB; ++j) c += h[b * SUB + j];
        tcounts[(uint64_t)t * kRadix + b] = c;
    }
}
}  // namespace

int main(int argc, char **argv) {
    const int lg = argc > 1 ? atoi(argv[1]) : 28;
    const int rounds = argc > 2 ? atoi(argv[2]) : 7;
    const uint64_t n = 1ull << lg;
    const uint64_t nt = sweep_tiles(n);
    uint32_t *in, *tc, *tc2;
    CK(hipMalloc(&in, n * 4));
    CK(hipMalloc(&tc, nt * kRadix * 4));
    CK(hipMalloc(&tc2, nt * kRadix * 4));
    hipStream_t s;
    CK(hipStreamCreate(&s));
    CK(launch_generate(0, 42, 0, n, (int32_t *)in, s));
    const int shift = 16;
    CK(launch_tile_counts(in, n, shift, false, tc, nullptr, s));
    CK(hipStreamSynchronize(s));
    std::vector<uint32_t> ref(nt * kRadix), got(nt * kRadix);
    CK(hipMemcpy(ref.data(), tc, nt * kRadix * 4, hipMemcpyDeviceToHost));
    struct V { const char *name; int id; std::vector<float> t; };
    std::vector<V> vs = {{"prod_k1", 0}, {"k1x_b256_dword", 1}, {"k1x_b256_vec", 2},
                         {"k1x_b512_dword", 3}, {"k1x_b512_vec", 4}, {"k1x_b256_vec_sub4", 5},
                         {"k1x_b1024_vec", 6}};
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    for (int r = 0; r < rounds; ++r) {
        for (auto &v : vs) {
            CK(hipEventRecord(e0, s));
            switch (v.id) {
                case 0: CK(launch_tile_counts(in, n, shift, false, tc2, nullptr, s)); break;
                case 1: k1x<256, false, 1><<<nt, 256, 0, s>>>(in, shift, tc2); break;
                case 2: k1x<256, true, 1><<<nt, 256, 0, s>>>(in, shift, tc2); break;
                case 3: k1x<512, false, 1><<<nt, 512, 0, s>>>(in, shift, tc2); break;
                case 4: k1x<512, true, 1><<<nt, 512, 0, s>>>(in, shift, tc2); break;
                case 5: k1x<256, true, 4><<<nt, 256, 0, s>>>(in, shift, tc2); break;
                case 6: k1x<1024, true, 1><<<nt, 1024, 0, s>>>(in, shift, tc2); break;
            }
            CK(hipEventRecord(e1, s));
            CK(hipEventSynchronize(e1));
            float m;
            CK(hipEventElapsedTime(&m, e0, e1));
            v.t.push_back(m);
            if (r == 0) {
                CK(hipMemcpy(got.data(), tc2, nt * kRadix * 4, hipMemcpyDeviceToHost));
                if (got != ref) { printf("MISMATCH %s\n", v.name); return 1; }
            }
        }
    }
    for (auto &v : vs) {
        std::sort(v.t.begin(), v.t.end());
        const float m = v.t[v.t.size() / 2];
        printf("{\"variant\": \"%s\", \"ms\": %.4f, \"GBps\": %.1f}\n", v.name, m,
               n * 4.0 / (m * 1e-3) / 1e9);
    }
    return 0;
}
