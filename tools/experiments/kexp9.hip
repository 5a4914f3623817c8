// kexp9.hip -- persistent tile-count kernel (development tool).  The product K1 runs one
// 8192-key tile per workgroup: its loads are exposed at every workgroup start, hidden only by
// the other workgroups on the CU.  Here G workgroups walk the tiles and load tile t + G while
// counting tile t (buffer loads, double-buffered LDS histogram).  Checked against the product.
//   run: kexp9 [log2n=28] [rounds=7]
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
template <int BLOCK, bool FIN>
__global__ __launch_bounds__(BLOCK) void k1p(const uint32_t *__restrict__ in, uint64_t n,
                                             int shift, uint32_t *__restrict__ tcounts) {
    constexpr int ITEMS = kSweepTile / BLOCK;
    __shared__ uint32_t s_h[2][kRadix];
    const uint32_t tid = threadIdx.x;
    const uint32_t nt = (uint32_t)((n + kSweepTile - 1) / kSweepTile);
    const uint32_t flipd = FIN ? (0x80u >> 0) : 0u;  // the flip changes bit 31: digit 3's top bit
    uint32_t t = blockIdx.x;
    if (t >= nt) return;
    auto tile_len = [&](uint32_t tt) -> uint32_t {
        const uint64_t t0 = (uint64_t)tt * kSweepTile;
        return (uint32_t)(n - t0 < (uint64_t)kSweepTile ? n - t0 : (uint64_t)kSweepTile);
    };
    uint32_t k[ITEMS];
    {
        const __amdgpu_buffer_rsrc_t rs = bucket_rsrc(in + (uint64_t)t * kSweepTile, tile_len(t) * 4u);
#pragma unroll
        for (int i = 0; i < ITEMS; ++i)
            k[i] = __builtin_amdgcn_raw_buffer_load_b32(rs, (i * BLOCK + (int)tid) * 4, 0, 0);
    }
    for (uint32_t b = tid; b < 2 * kRadix; b += BLOCK) (&s_h[0][0])[b] = 0;
    __syncthreads();
    int buf = 0;
    for (;;) {
        const uint32_t tn = t + gridDim.x;
        uint32_t kn[ITEMS];
        if (tn < nt) {
            const __amdgpu_buffer_rsrc_t rs =
                bucket_rsrc(in + (uint64_t)tn * kSweepTile, tile_len(tn) * 4u);
#pragma unroll
            for (int i = 0; i < ITEMS; ++i)
                kn[i] = __builtin_amdgcn_raw_buffer_load_b32(rs, (i * BLOCK + (int)tid) * 4, 0, 0);
        }
        const uint32_t len = tile_len(t);
        uint32_t *h = s_h[buf];
#pragma unroll
        for (int i = 0; i < ITEMS; ++i)
            if (tid < (len > (uint32_t)(i * BLOCK) ? len - (uint32_t)(i * BLOCK) : 0u))
                atomicAdd(&h[((k[i] >> shift) & 255u) ^ (shift == 24 ? flipd : 0u)], 1u);
        __syncthreads();
        for (uint32_t b = tid; b < kRadix; b += BLOCK) {
            tcounts[(uint64_t)t * kRadix + b] = h[b];
            h[b] = 0;  // read again two tiles later, after the next barrier
        }
        if (tn >= nt) break;
        t = tn;
        buf ^= 1;
#pragma unroll
        for (int i = 0; i < ITEMS; ++i) k[i] = kn[i];
    }
}
}  // namespace

int main(int argc, char **argv) {
    const int lg = argc > 1 ? atoi(argv[1]) : 28;
    const int rounds = argc > 2 ? atoi(argv[2]) : 7;
    const uint64_t n = (1ull << lg) - 1000;  // a partial last tile
    const uint64_t nt = sweep_tiles(n);
    uint32_t *in, *tc, *tc2;
    CK(hipMalloc(&in, n * 4));
    CK(hipMalloc(&tc, nt * kRadix * 4));
    CK(hipMalloc(&tc2, nt * kRadix * 4));
    hipStream_t s;
    CK(hipStreamCreate(&s));
    CK(launch_generate(0, 42, 0, n, (int32_t *)in, s));
    std::vector<uint32_t> ref(nt * kRadix), got(nt * kRadix);
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    for (int shift : {24, 16}) {
        CK(launch_tile_counts1(in, n, shift, true, tc, s));
        CK(hipStreamSynchronize(s));
        CK(hipMemcpy(ref.data(), tc, nt * kRadix * 4, hipMemcpyDeviceToHost));
        for (int v : {0, 1, 2, 4, 8, 101, 102, 104}) {
            std::vector<float> t;
            for (int r = 0; r < rounds; ++r) {
                CK(hipMemsetAsync(tc2, 0xff, nt * kRadix * 4, s));
                CK(hipEventRecord(e0, s));
                if (v == 0) CK(launch_tile_counts1(in, n, shift, true, tc2, s));
                else if (v < 100) k1p<512, true><<<std::min<uint64_t>(nt, 256ull * v), 512, 0, s>>>(in, n, shift, tc2);
                else k1p<1024, true><<<std::min<uint64_t>(nt, 256ull * (v - 100)), 1024, 0, s>>>(in, n, shift, tc2);
                CK(hipEventRecord(e1, s));
                CK(hipEventSynchronize(e1));
                float m;
                CK(hipEventElapsedTime(&m, e0, e1));
                t.push_back(m);
            }
            CK(hipMemcpy(got.data(), tc2, nt * kRadix * 4, hipMemcpyDeviceToHost));
            if (got != ref) { printf("MISMATCH v=%d shift=%d\n", v, shift); return 1; }
            std::sort(t.begin(), t.end());
            const float m = t[t.size() / 2];
            printf("{\"shift\": %d, \"variant\": %d, \"ms\": %.4f, \"GBps\": %.1f}\n", shift, v, m,
                   n * 4.0 / (m * 1e-3) / 1e9);
        }
    }
    return 0;
}
