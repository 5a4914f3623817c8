// kexp14.hip -- what bounds K11 (k_local_sort: a ~8K-key bucket sorted on its low two digits in
// LDS)?  (experiment, not the product).  2^28 random keys in buckets of 7500..9216 keys (class
// 2: 512 threads x 18 keys, the uniform 2^28 sort's level-2 children), timed as
//   product    launch_local_sort from gsort_kernels.hip
//   copy       the same load + buffer store with one LDS round trip (no sort)
//   noload     keys made in registers + sort + store
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/experiments/kexp14.hip -o kexp14
#include <stdio.h>
#include <stdlib.h>

#include <algorithm>
#include <random>
#include <vector>

#include "../../mpi-test_amd/csrc/gsort_kernels.hip"

using namespace gsort;

#define CK(x)                                                                            \
    do {                                                                                 \
        hipError_t e_ = (x);                                                             \
        if (e_ != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e_)); exit(1); } \
    } while (0)

namespace {
constexpr int BLOCK = 512, ITEMS = 18, TILE = BLOCK * ITEMS, WAVES = BLOCK / 64;

// V: 0 copy, 1 product body, 2 noload
template <int V>
__global__ __launch_bounds__(BLOCK) void k11x(const uint32_t *__restrict__ in,
                                              uint32_t *__restrict__ out,
                                              const unsigned long long *__restrict__ list) {
    __shared__ uint32_t s_a[TILE];
    __shared__ uint32_t s_wc[WAVES * kRadix];
    const uint64_t start = list[2 * blockIdx.x];
    const uint32_t len = (uint32_t)list[2 * blockIdx.x + 1];
    if (threadIdx.x < kRadix) s_wc[threadIdx.x] = 0;
    uint32_t k[ITEMS];
    if (V == 2) {
#pragma unroll
        for (int i = 0; i < ITEMS; ++i) {
            uint32_t z = (uint32_t)(start + i * BLOCK + threadIdx.x) * 0x9E3779B9u;
            z ^= z >> 15; z *= 0x85EBCA6Bu; z ^= z >> 13;
            k[i] = z;
        }
    } else {
        load_bucket<BLOCK, ITEMS, false>(in + start, len, k);
    }
    __syncthreads();
    if (V == 0) {
#pragma unroll
        for (int i = 0; i < ITEMS; ++i) s_a[i * BLOCK + threadIdx.x] = k[i];
        __syncthreads();
        const __amdgpu_buffer_rsrc_t rs = bucket_rsrc(out + start, len * 4u);
#pragma unroll
        for (int i = 0; i < ITEMS; ++i) {
            const uint32_t j = (uint32_t)(i * BLOCK + threadIdx.x);
            __builtin_amdgcn_raw_buffer_store_b32(s_a[(j * 67) % TILE] ^ kFlip, rs, (int)(j * 4u), 0, 0);
        }
        return;
    }
    sort_bucket<BLOCK, ITEMS, true>(k, len, 2, out + start, s_a, s_wc);
}

}  // namespace

int main() {
    const uint64_t n = 1ull << 28;
    uint32_t *in, *out;
    CK(hipMalloc(&in, n * 4));
    CK(hipMalloc(&out, n * 4));
    CK(launch_generate(0, 42, 0, n, reinterpret_cast<int32_t *>(in), 0));
    std::mt19937_64 rng(1);
    std::vector<unsigned long long> h;
    for (uint64_t a = 0; a < n;) {
        uint64_t len = 7500 + rng() % (9216 - 7500 + 1);
        len = std::min<uint64_t>(len, n - a);
        h.push_back(a);
        h.push_back(len);
        a += len;
    }
    const uint32_t nlist = (uint32_t)(h.size() / 2);
    unsigned long long *list;
    CK(hipMalloc(&list, h.size() * 8));
    CK(hipMemcpy(list, h.data(), h.size() * 8, hipMemcpyHostToDevice));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    auto time = [&](const char *name, auto launch) {
        std::vector<float> t;
        for (int r = 0; r < 12; ++r) {
            CK(hipEventRecord(e0, 0));
            launch();
            CK(hipEventRecord(e1, 0));
            CK(hipEventSynchronize(e1));
            float ms;
            CK(hipEventElapsedTime(&ms, e0, e1));
            if (r >= 2) t.push_back(ms);
        }
        std::sort(t.begin(), t.end());
        printf("%-12s median %.4f ms  min %.4f  (%.0f GB/s r+w)\n", name, t[t.size() / 2], t[0],
               n * 8.0 / (t[t.size() / 2] * 1e-3) / 1e9);
        fflush(stdout);
    };
    printf("%u buckets\n", nlist);
    time("product", [&] {
        CK(launch_local_sort(in, out, reinterpret_cast<const uint64_t *>(list), nlist, 2, 2, false,
                             true, 0));
    });
    // check one bucket is sorted on its low 16 bits
    {
        std::vector<uint32_t> o(h[1]);
        CK(hipMemcpy(o.data(), out, o.size() * 4, hipMemcpyDeviceToHost));
        bool ok = true;
        for (size_t i = 1; i < o.size(); ++i) ok &= (o[i - 1] & 0xffff) <= (o[i] & 0xffff);
        printf("bucket 0 sorted on 16 bits: %d\n", ok);
    }
    time("copy", [&] { k11x<0><<<nlist, BLOCK>>>(in, out, list); });
    time("noload", [&] { k11x<2><<<nlist, BLOCK>>>(in, out, list); });
    time("product2", [&] { k11x<1><<<nlist, BLOCK>>>(in, out, list); });
    return 0;
}
