// kexp8.hip -- K11 with the next bucket prefetched into registers (development tool).
// The product K11 holds one bucket per workgroup: its loads, its LDS passes and its stores run
// back to back, and only the other workgroups on the CU overlap them.  Here a grid of G
// workgroups walks the bucket list and issues the loads of its next bucket before sorting the
// current one.  Equal buckets of `bsize` keys, 2 digits, checked against the product K11.
//   run: kexp8 [log2n=28] [rounds=7]
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
template <int BLOCK, int ITEMS, int WPE>
__global__ __launch_bounds__(BLOCK) __attribute__((amdgpu_waves_per_eu(WPE, WPE))) void k11pf(const uint32_t *__restrict__ in,
                                               uint32_t *__restrict__ out,
                                               const unsigned long long *__restrict__ list,
                                               uint32_t nlist, int ndigits) {
    constexpr int WAVES = BLOCK / 64;
    constexpr int TILE = BLOCK * ITEMS;
    __shared__ uint32_t s_a[TILE];
    __shared__ uint32_t s_wc[WAVES * kRadix];
    uint32_t b = blockIdx.x;
    uint64_t start = list[2 * b];
    uint32_t len = (uint32_t)list[2 * b + 1];
    uint32_t k[ITEMS];
    load_tile<BLOCK, ITEMS, false>(in + start + threadIdx.x, len == (uint32_t)TILE, len, k);
    for (;;) {
        const uint32_t nb = b + gridDim.x;
        uint64_t nstart = 0;
        uint32_t nlen = 0;
        uint32_t kn[ITEMS];
        if (nb < nlist) {
            nstart = list[2 * nb];
            nlen = (uint32_t)list[2 * nb + 1];
            load_tile<BLOCK, ITEMS, false>(in + nstart + threadIdx.x, nlen == (uint32_t)TILE,
                                           nlen, kn);
        }
        if (threadIdx.x < kRadix) s_wc[threadIdx.x] = 0;
        __syncthreads();
        sort_bucket<BLOCK, ITEMS, true>(k, len, ndigits, out + start, s_a, s_wc);
        if (nb >= nlist) break;
        b = nb;
        start = nstart;
        len = nlen;
#pragma unroll
        for (int i = 0; i < ITEMS; ++i) k[i] = kn[i];
    }
}
}  // namespace

int main(int argc, char **argv) {
    const int lg = argc > 1 ? atoi(argv[1]) : 28;
    const int rounds = argc > 2 ? atoi(argv[2]) : 7;
    const uint64_t n = 1ull << lg;
    uint32_t *in, *out, *ref;
    unsigned long long *list;
    CK(hipMalloc(&in, n * 4));
    CK(hipMalloc(&out, n * 4));
    CK(hipMalloc(&ref, n * 4));
    CK(hipMalloc(&list, (n / 1024) * 16));
    hipStream_t s;
    CK(hipStreamCreate(&s));
    CK(launch_generate(0, 42, 0, n, (int32_t *)in, s));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    std::vector<uint32_t> h_ref(n), h_out(n);
    for (uint64_t bsize : {8192ull, 4096ull}) {
        const uint64_t nb = n / bsize;
        std::vector<unsigned long long> hl(2 * nb);
        for (uint64_t b = 0; b < nb; ++b) { hl[2 * b] = b * bsize; hl[2 * b + 1] = bsize - (b % 3); }
        CK(hipMemcpy(list, hl.data(), nb * 16, hipMemcpyHostToDevice));
        const int cls = local_class(bsize);
        for (int grid_mult : {0}) {
            std::vector<float> t;
            for (int r = 0; r < rounds; ++r) {
                CK(hipEventRecord(e0, s));
                if (grid_mult == 0) {
                    CK(launch_local_sort(in, out, reinterpret_cast<const uint64_t *>(list),
                                         (uint32_t)nb, cls, 2, false, true, s));
                } else {
                    const uint32_t G = std::min<uint64_t>(nb, 256ull * (grid_mult % 100));
                    if (grid_mult > 100) {  // fewer waves per SIMD, no spills
                        if (cls == 1) k11pf<256, 18, 4><<<G, 256, 0, s>>>(in, out, list, nb, 2);
                        else k11pf<512, 18, 4><<<G, 512, 0, s>>>(in, out, list, nb, 2);
                    } else if (cls == 1) k11pf<256, 18, 7><<<G, 256, 0, s>>>(in, out, list, nb, 2);
                    else k11pf<512, 18, 6><<<G, 512, 0, s>>>(in, out, list, nb, 2);
                }
                CK(hipEventRecord(e1, s));
                CK(hipEventSynchronize(e1));
                float m;
                CK(hipEventElapsedTime(&m, e0, e1));
                t.push_back(m);
            }
            CK(hipMemcpy(grid_mult == 0 ? h_ref.data() : h_out.data(), out, n * 4,
                         hipMemcpyDeviceToHost));
            // digit 0 is ranked unstably and the test buckets do not share their top 16 bits,
            // so only the low 16 bits' order and each bucket's multiset are determined
            if (grid_mult != 0) {
                for (uint64_t i = 0; i < n; ++i)
                    if ((h_out[i] & 0xFFFFu) != (h_ref[i] & 0xFFFFu)) { printf("MISMATCH grid_mult %d at %llu\n", grid_mult, (unsigned long long)i); return 1; }
                for (uint64_t b = 0; b < nb; b += 101) {
                    std::vector<uint32_t> x(h_out.begin() + b * bsize, h_out.begin() + (b + 1) * bsize);
                    std::vector<uint32_t> y(h_ref.begin() + b * bsize, h_ref.begin() + (b + 1) * bsize);
                    std::sort(x.begin(), x.end());
                    std::sort(y.begin(), y.end());
                    if (x != y) { printf("NOT A PERMUTATION grid_mult %d bucket %llu\n", grid_mult, (unsigned long long)b); return 1; }
                }
            }
            std::sort(t.begin(), t.end());
            const float m = t[t.size() / 2];
            printf("{\"bucket\": %llu, \"class\": %d, \"grid_mult\": %d, \"ms\": %.4f, \"GBps\": %.1f}\n",
                   (unsigned long long)bsize, cls, grid_mult, m, n * 8.0 / (m * 1e-3) / 1e9);
        }
    }
    return 0;
}
