// kexp3.hip -- K11 (in-LDS bucket sort) experiments (development tool).
// Splits 2^lg uniform keys into equal buckets of `bsize` keys and times K11 over all of them
// for 1..3 digits and both workgroup sizes; checks that every bucket comes out sorted on the
// sorted digits and is a permutation of its input.
//   run: kexp3 [log2n=28] [rounds=5]
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

int main(int argc, char **argv) {
    const int lg = argc > 1 ? atoi(argv[1]) : 28;
    const int rounds = argc > 2 ? atoi(argv[2]) : 5;
    const uint64_t n = 1ull << lg;
    uint32_t *in, *out;
    unsigned long long *list;
    CK(hipMalloc(&in, n * 4));
    CK(hipMalloc(&out, n * 4));
    CK(hipMalloc(&list, (n / 1024) * 16));
    hipStream_t s;
    CK(hipStreamCreate(&s));
    CK(launch_generate(0, 42, 0, n, (int32_t *)in, s));
    std::vector<uint32_t> h_in(n), h_out(n);
    CK(hipMemcpy(h_in.data(), in, n * 4, hipMemcpyDeviceToHost));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    struct Cfg { uint64_t bsize; int block, items; };
    const Cfg cfgs[] = {{4096, 512, 16}, {4096, 256, 16}, {2048, 256, 16}, {2048, 256, 8},
                        {8192, 512, 16}, {8192, 512, 18}, {9000, 512, 18}, {9000, 512, 32},
                        {9000, 1024, 16}, {16384, 512, 32}, {16384, 1024, 16}};
    for (const Cfg &cf : cfgs) {
        const uint64_t bsize = cf.bsize, nb = n / bsize;
        std::vector<unsigned long long> hl(2 * nb);
        for (uint64_t b = 0; b < nb; ++b) { hl[2 * b] = b * bsize; hl[2 * b + 1] = bsize; }
        CK(hipMemcpy(list, hl.data(), nb * 16, hipMemcpyHostToDevice));
        for (int nd = 2; nd <= 3; ++nd) {
            std::vector<float> t;
            for (int r = 0; r < rounds; ++r) {
                CK(hipEventRecord(e0, s));
#define L(B, I) if (cf.block == B && cf.items == I) k_local_sort<B, I, true, true><<<nb, B, 0, s>>>(in, out, list, nd)
                L(256, 8); L(256, 16); L(512, 16); L(512, 18); L(512, 32); L(1024, 16);
#undef L
                CK(hipEventRecord(e1, s));
                CK(hipEventSynchronize(e1));
                float m;
                CK(hipEventElapsedTime(&m, e0, e1));
                t.push_back(m);
            }
            CK(hipMemcpy(h_out.data(), out, n * 4, hipMemcpyDeviceToHost));
            const uint32_t mask = (1u << (8 * nd)) - 1;
            for (uint64_t b = 0; b < nb; b += 97) {
                std::vector<uint32_t> a(h_in.begin() + b * bsize, h_in.begin() + (b + 1) * bsize);
                std::vector<uint32_t> o(h_out.begin() + b * bsize, h_out.begin() + (b + 1) * bsize);
                for (uint64_t i = 1; i < bsize; ++i)
                    if ((o[i] & mask) < (o[i - 1] & mask)) { printf("UNSORTED b=%llu\n", (unsigned long long)b); return 1; }
                std::sort(a.begin(), a.end());
                std::sort(o.begin(), o.end());
                if (a != o) { printf("NOT A PERMUTATION b=%llu\n", (unsigned long long)b); return 1; }
            }
            std::sort(t.begin(), t.end());
            const float m = t[t.size() / 2];
            printf("{\"bucket\": %llu, \"digits\": %d, \"block\": %d, \"items\": %d, \"ms\": %.4f, \"GBps\": %.1f}\n",
                   (unsigned long long)bsize, nd, cf.block, cf.items, m, nb * bsize * 8.0 / (m * 1e-3) / 1e9);
        }
    }
    return 0;
}
