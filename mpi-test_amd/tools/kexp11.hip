// kexp11.hip -- K18 (receive-side counting sort of 16-bit buckets) in isolation (development
// tool): one source run of nb buckets x bsize packed keys, timed and checked for sortedness.
//   run: kexp11 [log2_bucket=16] [buckets=4096] [rounds=5]
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
    const int lb = argc > 1 ? atoi(argv[1]) : 16;
    const uint32_t nb = argc > 2 ? (uint32_t)atoi(argv[2]) : 4096;
    const int rounds = argc > 3 ? atoi(argv[3]) : 5;
    const uint64_t bsize = 1ull << lb, n = nb * bsize;
    std::vector<uint16_t> h_in(n);
    uint64_t x = 88172645463325252ull;
    for (auto &v : h_in) { x ^= x << 13; x ^= x >> 7; x ^= x << 17; v = (uint16_t)x; }
    std::vector<unsigned long long> pos(kBuckets16 + 1), list(2 * nb), roff(1, 0);
    for (uint32_t h = 0; h <= kBuckets16; ++h) pos[h] = std::min<uint64_t>(h, nb) * bsize;
    for (uint32_t i = 0; i < nb; ++i) { list[2 * i] = i; list[2 * i + 1] = bsize; }
    uint16_t *d_in;
    uint32_t *d_out;
    unsigned long long *d_pos, *d_list, *d_roff;
    CK(hipMalloc(&d_in, n * 2));
    CK(hipMalloc(&d_out, n * 4));
    CK(hipMalloc(&d_pos, pos.size() * 8));
    CK(hipMalloc(&d_list, list.size() * 8));
    CK(hipMalloc(&d_roff, 8));
    CK(hipMemcpy(d_in, h_in.data(), n * 2, hipMemcpyHostToDevice));
    CK(hipMemcpy(d_pos, pos.data(), pos.size() * 8, hipMemcpyHostToDevice));
    CK(hipMemcpy(d_list, list.data(), list.size() * 8, hipMemcpyHostToDevice));
    CK(hipMemcpy(d_roff, roff.data(), 8, hipMemcpyHostToDevice));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    std::vector<float> t;
    for (int r = 0; r < rounds; ++r) {
        CK(hipEventRecord(e0, 0));
        // bstart == pos for one source
        k_hist_expand<<<nb, 1024>>>(d_in, d_pos, d_roff, 1, d_pos, d_list, d_out);
        CK(hipEventRecord(e1, 0));
        CK(hipEventSynchronize(e1));
        float m;
        CK(hipEventElapsedTime(&m, e0, e1));
        t.push_back(m);
    }
    std::vector<uint32_t> out(n);
    CK(hipMemcpy(out.data(), d_out, n * 4, hipMemcpyDeviceToHost));
    for (uint32_t b = 0; b < nb; ++b) {
        std::vector<uint32_t> ref(h_in.begin() + b * bsize, h_in.begin() + (b + 1) * bsize);
        std::sort(ref.begin(), ref.end());
        for (uint64_t i = 0; i < bsize; ++i)
            if (out[b * bsize + i] != (((b << 16) | ref[i]) ^ kFlip)) {
                printf("MISMATCH bucket %u at %llu\n", b, (unsigned long long)i);
                return 1;
            }
        if (b > 16) break;
    }
    std::sort(t.begin(), t.end());
    const float m = t[t.size() / 2];
    printf("{\"bucket\": %llu, \"buckets\": %u, \"ms\": %.4f, \"GBps\": %.1f, \"us_per_bucket_per_cu\": %.2f}\n",
           (unsigned long long)bsize, nb, m, n * 6.0 / (m * 1e-3) / 1e9, m * 1e3 / (nb / 256.0));
    return 0;
}
