// kexp15.hip -- K18c (k_count_expand, the receive-side one-read counting sort) in isolation
// (development tool): nb buckets of 2^lb random packed u16 keys, one source run; the product
// kernel timed and its output checked.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -I mpi-test_amd/csrc -I include tools/experiments/kexp15.hip -o kexp15
//   run: kexp15 [log2_bucket=16] [buckets=4096] [rounds=5]
#include <stdio.h>
#include <stdlib.h>

#include <algorithm>
#include <vector>

#include "gsort_kernels.hip"

using namespace gsort;

#define CK(x)                                                                         \
    do {                                                                              \
        hipError_t e = (x);                                                           \
        if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); exit(1); } \
    } while (0)

namespace {
}  // namespace

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
    unsigned long long *d_pos, *d_list, *d_roff, *d_prof;
    CK(hipMalloc(&d_in, n * 2));
    CK(hipMalloc(&d_out, n * 4));
    CK(hipMalloc(&d_pos, pos.size() * 8));
    CK(hipMalloc(&d_list, list.size() * 8));
    CK(hipMalloc(&d_roff, 8));
    CK(hipMalloc(&d_prof, (size_t)nb * 6 * 8));
    CK(hipMemcpy(d_in, h_in.data(), n * 2, hipMemcpyHostToDevice));
    CK(hipMemcpy(d_pos, pos.data(), pos.size() * 8, hipMemcpyHostToDevice));
    CK(hipMemcpy(d_list, list.data(), list.size() * 8, hipMemcpyHostToDevice));
    CK(hipMemcpy(d_roff, roff.data(), 8, hipMemcpyHostToDevice));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    std::vector<unsigned long long> prof((size_t)nb * 6);
    for (int mode : {-1}) {
        std::vector<float> t;
        for (int r = 0; r < rounds; ++r) {
            CK(hipEventRecord(e0, 0));
            switch (mode) {  // bstart == pos for one source
                case -1: CK(launch_count_expand(d_in, true, reinterpret_cast<uint64_t *>(d_pos),
                                                reinterpret_cast<uint64_t *>(d_roff), 1,
                                                reinterpret_cast<uint64_t *>(d_pos),
                                                reinterpret_cast<uint64_t *>(d_list), nb, 256, d_out, 0)); break;
            }
            CK(hipEventRecord(e1, 0));
            CK(hipEventSynchronize(e1));
            float m;
            CK(hipEventElapsedTime(&m, e0, e1));
            t.push_back(m);
        }
        std::sort(t.begin(), t.end());
        double ph[4] = {0, 0, 0, 0};
        if (mode >= 0) {
            CK(hipMemcpy(prof.data(), d_prof, prof.size() * 8, hipMemcpyDeviceToHost));
            for (uint32_t b = 0; b < nb; ++b)
                for (int k = 0; k < 4; ++k) ph[k] += (double)(prof[6 * b + k + 1] - prof[6 * b + k]) * 10.0 / nb;  // ns
        }
        const double ms = t[t.size() / 2];
        printf("bucket %7llu: %.4f ms = %.0f GB/s at 6 B/key (2^%d keys)\n",
               (unsigned long long)bsize, ms, n * 6.0 / (ms * 1e6), (int)__builtin_ctzll(n));
        if (mode > 0) continue;
        std::vector<uint32_t> out(n);
        CK(hipMemcpy(out.data(), d_out, n * 4, hipMemcpyDeviceToHost));
        for (uint32_t b = 0; b < nb; b += std::max<uint32_t>(1, nb / 16)) {
            std::vector<uint32_t> ref(h_in.begin() + b * bsize, h_in.begin() + (b + 1) * bsize);
            std::sort(ref.begin(), ref.end());
            for (uint64_t i = 0; i < bsize; ++i)
                if (out[b * bsize + i] != (((b << 16) | ref[i]) ^ kFlip)) {
                    printf("MISMATCH mode %d bucket %u at %llu\n", mode, b, (unsigned long long)i);
                    return 1;
                }
        }
    }
    return 0;
}
