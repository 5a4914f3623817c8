// kbench.hip -- kernel microbenchmark for the LSD pass (development tool, not the product).
// Includes the product kernels verbatim, instantiates alternative K3 geometries, times every
// kernel of a 4-pass sort interleaved in ONE process (cdna_hip_programming.md 5.4 rule 24) on
// 2^28 uniform keys, and verifies every output (sorted + same multiset fingerprint).
//   build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -I../include -Icsrc tools/kbench.hip
//   run:   kbench [log2n=28] [rounds=5]
#include <stdio.h>
#include <stdlib.h>

#include <algorithm>
#include <numeric>
#include <vector>

#include "../csrc/gsort_kernels.hip"

using namespace gsort;

#define CK(x)                                                                         \
    do {                                                                              \
        hipError_t e = (x);                                                           \
        if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); exit(1); } \
    } while (0)

typedef void (*ScatterFn)(const uint32_t *, uint32_t *, uint64_t, int, const uint32_t *,
                          const unsigned long long *, const unsigned long long *, bool, bool,
                          hipStream_t);

template <int B, int I>
void scatter(const uint32_t *in, uint32_t *out, uint64_t n, int shift, const uint32_t *toff,
             const unsigned long long *gp, const unsigned long long *bs, bool fin, bool fout,
             hipStream_t s) {
    const unsigned g = (unsigned)sweep_tiles(n);
    if (fin) k_scatter<B, I, true, false><<<g, B, 0, s>>>(in, out, n, shift, toff, gp, bs);
    else if (fout) k_scatter<B, I, false, true><<<g, B, 0, s>>>(in, out, n, shift, toff, gp, bs);
    else k_scatter<B, I, false, false><<<g, B, 0, s>>>(in, out, n, shift, toff, gp, bs);
}

__global__ void k_copy4(const uint4 *in, uint4 *out, uint64_t n4) {
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n4;
         i += (uint64_t)gridDim.x * blockDim.x)
        out[i] = in[i];
}

struct Variant {
    const char *name;
    ScatterFn fn;
    std::vector<float> count, scan, pass;
};

int main(int argc, char **argv) {
    const int lg = argc > 1 ? atoi(argv[1]) : 28;
    const int rounds = argc > 2 ? atoi(argv[2]) : 5;
    const uint64_t n = 1ull << lg;
    uint32_t *in, *tmp, *out, *tc;
    unsigned long long *gs, *hist, *acc;
    CK(hipMalloc(&in, n * 4));
    CK(hipMalloc(&tmp, n * 4));
    CK(hipMalloc(&out, n * 4));
    CK(hipMalloc(&tc, sweep_tiles(n) * kRadix * 4));
    CK(hipMalloc(&gs, scan_groups(n) * kRadix * 8));
    CK(hipMalloc(&hist, 4 * kRadix * 8));
    unsigned long long *tot, *bases;
    CK(hipMalloc(&tot, kRadix * 8));
    CK(hipMalloc(&bases, kRadix * 8));
    CK(hipMalloc(&acc, 64));
    hipStream_t s;
    CK(hipStreamCreate(&s));
    CK(launch_generate(0, 42, 0, n, (int32_t *)in, s));
    hipEvent_t ev[8];
    for (auto &x : ev) CK(hipEventCreate(&x));
    auto ms = [&](hipEvent_t a, hipEvent_t b) { float m; CK(hipEventElapsedTime(&m, a, b)); return m; };
    unsigned long long fin[3], fo[3];
    CK(hipMemset(acc, 0, 24));
    CK(launch_fingerprint((const int32_t *)in, n, acc, s));
    CK(hipMemcpyAsync(fin, acc, 24, hipMemcpyDeviceToHost, s));
    CK(hipStreamSynchronize(s));

    std::vector<Variant> vs = {
        {"k3_b512_i16", scatter<512, 16>},
        {"k3_b256_i32", scatter<256, 32>},
        {"k3_b1024_i8", scatter<1024, 8>},
    };
    std::vector<float> t_all4, t_copy;
    for (int r = 0; r < rounds; ++r) {
        CK(hipEventRecord(ev[0], s));
        k_copy4<<<4096, 256, 0, s>>>((const uint4 *)in, (uint4 *)tmp, n / 4);
        CK(hipEventRecord(ev[1], s));
        CK(hipEventSynchronize(ev[1]));
        t_copy.push_back(ms(ev[0], ev[1]));
        for (auto &v : vs) {
            const uint32_t *src = in;
            uint32_t *dsts[4] = {tmp, out, tmp, out};
            for (int p = 0; p < 4; ++p) {
                CK(hipEventRecord(ev[0], s));
                if (p == 0) {
                    CK(hipMemsetAsync(hist, 0, 4 * kRadix * 8, s));
                    CK(launch_tile_counts(src, n, 0, true, tc, (uint64_t *)hist, s));
                } else {
                    CK(launch_tile_counts(src, n, 8 * p, false, tc, nullptr, s));
                }
                CK(hipEventRecord(ev[1], s));
                CK(launch_scan_tiles(tc, n, (uint64_t *)gs, (uint64_t *)tot, (uint64_t *)bases, s));
                CK(hipEventRecord(ev[2], s));
                v.fn(src, dsts[p], n, 8 * p, tc, gs, bases, p == 0, p == 3, s);
                CK(hipEventRecord(ev[3], s));
                CK(hipEventSynchronize(ev[3]));
                (p == 0 ? t_all4 : v.count).push_back(ms(ev[0], ev[1]));
                v.scan.push_back(ms(ev[1], ev[2]));
                v.pass.push_back(ms(ev[2], ev[3]));
                src = dsts[p];
            }
            CK(hipMemset(acc, 0, 24));
            CK(launch_fingerprint((const int32_t *)out, n, acc, s));
            CK(hipMemcpyAsync(fo, acc, 24, hipMemcpyDeviceToHost, s));
            CK(hipStreamSynchronize(s));
            if (fo[0] != fin[0] || fo[1] != fin[1] || fo[2] != 0) {
                printf("VERIFY FAIL %s desc=%llu\n", v.name, fo[2]);
                return 1;
            }
        }
    }
    auto med = [](std::vector<float> x) { std::sort(x.begin(), x.end()); return x[x.size() / 2]; };
    const double gb4 = n * 4.0 / 1e9;
    printf("{\"n\": %llu, \"copy_ms\": %.4f, \"copy_GBps\": %.1f, \"k1_all4_ms\": %.4f, \"k1_all4_GBps\": %.1f}\n",
           (unsigned long long)n, med(t_copy), 2 * gb4 / (med(t_copy) * 1e-3), med(t_all4),
           gb4 / (med(t_all4) * 1e-3));
    for (auto &v : vs) {
        const double total = med(t_all4) + 3 * med(v.count) + 4 * med(v.scan) + 4 * med(v.pass);
        printf("{\"variant\": \"%s\", \"k1_ms\": %.4f, \"k1_GBps\": %.1f, \"k2_ms\": %.4f, \"k3_ms\": %.4f, \"k3_GBps\": %.1f, \"sort_ms\": %.4f, \"GKeys_s\": %.2f}\n",
               v.name, med(v.count), gb4 / (med(v.count) * 1e-3), med(v.scan), med(v.pass),
               2 * gb4 / (med(v.pass) * 1e-3), total, n / (total * 1e-3) / 1e9);
    }
    return 0;
}
