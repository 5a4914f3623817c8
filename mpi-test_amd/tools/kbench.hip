// kbench.hip -- kernel microbenchmark for the onesweep pass geometry (development tool, not
// the product).  Includes the product kernels verbatim and instantiates other tile shapes /
// ablations, times them interleaved in ONE process (cdna_hip_programming.md 5.4 rule 24) on
// 2^28 uniform keys, and verifies every non-ablation output (sorted + same fingerprint).
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

struct Bufs {
    uint32_t *in, *tmp, *out;
    unsigned long long *status, *base, *hist, *acc;
    uint32_t *ctr;
    uint64_t n;
};

template <int B, int I, bool NOLB, bool EARLY = true, int W = 8>
void launch(const Bufs &b, const uint32_t *src, uint32_t *dst, int pass, uint32_t epoch,
            bool fin, bool fout, hipStream_t s) {
    const unsigned g = (unsigned)((b.n + B * I - 1) / (B * I));
    auto *base = b.base + pass * kRadix;
    uint32_t *ctr = b.ctr + pass, *err = b.ctr + 63;
    if (fin)
        k_onesweep<B, I, true, false, NOLB, EARLY, W><<<g, B, 0, s>>>(src, dst, b.n, 8 * pass, base,
                                                            b.status, ctr, err, epoch);
    else if (fout)
        k_onesweep<B, I, false, true, NOLB, EARLY, W><<<g, B, 0, s>>>(src, dst, b.n, 8 * pass, base,
                                                            b.status, ctr, err, epoch);
    else
        k_onesweep<B, I, false, false, NOLB, EARLY, W><<<g, B, 0, s>>>(src, dst, b.n, 8 * pass, base,
                                                             b.status, ctr, err, epoch);
}

typedef void (*LaunchFn)(const Bufs &, const uint32_t *, uint32_t *, int, uint32_t, bool, bool,
                         hipStream_t);
struct Variant {
    const char *name;
    LaunchFn fn;
    bool verify;
    std::vector<float> ms[4];
};

__global__ void k_copy4(const uint4 *in, uint4 *out, uint64_t n4) {
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n4;
         i += (uint64_t)gridDim.x * blockDim.x)
        out[i] = in[i];
}

int main(int argc, char **argv) {
    const int lg = argc > 1 ? atoi(argv[1]) : 28;
    const int rounds = argc > 2 ? atoi(argv[2]) : 5;
    Bufs b;
    b.n = 1ull << lg;
    CK(hipMalloc(&b.in, b.n * 4));
    CK(hipMalloc(&b.tmp, b.n * 4));
    CK(hipMalloc(&b.out, b.n * 4));
    const size_t st_bytes = (b.n / 2048 + 1) * kRadix * 8;
    CK(hipMalloc(&b.status, st_bytes));
    CK(hipMalloc(&b.base, 4 * kRadix * 8));
    CK(hipMalloc(&b.hist, 4 * kRadix * 8));
    CK(hipMalloc(&b.acc, 64));
    CK(hipMalloc(&b.ctr, 64 * 4));
    CK(hipMemset(b.status, 0, st_bytes));
    hipStream_t s;
    CK(hipStreamCreate(&s));
    CK(launch_generate(0, 42, 0, b.n, (int32_t *)b.in, s));
    CK(hipMemsetAsync(b.hist, 0, 4 * kRadix * 8, s));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    // hist4 + reference copy ceiling
    std::vector<float> t_hist, t_copy;
    for (int r = 0; r < rounds; ++r) {
        CK(hipMemsetAsync(b.hist, 0, 4 * kRadix * 8, s));
        CK(hipEventRecord(e0, s));
        CK(launch_hist4(b.in, b.n, (uint64_t *)b.hist, s));
        CK(hipEventRecord(e1, s));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        t_hist.push_back(ms);
        CK(hipEventRecord(e0, s));
        k_copy4<<<4096, 256, 0, s>>>((const uint4 *)b.in, (uint4 *)b.tmp, b.n / 4);
        CK(hipEventRecord(e1, s));
        CK(hipEventSynchronize(e1));
        CK(hipEventElapsedTime(&ms, e0, e1));
        t_copy.push_back(ms);
    }
    std::vector<unsigned long long> h(4 * kRadix), base(4 * kRadix);
    CK(hipMemcpy(h.data(), b.hist, h.size() * 8, hipMemcpyDeviceToHost));
    for (int p = 0; p < 4; ++p) {
        unsigned long long acc = 0;
        for (int d = 0; d < kRadix; ++d) { base[p * kRadix + d] = acc; acc += h[p * kRadix + d]; }
    }
    CK(hipMemcpy(b.base, base.data(), base.size() * 8, hipMemcpyHostToDevice));
    // fingerprint of the input
    unsigned long long fin[3], fo[3];
    CK(hipMemset(b.acc, 0, 24));
    CK(launch_fingerprint((const int32_t *)b.in, b.n, b.acc, s));
    CK(hipMemcpyAsync(fin, b.acc, 24, hipMemcpyDeviceToHost, s));
    CK(hipStreamSynchronize(s));

    std::vector<Variant> vs = {
        {"b512_i16_early_w8", launch<512, 16, false, true, 8>, true},
        {"b512_i16_late_w8", launch<512, 16, false, false, 8>, true},
        {"b512_i16_early_w1", launch<512, 16, false, true, 1>, true},
        {"b512_i16_early_w16", launch<512, 16, false, true, 16>, true},
        {"b512_i16_late_w16", launch<512, 16, false, false, 16>, true},
        {"b256_i16_early_w8", launch<256, 16, false, true, 8>, true},
        {"b256_i32_early_w8", launch<256, 32, false, true, 8>, true},
        {"b512_i24_early_w8", launch<512, 24, false, true, 8>, true},
        {"b1024_i16_early_w8", launch<1024, 16, false, true, 8>, true},
        {"b512_i16_nolookback", launch<512, 16, true>, false},
    };
    uint32_t epoch = 1;
    for (int r = 0; r < rounds; ++r) {
        for (auto &v : vs) {
            CK(hipMemsetAsync(b.ctr, 0, 64 * 4, s));
            const uint32_t *src = b.in;
            uint32_t *dsts[4] = {b.tmp, b.out, b.tmp, b.out};
            for (int p = 0; p < 4; ++p) {
                CK(hipEventRecord(e0, s));
                v.fn(b, src, dsts[p], p, epoch++, p == 0, p == 3, s);
                CK(hipEventRecord(e1, s));
                CK(hipEventSynchronize(e1));
                float ms;
                CK(hipEventElapsedTime(&ms, e0, e1));
                v.ms[p].push_back(ms);
                src = dsts[p];
            }
            uint32_t err = 0;
            CK(hipMemcpy(&err, b.ctr + 63, 4, hipMemcpyDeviceToHost));
            if (v.verify) {
                CK(hipMemset(b.acc, 0, 24));
                CK(launch_fingerprint((const int32_t *)b.out, b.n, b.acc, s));
                CK(hipMemcpyAsync(fo, b.acc, 24, hipMemcpyDeviceToHost, s));
                CK(hipStreamSynchronize(s));
                if (err || fo[0] != fin[0] || fo[1] != fin[1] || fo[2] != 0) {
                    printf("VERIFY FAIL %s err=%u desc=%llu\n", v.name, err, fo[2]);
                    return 1;
                }
            }
        }
    }
    auto med = [](std::vector<float> x) { std::sort(x.begin(), x.end()); return x[x.size() / 2]; };
    const double gb = b.n * 8.0 / 1e9;
    printf("{\"n\": %llu, \"hist4_ms\": %.4f, \"hist4_GBps\": %.1f, \"copy_ms\": %.4f, \"copy_GBps\": %.1f}\n",
           (unsigned long long)b.n, med(t_hist), b.n * 4.0 / 1e9 / (med(t_hist) * 1e-3), med(t_copy),
           gb / (med(t_copy) * 1e-3));
    for (auto &v : vs) {
        double tot = 0;
        printf("{\"variant\": \"%s\", \"pass_ms\": [", v.name);
        for (int p = 0; p < 4; ++p) { printf("%s%.4f", p ? ", " : "", med(v.ms[p])); tot += med(v.ms[p]); }
        printf("], \"avg_pass_GBps\": %.1f, \"verified\": %s}\n", gb / (tot / 4 * 1e-3),
               v.verify ? "true" : "false");
    }

#ifdef GSORT_KBENCH_STAMPS
    {
        // one stamped run of pass 1 (b512_i16, late lookback, W=8) on the sorted-by-digit-0 data
        const uint64_t tiles = (b.n + 8191) / 8192;
        unsigned long long *d_st;
        CK(hipMalloc(&d_st, tiles * 64));
        CK(hipMemset(d_st, 0, tiles * 64));
        CK(hipMemcpyToSymbol(HIP_SYMBOL(g_stamps), &d_st, sizeof(d_st)));
        CK(hipMemsetAsync(b.ctr, 0, 64 * 4, s));
        launch<512, 16, false, true, 8>(b, b.in, b.tmp, 0, epoch++, true, false, s);
        CK(hipMemsetAsync(b.ctr, 0, 64 * 4, s));
        launch<512, 16, false, false, 8>(b, b.tmp, b.out, 1, epoch++, false, false, s);
        CK(hipStreamSynchronize(s));
        std::vector<unsigned long long> st(tiles * 8);
        CK(hipMemcpy(st.data(), d_st, tiles * 64, hipMemcpyDeviceToHost));
        unsigned long long t_min = ~0ull, t_max = 0;
        double ph[3] = {0, 0, 0};
        std::vector<double> lbw, rnd, spn;
        for (uint64_t t = 0; t < tiles; ++t) {
            const unsigned long long *x = &st[t * 8];
            t_min = std::min(t_min, x[0]);
            t_max = std::max(t_max, x[3]);
            ph[0] += x[1] - x[0]; ph[1] += x[2] - x[1]; ph[2] += x[3] - x[2];
            rnd.push_back((double)x[4]); spn.push_back((double)x[5]);
        }
        auto pct = [](std::vector<double> v, double q) { std::sort(v.begin(), v.end()); return v[(size_t)(q * (v.size() - 1))]; };
        // concurrency: average number of tiles between their t0 and t3
        printf("{\"stamps\": true, \"tiles\": %llu, \"span_us\": %.1f, \"avg_us\": {\"load_rank\": %.2f, \"scan_scatter_lookback\": %.2f, \"writeout\": %.2f}, \"avg_tiles_in_flight\": %.1f, \"lb_rounds\": {\"mean\": %.2f, \"p50\": %.0f, \"p99\": %.0f, \"max\": %.0f}, \"lb_spins\": {\"mean\": %.2f, \"p50\": %.0f, \"p99\": %.0f, \"max\": %.0f}}\n",
               (unsigned long long)tiles, (t_max - t_min) / 100.0, ph[0] / tiles / 100.0, ph[1] / tiles / 100.0, ph[2] / tiles / 100.0,
               (ph[0] + ph[1] + ph[2]) / (double)(t_max - t_min),
               std::accumulate(rnd.begin(), rnd.end(), 0.0) / tiles, pct(rnd, .5), pct(rnd, .99), pct(rnd, 1.0),
               std::accumulate(spn.begin(), spn.end(), 0.0) / tiles, pct(spn, .5), pct(spn, .99), pct(spn, 1.0));
        // timeline sample: first 8 tiles and 8 mid tiles
        for (uint64_t t : {0ull, 1ull, 2ull, 100ull, 1000ull, 1001ull, 1002ull, 20000ull, 20001ull}) {
            if (t >= tiles) continue;
            const unsigned long long *x = &st[t * 8];
            printf("{\"tile\": %llu, \"xcc\": %llu, \"t0_us\": %.2f, \"rank_us\": %.2f, \"lb_us\": %.2f, \"wo_us\": %.2f, \"rounds\": %llu, \"spins\": %llu}\n",
                   (unsigned long long)t, x[6], (x[0] - t_min) / 100.0, (x[1] - x[0]) / 100.0, (x[2] - x[1]) / 100.0, (x[3] - x[2]) / 100.0, x[4], x[5]);
        }
    }
#endif
    return 0;
}
