// lds_hi_check.hip -- experiment (not product): does a workgroup with a >128 KiB LDS allocation
// (K1h's 129 KiB 16-bit histogram, gsort_kernels.hip k_counts_h16) count correctly when other
// kernels already hold LDS on the same CUs (concurrent streams, as the in-process rank group
// runs 8 contexts on one GPU)?  Kernel B histograms known keys into 32768 packed LDS words with
// atomics and stores them; the host compares with the exact histogram.  Kernel A occupies LDS
// (occ KiB per workgroup, 1-2 workgroups per CU) and spins.  Writes only its own outputs.
//   hipcc --offload-arch=gfx950 -O3 tools/lds_hi_check.hip -o /tmp/lds_hi_check
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#include <vector>

#define CK(x)                                                                   \
    do {                                                                        \
        hipError_t e_ = (x);                                                    \
        if (e_ != hipSuccess) {                                                 \
            fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x,          \
                    hipGetErrorString(e_));                                     \
            exit(2);                                                            \
        }                                                                       \
    } while (0)

constexpr int kWords = 32768;

template <int OCC_WORDS>
__global__ __launch_bounds__(256) void k_occupy(uint32_t *sink, long long cycles) {
    __shared__ uint32_t s[OCC_WORDS];
    for (int i = threadIdx.x; i < OCC_WORDS; i += 256) s[i] = i;
    __syncthreads();
    const long long t0 = clock64();
    uint32_t acc = 0;
    while (clock64() - t0 < cycles) acc += s[(acc + threadIdx.x) % OCC_WORDS];
    if (acc == 0xdeadbeef) sink[blockIdx.x] = acc;
}

__global__ __launch_bounds__(1024) void k_hist(const uint32_t *keys, int per_block,
                                               uint32_t *out) {
    __shared__ uint32_t s_h[kWords];
    __shared__ uint32_t s_pad[256];
    for (int i = threadIdx.x; i < kWords; i += 1024) s_h[i] = 0;
    if (threadIdx.x < 256) s_pad[threadIdx.x] = 0;
    __syncthreads();
    const uint32_t *k = keys + (size_t)blockIdx.x * per_block;
    for (int i = threadIdx.x; i < per_block; i += 1024) {
        const uint32_t b = k[i] >> 16;
        atomicAdd(&s_h[b >> 1], 1u << ((b & 1u) << 4));
        atomicAdd(&s_pad[k[i] & 255u], 1u);
    }
    __syncthreads();
    uint32_t *o = out + (size_t)blockIdx.x * (kWords + 256);
    for (int i = threadIdx.x; i < kWords; i += 1024) o[i] = s_h[i];
    if (threadIdx.x < 256) o[kWords + threadIdx.x] = s_pad[threadIdx.x];
}

int main(int argc, char **argv) {
    const int trials = argc > 1 ? atoi(argv[1]) : 20;
    const int nblk = 256, per = 8192;
    std::vector<uint32_t> h((size_t)nblk * per);
    uint64_t x = 88172645463325252ull;
    for (auto &v : h) { x ^= x << 13; x ^= x >> 7; x ^= x << 17; v = (uint32_t)x; }
    std::vector<uint32_t> want((size_t)nblk * (kWords + 256), 0);
    for (int b = 0; b < nblk; ++b)
        for (int i = 0; i < per; ++i) {
            const uint32_t k = h[(size_t)b * per + i], hb = k >> 16;
            want[(size_t)b * (kWords + 256) + (hb >> 1)] += 1u << ((hb & 1u) << 4);
            want[(size_t)b * (kWords + 256) + kWords + (k & 255u)] += 1;
        }
    uint32_t *d_keys, *d_out, *d_sink;
    CK(hipMalloc(&d_keys, h.size() * 4));
    CK(hipMalloc(&d_out, want.size() * 4));
    CK(hipMalloc(&d_sink, 4096 * 4));
    CK(hipMemcpy(d_keys, h.data(), h.size() * 4, hipMemcpyHostToDevice));
    hipStream_t sa, sb;
    CK(hipStreamCreateWithFlags(&sa, hipStreamNonBlocking));
    CK(hipStreamCreateWithFlags(&sb, hipStreamNonBlocking));
    std::vector<uint32_t> got(want.size());
    long long bad_total = 0;
    for (int occ_case = 0; occ_case < 4; ++occ_case) {
        for (int t = 0; t < trials; ++t) {
            CK(hipMemset(d_out, 0xff, want.size() * 4));
            CK(hipDeviceSynchronize());
            const long long cyc = 2000000;  // ~1 ms at ~2 GHz
            switch (occ_case) {  // A first: its workgroups hold LDS when B's arrive
                case 0: break;   // no occupier: baseline
                case 1: k_occupy<1024><<<512, 256, 0, sa>>>(d_sink, cyc); break;   // 4 KiB
                case 2: k_occupy<5120><<<512, 256, 0, sa>>>(d_sink, cyc); break;   // 20 KiB
                case 3: k_occupy<7680><<<256, 256, 0, sa>>>(d_sink, cyc); break;   // 30 KiB
            }
            k_hist<<<nblk, 1024, 0, sb>>>(d_keys, per, d_out);
            CK(hipGetLastError());
            CK(hipDeviceSynchronize());
            CK(hipMemcpy(got.data(), d_out, got.size() * 4, hipMemcpyDeviceToHost));
            long long bad = 0;
            for (size_t i = 0; i < got.size(); ++i) bad += got[i] != want[i];
            bad_total += bad;
            if (bad) printf("occ_case %d trial %d: %lld wrong words\n", occ_case, t, bad);
        }
        printf("occ_case %d done\n", occ_case);
    }
    printf("RESULT wrong_words=%lld\n", bad_total);
    return bad_total ? 1 : 0;
}
