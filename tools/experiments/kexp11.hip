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


namespace {
// MODE bits: 1 = keys read once into registers (len <= 65536), 2 = no expansion stores
// (a dummy sum instead), 4 = no histogram atomics
template <int MODE>
__global__ __launch_bounds__(1024) void k18v(const uint16_t *__restrict__ recv,
                                             const unsigned long long *__restrict__ pos,
                                             const unsigned long long *__restrict__ bstart,
                                             const unsigned long long *__restrict__ list,
                                             uint32_t *__restrict__ out) {
    constexpr uint32_t HB = 32768, NT = 1024, PER = HB / NT;
    __shared__ uint32_t s_c[HB + HB / 32];
    __shared__ uint32_t s_w[NT / 64];
    const uint32_t tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const uint32_t h = (uint32_t)list[2 * blockIdx.x];
    const uint64_t a = pos[h], np = pos[h + 1] - a;
    const uint16_t *src = recv + a;
    uint32_t *dst = out + bstart[h];
    uint32_t base = 0, dummy = 0;
    auto pad = [](uint32_t b) { return b + (b >> 5); };
    uint32_t kr[32];  // MODE & 1: 64 keys per thread, two per register
    if (MODE & 1) {
#pragma unroll
        for (int u = 0; u < 32; ++u) {
            const uint32_t j0 = (2 * u) * NT + tid, j1 = (2 * u + 1) * NT + tid;
            const uint32_t x0 = j0 < np ? src[j0] : 0x10000u;
            const uint32_t x1 = j1 < np ? src[j1] : 0x10000u;
            kr[u] = (x0 & 0xFFFFu) | (x1 << 16) | (x0 >> 16 ? 0u : 0u);
            if (x0 == 0x10000u) kr[u] = (kr[u] & 0xFFFF0000u) | 0xFFFFu;  // marks below
        }
    }
    for (uint32_t half = 0; half < 2; ++half) {
        for (uint32_t i = tid; i < HB + HB / 32; i += NT) s_c[i] = 0;
        __syncthreads();
        if (MODE & 1) {
#pragma unroll
            for (int u = 0; u < 32; ++u) {
                const uint32_t j0 = (2 * u) * NT + tid, j1 = (2 * u + 1) * NT + tid;
                const uint32_t x0 = kr[u] & 0xFFFFu, x1 = kr[u] >> 16;
                if (!(MODE & 4)) {
                    if (j0 < np && (x0 >> 15) == half) atomicAdd(&s_c[pad(x0 & (HB - 1))], 1u);
                    if (j1 < np && (x1 >> 15) == half) atomicAdd(&s_c[pad(x1 & (HB - 1))], 1u);
                }
            }
        } else {
#pragma unroll 1
            for (uint32_t j0 = 0; j0 < np; j0 += 8 * NT) {
                uint32_t v[8];
#pragma unroll
                for (int u = 0; u < 8; ++u) {
                    const uint32_t j = j0 + u * NT + tid;
                    v[u] = j < np ? src[j] : 0x10000u;
                }
                if (!(MODE & 4)) {
#pragma unroll
                    for (int u = 0; u < 8; ++u)
                        if ((v[u] >> 15) == half) atomicAdd(&s_c[pad(v[u] & (HB - 1))], 1u);
                } else {
#pragma unroll
                    for (int u = 0; u < 8; ++u) dummy += v[u];
                }
            }
        }
        __syncthreads();
        uint32_t c[PER], sum = 0;
#pragma unroll
        for (uint32_t j = 0; j < PER; ++j) { c[j] = s_c[pad(tid * PER + j)]; sum += c[j]; }
        uint32_t x = sum;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const uint32_t t = __shfl_up(x, o);
            if ((int)lane >= o) x += t;
        }
        if (lane == 63) s_w[w] = x;
        __syncthreads();
        uint32_t run = base + x - sum, total = 0;
        for (uint32_t ww = 0; ww < NT / 64; ++ww) {
            const uint32_t sw = s_w[ww];
            if (ww < w) run += sw;
            total += sw;
        }
#pragma unroll
        for (uint32_t j = 0; j < PER; ++j) { s_c[pad(tid * PER + j)] = run; run += c[j]; }
        __syncthreads();
        const uint32_t end_all = base + total;
#pragma unroll 1
        for (uint32_t j = 0; j < PER; ++j) {
            const uint32_t b = j * NT + tid;
            const uint32_t st = s_c[pad(b)];
            const uint32_t en = b + 1 < HB ? s_c[pad(b + 1)] : end_all;
            const uint32_t key = ((h << 16) | (half << 15) | b) ^ kFlip;
            if (MODE & 2) dummy += st * 3 + en;
            else for (uint32_t q = st; q < en; ++q) dst[q] = key;
        }
        base = end_all;
        __syncthreads();
    }
    if (dummy == 0x12345678u) out[0] = dummy;
}
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
    for (int mode : {-1, 0, 1, 2, 4, 6, 3}) {
    std::vector<float> t;
    for (int r = 0; r < rounds; ++r) {
        CK(hipEventRecord(e0, 0));
        // bstart == pos for one source
        switch (mode) {
            case -1: k_hist_expand<<<nb, 1024>>>(d_in, d_pos, d_roff, 1, d_pos, d_list, d_out); break;
            case 0: k18v<0><<<nb, 1024>>>(d_in, d_pos, d_pos, d_list, d_out); break;
            case 1: k18v<1><<<nb, 1024>>>(d_in, d_pos, d_pos, d_list, d_out); break;
            case 2: k18v<2><<<nb, 1024>>>(d_in, d_pos, d_pos, d_list, d_out); break;
            case 4: k18v<4><<<nb, 1024>>>(d_in, d_pos, d_pos, d_list, d_out); break;
            case 6: k18v<6><<<nb, 1024>>>(d_in, d_pos, d_pos, d_list, d_out); break;
            case 3: k18v<3><<<nb, 1024>>>(d_in, d_pos, d_pos, d_list, d_out); break;
        }
        CK(hipEventRecord(e1, 0));
        CK(hipEventSynchronize(e1));
        float m;
        CK(hipEventElapsedTime(&m, e0, e1));
        t.push_back(m);
    }
    std::sort(t.begin(), t.end());
    printf("{\"mode\": %d, \"bucket\": %llu, \"ms\": %.4f, \"us_per_bucket_per_cu\": %.2f}\n", mode,
           (unsigned long long)bsize, t[t.size() / 2], t[t.size() / 2] * 1e3 / (nb / 256.0));
    if (mode == 2 || mode == 6 || mode == 3 || mode == 4) continue;
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
    }
    return 0;
}
