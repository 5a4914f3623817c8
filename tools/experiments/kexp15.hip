// kexp15.hip -- K18c (k_count_expand, the receive-side one-read counting sort) in isolation
// (development tool): nb buckets of 2^lb random packed u16 keys, one source run; per-phase
// timestamps (wall_clock64, 100 MHz) of a profiled copy with ablations, the product kernel
// timed and its output checked.
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
template <typename T, int MODE>
__global__ __launch_bounds__(1024) void k18p(unsigned long long *prof, const T *__restrict__ recv,
                                                       const unsigned long long *__restrict__ pos,
                                                       const unsigned long long *__restrict__ roff,
                                                       int P,
                                                       const unsigned long long *__restrict__ bstart,
                                                       const unsigned long long *__restrict__ list,
                                                       uint32_t *__restrict__ out) {
    constexpr uint32_t NT = 1024, NW = NT / 64, WORDS = 32768, CW = 128;  // words per chunk
    constexpr uint32_t CH = WORDS / NW / CW;                               // 16 chunks per wave
    __shared__ uint32_t s_h[WORDS];
    __shared__ uint4 s_mark[NW * 64];  // 256 slots per wave
    __shared__ uint32_t s_base[NW * CH];
    __shared__ uint32_t s_wsum[NW];
    __shared__ uint64_t s_src[64];
    __shared__ uint32_t s_len[64];
    __shared__ uint32_t s_wb[kCxWrapMax];
    __shared__ int32_t s_wd[kCxWrapMax];
    __shared__ uint32_t s_nw;
    const uint32_t tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    unsigned long long *pf = prof + 6 * blockIdx.x;
    if (tid == 0) pf[0] = wall_clock64();
    const uint32_t h = (uint32_t)list[2 * blockIdx.x];
    const uint32_t len = (uint32_t)list[2 * blockIdx.x + 1];
    if ((int)tid < P) {
        const uint64_t a = pos[(uint64_t)tid * (kBuckets16 + 1) + h];
        const uint64_t b = pos[(uint64_t)tid * (kBuckets16 + 1) + h + 1];
        s_src[tid] = roff[tid] + a;
        s_len[tid] = (uint32_t)(b - a);
    }
    if (tid == 0) s_nw = 0;
    {
        uint4 *z = reinterpret_cast<uint4 *>(s_h);
#pragma unroll
        for (uint32_t i = 0; i < WORDS / 4 / NT; ++i) z[i * NT + tid] = make_uint4(0, 0, 0, 0);
    }
    __syncthreads();
    if (tid == 0) pf[1] = wall_clock64();
    const bool wrap = len >= 65536u;  // below that no half can wrap
#pragma unroll 1
    for (int p = 0; p < P; ++p) {
        if (MODE & 2) {
            const T *sp = recv + s_src[p];
            uint32_t dm = 0;
            for (uint32_t j = tid; j < s_len[p]; j += 1024) dm += sp[j];
            if (dm == 0x12345u) s_nw = 1;
        } else if (wrap) cx_count_piece<true>(recv + s_src[p], s_len[p], s_h, &s_nw, s_wb, s_wd);
        else cx_count_piece<false>(recv + s_src[p], s_len[p], s_h, &s_nw, s_wb, s_wd);
    }
    __syncthreads();
    if (tid == 0) pf[2] = wall_clock64();
    const uint32_t nw = min(s_nw, kCxWrapMax);  // uniform; 0 unless a half wrapped
    const uint32_t w0 = w * (WORDS / NW);
    // lane's 4 bins of chunk j: counts (wrap corrections applied)
    auto counts = [&](uint32_t j, uint32_t (&c)[4]) {
        const uint32_t wd = w0 + CW * j + 2 * lane;
        const uint2 x = *reinterpret_cast<const uint2 *>(s_h + wd);
        c[0] = x.x & 0xFFFFu;
        c[1] = x.x >> 16;
        c[2] = x.y & 0xFFFFu;
        c[3] = x.y >> 16;
        for (uint32_t e = 0; e < nw; ++e) {
            const uint32_t b = s_wb[e] - 2 * wd;  // bin relative to the lane's first
            if (b < 4u) {
                const uint32_t d = (uint32_t)s_wd[e];
                c[0] += b == 0 ? d : 0u;
                c[1] += b == 1 ? d : 0u;
                c[2] += b == 2 ? d : 0u;
                c[3] += b == 3 ? d : 0u;
            }
        }
    };
    // chunk totals
#pragma unroll 1
    for (uint32_t j = 0; j < CH; ++j) {
        uint32_t c[4];
        counts(j, c);
        const uint32_t x = wave_incl_add(c[0] + c[1] + c[2] + c[3]);
        if (lane == 63) s_base[w * CH + j] = x;
    }
    __syncthreads();
    // exclusive scan of the 256 chunk totals in (wave, chunk) = bin order
    {
        uint32_t v = 0, x = 0;
        if (tid < NW * CH) { v = s_base[tid]; x = wave_incl_add(v); }
        if (tid < NW * CH && lane == 63) s_wsum[w] = x;
        __syncthreads();
        if (tid < NW * CH) {
            uint32_t off = 0;
            for (uint32_t ww = 0; ww < w; ++ww) off += s_wsum[ww];
            s_base[tid] = off + x - v;
        }
        __syncthreads();
    }
    if (tid == 0) pf[3] = wall_clock64();
    if (MODE & 4) { if (tid == 0) pf[4] = pf[5] = wall_clock64(); return; }
    uint4 *mk4 = s_mark + 64 * w;
    uint32_t *mk = reinterpret_cast<uint32_t *>(mk4);
    uint32_t *dst = out + bstart[h];
    const uint32_t hk = (h << 16) ^ kFlip;
#pragma unroll 1
    for (uint32_t j = 0; j < CH; ++j) {
        uint32_t c[4];
        counts(j, c);
        const uint32_t t = c[0] + c[1] + c[2] + c[3];
        const uint32_t x = wave_incl_add(t);
        const uint32_t tot = (uint32_t)__builtin_amdgcn_readlane((int)x, 63);
        if (tot == 0) continue;
        uint32_t st[4];  // first slot of each of the lane's bins
        st[0] = x - t;
        st[1] = st[0] + c[0];
        st[2] = st[1] + c[1];
        st[3] = st[2] + c[2];
        const uint32_t b0 = 2 * (w0 + CW * j + 2 * lane) + 1;  // mark = bin + 1
        uint32_t *d = dst + s_base[w * CH + j];
        // windows aligned to 16 B in out: window r covers slots [256 r - off, +256)
        const uint32_t off = (uint32_t)(reinterpret_cast<uintptr_t>(d) >> 2) & 3u;
        uint32_t carry = 0;
#pragma unroll 1
        for (uint32_t r0 = 0; r0 < tot + off; r0 += 256) {
            const uint32_t ws = r0 - off;  // window start slot (mod 2^32)
            mk4[lane] = make_uint4(0, 0, 0, 0);
            __builtin_amdgcn_wave_barrier();
#pragma unroll
            for (int i = 0; i < 4; ++i)
                if (c[i] && st[i] - ws < 256u) mk[st[i] - ws] = b0 + i;
            __builtin_amdgcn_wave_barrier();
            const uint4 m = mk4[lane];
            const uint32_t a0 = m.x, a1 = max(a0, m.y), a2 = max(a1, m.z), a3 = max(a2, m.w);
            const uint32_t S = wave_incl_max(a3);
            // the lanes below: S of lane - 1 (DPP wave shift right by one; lane 0 reads 0)
            const uint32_t prev = max(carry, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)S, 0x138, 0xf, 0xf, true));
            carry = max(carry, (uint32_t)__builtin_amdgcn_readlane((int)S, 63));
            const uint32_t q = ws + 4 * lane;  // this lane's first slot
            const uint4 v = make_uint4(hk | (max(prev, a0) - 1), hk | (max(prev, a1) - 1),
                                       hk | (max(prev, a2) - 1), hk | (max(prev, a3) - 1));
            if (MODE & 1) {
                if ((v.x ^ v.y ^ v.z ^ v.w) == 0x7u) d[0] = 1;
            } else if (q < tot && q + 4 <= tot && q + 4 > q) {
                *reinterpret_cast<uint4 *>(d + q) = v;  // 16-B aligned
            } else {
                if (q < tot) d[q] = v.x;
                if (q + 1 < tot) d[q + 1] = v.y;
                if (q + 2 < tot) d[q + 2] = v.z;
                if (q + 3 < tot) d[q + 3] = v.w;
            }
            __builtin_amdgcn_wave_barrier();
        }
    }
    __syncthreads();
    if (tid == 0) pf[4] = wall_clock64();
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
    for (int mode : {-1, 0, 1, 2, 4, 6}) {
        std::vector<float> t;
        for (int r = 0; r < rounds; ++r) {
            CK(hipEventRecord(e0, 0));
            switch (mode) {  // bstart == pos for one source
                case -1: CK(launch_count_expand(d_in, true, reinterpret_cast<uint64_t *>(d_pos),
                                                reinterpret_cast<uint64_t *>(d_roff), 1,
                                                reinterpret_cast<uint64_t *>(d_pos),
                                                reinterpret_cast<uint64_t *>(d_list), nb, d_out, 0)); break;
                case 0: k18p<uint16_t, 0><<<nb, 1024>>>(d_prof, d_in, d_pos, d_roff, 1, d_pos, d_list, d_out); break;
                case 1: k18p<uint16_t, 1><<<nb, 1024>>>(d_prof, d_in, d_pos, d_roff, 1, d_pos, d_list, d_out); break;
                case 2: k18p<uint16_t, 2><<<nb, 1024>>>(d_prof, d_in, d_pos, d_roff, 1, d_pos, d_list, d_out); break;
                case 4: k18p<uint16_t, 4><<<nb, 1024>>>(d_prof, d_in, d_pos, d_roff, 1, d_pos, d_list, d_out); break;
                case 6: k18p<uint16_t, 6><<<nb, 1024>>>(d_prof, d_in, d_pos, d_roff, 1, d_pos, d_list, d_out); break;
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
        printf("mode %2d bucket %7llu: %.4f ms = %.0f GB/s at 6 B/key; per block us: zero %.2f hist %.2f scan %.2f expand %.2f\n",
               mode, (unsigned long long)bsize, ms, n * 6.0 / (ms * 1e6), ph[0] / 1e3, ph[1] / 1e3, ph[2] / 1e3, ph[3] / 1e3);
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
