// kexp.hip -- K3 design experiments (development tool, not the product).
// Times variants of the LSD rank+scatter pass against the product K3 on the same input and
// checks every variant's output is bit-identical to the product's.
//   build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -I../../include -I../csrc kexp.hip
//   run:   kexp [log2n=28] [rounds=5]
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
// RANK: 0 = read/modify/write chain (product), 1 = leader ds_add_rtn + bpermute,
//       2 = fake ranks (timing only: no ranking work; output wrong)
// WOUT: false = skip the global write-out (timing only)
template <int BLOCK, int ITEMS, int RANK, bool WOUT, int MINB>
__global__ __launch_bounds__(BLOCK, MINB) void k3x(const uint32_t *__restrict__ in,
                                                   uint32_t *__restrict__ out, uint64_t n,
                                                   int shift, const uint32_t *__restrict__ toff,
                                                   const unsigned long long *__restrict__ gpfx,
                                                   const unsigned long long *__restrict__ bases) {
    constexpr int WAVES = BLOCK / 64;
    constexpr int TILE = BLOCK * ITEMS;
    __shared__ uint32_t s_keys[TILE];
    __shared__ uint32_t s_wofs[WAVES * kRadix];
    __shared__ uint32_t *s_dst[kRadix];
    __shared__ uint32_t s_wsum[kRadix / 64];
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const uint32_t tile = xcd_tile(blockIdx.x, gridDim.x);
    const uint64_t tbase = (uint64_t)tile * TILE;
    const bool full = tbase + TILE <= n;
    for (int i = tid; i < WAVES * kRadix; i += BLOCK) s_wofs[i] = 0;
    uint32_t *dst_base = nullptr;
    if (tid < kRadix)
        dst_base = out + bases[tid] + gpfx[(uint64_t)(tile / kScanGroup) * kRadix + tid] +
                   toff[(uint64_t)tile * kRadix + tid];
    uint32_t k[ITEMS];
    {
        const uint32_t *src = in + tbase + (uint64_t)w * 64 * ITEMS + lane;
        const uint64_t lim = n - tbase;
        const uint64_t o = (uint64_t)w * 64 * ITEMS + lane;
#pragma unroll
        for (int i = 0; i < ITEMS; ++i)
            k[i] = (full || o + i * 64 < lim) ? src[i * 64] : 0xFFFFFFFFu;
    }
    __syncthreads();
    uint32_t rk[(ITEMS + 1) / 2];
    uint32_t *wc = s_wofs + w * kRadix;
#pragma unroll
    for (int i = 0; i < ITEMS; ++i) {
        const uint32_t d = (k[i] >> shift) & 255u;
        uint32_t r;
        if (RANK == 2) {
            r = (uint32_t)(i * 64 + lane) / 256u;  // fake
            if (lane == 0) atomicAdd(&wc[d], 64u);
        } else {
            uint32_t plo = ~0u, phi = ~0u;
#pragma unroll
            for (int b = 0; b < 8; ++b) {
                const uint32_t m = (uint32_t)__builtin_amdgcn_sbfe((int32_t)d, b, 1);
                uint64_t bal;
                asm("v_cmp_ne_u32_e64 %0, 0, %1" : "=s"(bal) : "v"(m));
                plo = __builtin_amdgcn_bitop3_b32(plo, (uint32_t)bal, m, 0x90);
                phi = __builtin_amdgcn_bitop3_b32(phi, (uint32_t)(bal >> 32), m, 0x90);
            }
            const uint32_t below =
                __builtin_amdgcn_mbcnt_hi(phi, __builtin_amdgcn_mbcnt_lo(plo, 0u));
            const uint32_t cnt = (uint32_t)(__popc(plo) + __popc(phi));
            if (RANK == 0) {
                const uint32_t prev = wc[d];
                r = prev + below;
                wc[d] = prev + cnt;
            } else {
                const uint32_t lead = plo ? (uint32_t)__builtin_ctz(plo)
                                          : 32u + (uint32_t)__builtin_ctz(phi);
                uint32_t prev = 0;
                if (below == 0) prev = __hip_atomic_fetch_add(&wc[d], cnt, __ATOMIC_RELAXED,
                                                              __HIP_MEMORY_SCOPE_WORKGROUP);
                prev = (uint32_t)__builtin_amdgcn_ds_bpermute((int)(lead << 2), (int)prev);
                r = prev + below;
            }
        }
        if (i & 1) rk[i >> 1] |= r << 16; else rk[i >> 1] = r;
    }
    __syncthreads();
    uint32_t tcount = 0, excl = 0;
    if (tid < kRadix) {
#pragma unroll
        for (int ww = 0; ww < WAVES; ++ww) tcount += s_wofs[ww * kRadix + tid];
        uint32_t v = tcount;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const uint32_t t = __shfl_up(v, o);
            if (lane >= o) v += t;
        }
        if (lane == 63) s_wsum[w] = v;
        excl = v - tcount;
    }
    __syncthreads();
    if (tid < kRadix) {
        uint32_t start = excl;
        for (int ww = 0; ww < w; ++ww) start += s_wsum[ww];
        s_dst[tid] = dst_base - start;
        uint32_t off = start;
#pragma unroll
        for (int ww = 0; ww < WAVES; ++ww) {
            const uint32_t cw = s_wofs[ww * kRadix + tid];
            s_wofs[ww * kRadix + tid] = off;
            off += cw;
        }
    }
    __syncthreads();
#pragma unroll
    for (int i = 0; i < ITEMS; ++i) {
        const uint32_t d = (k[i] >> shift) & 255u;
        const uint32_t r = (i & 1) ? (rk[i >> 1] >> 16) : (rk[i >> 1] & 0xFFFFu);
        s_keys[(wc[d] + r) & (TILE - 1)] = k[i];
    }
    __syncthreads();
    const uint32_t lim = full ? (uint32_t)TILE : (uint32_t)(n - tbase);
#pragma unroll
    for (int i = 0; i < ITEMS; ++i) {
        const uint32_t j = (uint32_t)(i * BLOCK + tid);
        if (full || j < lim) {
            const uint32_t key = s_keys[j];
            if (WOUT && RANK == 2) {  // fake ranks: keep every store inside the buffer
                const int64_t idx = (s_dst[(key >> shift) & 255u] + j) - out;
                out[(uint64_t)idx & (n - 1)] = key;
            } else if (WOUT) s_dst[(key >> shift) & 255u][j] = key;
            else if (key == 0x12345678u) out[j] = key;
        }
    }
}

typedef void (*Fn)(const uint32_t *, uint32_t *, uint64_t, int, const uint32_t *,
                   const unsigned long long *, const unsigned long long *, hipStream_t);

template <int B, int I, int RANK, bool WOUT, int MINB>
void run3(const uint32_t *in, uint32_t *out, uint64_t n, int shift, const uint32_t *toff,
          const unsigned long long *gp, const unsigned long long *bs, hipStream_t s) {
    k3x<B, I, RANK, WOUT, MINB><<<(unsigned)sweep_tiles(n), B, 0, s>>>(in, out, n, shift, toff, gp, bs);
}
void prod(const uint32_t *in, uint32_t *out, uint64_t n, int shift, const uint32_t *toff,
          const unsigned long long *gp, const unsigned long long *bs, hipStream_t s) {
    (void)launch_scatter(in, out, n, shift, toff, (const uint64_t *)gp, (const uint64_t *)bs,
                         false, false, s);
}
struct V { const char *name; Fn fn; bool check; std::vector<float> t; };
}  // namespace

int main(int argc, char **argv) {
    const int lg = argc > 1 ? atoi(argv[1]) : 28;
    const int rounds = argc > 2 ? atoi(argv[2]) : 5;
    const uint64_t n = 1ull << lg;
    uint32_t *in, *ref, *out, *tc;
    unsigned long long *gs, *tot, *bases;
    CK(hipMalloc(&in, n * 4));
    CK(hipMalloc(&ref, n * 4));
    CK(hipMalloc(&out, n * 4));
    CK(hipMalloc(&tc, sweep_tiles(n) * kRadix * 4));
    CK(hipMalloc(&gs, scan_groups(n) * kRadix * 8));
    CK(hipMalloc(&tot, kRadix * 8));
    CK(hipMalloc(&bases, kRadix * 8));
    hipStream_t s;
    CK(hipStreamCreate(&s));
    CK(launch_generate(0, 42, 0, n, (int32_t *)in, s));
    const int shift = 8;  // a middle digit
    CK(launch_tile_counts(in, n, shift, false, tc, nullptr, s));
    CK(launch_scan_tiles(tc, n, (uint64_t *)gs, (uint64_t *)tot, (uint64_t *)bases, s));
    prod(in, ref, n, shift, tc, gs, bases, s);
    CK(hipStreamSynchronize(s));
    std::vector<V> vs = {
        {"prod_b512_i16", prod, true},
        {"rank0_b512_i16", run3<512, 16, 0, true, 1>, true},
        {"rank1_b512_i16", run3<512, 16, 1, true, 1>, true},
        {"rank1_b512_i16_minb3", run3<512, 16, 1, true, 3>, true},
        {"rank0_b512_i16_minb3", run3<512, 16, 0, true, 3>, true},
        {"rank1_b256_i32", run3<256, 32, 1, true, 1>, true},
        {"rank1_b1024_i8", run3<1024, 8, 1, true, 1>, true},
        {"rank2_fake_b512_i16", run3<512, 16, 2, true, 1>, false},
        {"rank1_nowrite_b512_i16", run3<512, 16, 1, false, 1>, false},
        {"rank2_nowrite_b512_i16", run3<512, 16, 2, false, 1>, false},
    };
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    std::vector<uint32_t> h_ref(n), h_out(n);
    CK(hipMemcpy(h_ref.data(), ref, n * 4, hipMemcpyDeviceToHost));
    for (int r = 0; r < rounds; ++r) {
        for (auto &v : vs) {
            CK(hipMemsetAsync(out, 0, n * 4, s));
            CK(hipEventRecord(e0, s));
            v.fn(in, out, n, shift, tc, gs, bases, s);
            CK(hipEventRecord(e1, s));
            CK(hipEventSynchronize(e1));
            float m;
            CK(hipEventElapsedTime(&m, e0, e1));
            v.t.push_back(m);
            if (r == 0 && v.check) {
                CK(hipMemcpy(h_out.data(), out, n * 4, hipMemcpyDeviceToHost));
                if (h_out != h_ref) { printf("MISMATCH %s\n", v.name); return 1; }
            }
        }
    }
    for (auto &v : vs) {
        std::sort(v.t.begin(), v.t.end());
        const float m = v.t[v.t.size() / 2];
        printf("{\"variant\": \"%s\", \"ms\": %.4f, \"GBps\": %.1f, \"checked\": %d}\n", v.name, m,
               n * 8.0 / (m * 1e-3) / 1e9, (int)v.check);
    }
    return 0;
}
