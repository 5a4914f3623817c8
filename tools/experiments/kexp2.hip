// kexp2.hip -- unstable (MSD-style) partition pass experiments (development tool).
// K3u: scatter a tile by one digit with LDS atomic ranks (no ballots): the order inside a digit
// run is arbitrary, which is fine for an MSD partition of a keys-only sort.
//   A: ranks from ds_add_rtn on per-tile counters, scan after a barrier
//   B: ranks from ds_add_rtn on cursors pre-set from the tile's K1 counts (one atomic = final
//      LDS slot, no barrier between ranking and scatter)
// Checks: output is partitioned by the digit (non-decreasing digit) and a permutation
// (sum/xor of mix64) of the input.
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

template <int BLOCK, int ITEMS, int MODE>
__global__ __launch_bounds__(BLOCK) void k3u(const uint32_t *__restrict__ in,
                                             uint32_t *__restrict__ out, uint64_t n, int shift,
                                             const uint32_t *__restrict__ tcnt,
                                             const uint32_t *__restrict__ toff,
                                             const unsigned long long *__restrict__ gpfx,
                                             const unsigned long long *__restrict__ bases) {
    constexpr int TILE = BLOCK * ITEMS;
    __shared__ uint32_t s_keys[TILE];
    __shared__ uint32_t s_cur[kRadix];
    __shared__ uint32_t *s_dst[kRadix];
    __shared__ uint32_t s_wsum[kRadix / 64];
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const uint32_t tile = xcd_tile(blockIdx.x, gridDim.x);
    const uint64_t tbase = (uint64_t)tile * TILE;
    const bool full = tbase + TILE <= n;
    const uint32_t lim = full ? (uint32_t)TILE : (uint32_t)(n - tbase);
    uint32_t *dst_base = nullptr;
    uint32_t c = 0;
    if (tid < kRadix) {
        dst_base = out + bases[tid] + gpfx[(uint64_t)(tile / kScanGroup) * kRadix + tid] +
                   toff[(uint64_t)tile * kRadix + tid];
        if (MODE == 0) s_cur[tid] = 0;
        else c = tcnt[(uint64_t)tile * kRadix + tid];
    }
    uint32_t k[ITEMS];
    const uint32_t *src = in + tbase + tid;
#pragma unroll
    for (int i = 0; i < ITEMS; ++i)
        k[i] = (full || (uint32_t)(i * BLOCK + tid) < lim) ? src[i * BLOCK] : 0u;
    auto scan_digits = [&](uint32_t cnt) {  // tid < 256: exclusive scan of cnt over digits
        uint32_t v = cnt;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const uint32_t t = __shfl_up(v, o);
            if (lane >= o) v += t;
        }
        if (lane == 63) s_wsum[w] = v;
        return v - cnt;
    };
    if (MODE == 0) {
        __syncthreads();
        uint32_t r[ITEMS];
#pragma unroll
        for (int i = 0; i < ITEMS; ++i)
            if (full || (uint32_t)(i * BLOCK + tid) < lim)
                r[i] = atomicAdd(&s_cur[(k[i] >> shift) & 255u], 1u);
        __syncthreads();
        uint32_t excl = 0;
        if (tid < kRadix) excl = scan_digits(s_cur[tid]);
        __syncthreads();
        if (tid < kRadix) {
            for (int ww = 0; ww < w; ++ww) excl += s_wsum[ww];
            s_cur[tid] = excl;
            s_dst[tid] = dst_base - excl;
        }
        __syncthreads();
#pragma unroll
        for (int i = 0; i < ITEMS; ++i)
            if (full || (uint32_t)(i * BLOCK + tid) < lim)
                s_keys[s_cur[(k[i] >> shift) & 255u] + r[i]] = k[i];
    } else {
        uint32_t excl = 0;
        if (tid < kRadix) excl = scan_digits(c);
        __syncthreads();
        if (tid < kRadix) {
            for (int ww = 0; ww < w; ++ww) excl += s_wsum[ww];
            s_cur[tid] = excl;
            s_dst[tid] = dst_base - excl;
        }
        __syncthreads();
#pragma unroll
        for (int i = 0; i < ITEMS; ++i)
            if (full || (uint32_t)(i * BLOCK + tid) < lim)
                s_keys[atomicAdd(&s_cur[(k[i] >> shift) & 255u], 1u)] = k[i];
    }
    __syncthreads();
#pragma unroll
    for (int i = 0; i < ITEMS; ++i) {
        const uint32_t j = (uint32_t)(i * BLOCK + tid);
        if (full || j < lim) {
            const uint32_t key = s_keys[j];
            s_dst[(key >> shift) & 255u][j] = key;
        }
    }
}

typedef void (*Fn)(const uint32_t *, uint32_t *, uint64_t, int, const uint32_t *, const uint32_t *,
                   const unsigned long long *, const unsigned long long *, hipStream_t);
template <int B, int I, int MODE>
void run(const uint32_t *in, uint32_t *out, uint64_t n, int shift, const uint32_t *tc,
         const uint32_t *toff, const unsigned long long *gp, const unsigned long long *bs,
         hipStream_t s) {
    k3u<B, I, MODE><<<(unsigned)sweep_tiles(n), B, 0, s>>>(in, out, n, shift, tc, toff, gp, bs);
}
void prod(const uint32_t *in, uint32_t *out, uint64_t n, int shift, const uint32_t *,
          const uint32_t *toff, const unsigned long long *gp, const unsigned long long *bs,
          hipStream_t s) {
    (void)launch_scatter(in, out, n, shift, toff, (const uint64_t *)gp, (const uint64_t *)bs,
                         false, false, s);
}
void prod_u(const uint32_t *in, uint32_t *out, uint64_t n, int shift, const uint32_t *,
            const uint32_t *toff, const unsigned long long *gp, const unsigned long long *bs,
            hipStream_t s) {
    (void)launch_partition(in, out, n, shift, toff, (const uint64_t *)gp, (const uint64_t *)bs,
                           false, s);
}
struct V { const char *name; Fn fn; std::vector<float> t; bool check = true; };
uint64_t mix(uint64_t z) {
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
    return z ^ (z >> 31);
}
}  // namespace

int main(int argc, char **argv) {
    const int lg = argc > 1 ? atoi(argv[1]) : 28;
    const int rounds = argc > 2 ? atoi(argv[2]) : 5;
    const int shift = argc > 3 ? atoi(argv[3]) : 24;
    const uint64_t n = 1ull << lg;
    uint32_t *in, *out, *tc, *tc_raw;
    unsigned long long *gs, *tot, *bases;
    CK(hipMalloc(&in, n * 4));
    CK(hipMalloc(&out, n * 4));
    CK(hipMalloc(&tc, sweep_tiles(n) * kRadix * 4));
    CK(hipMalloc(&tc_raw, sweep_tiles(n) * kRadix * 4));
    CK(hipMalloc(&gs, scan_groups(n) * kRadix * 8));
    CK(hipMalloc(&tot, kRadix * 8));
    CK(hipMalloc(&bases, kRadix * 8));
    hipStream_t s;
    CK(hipStreamCreate(&s));
    CK(launch_generate(0, 42, 0, n, (int32_t *)in, s));
    const uint32_t data_xor = argc > 4 ? (uint32_t)strtoul(argv[4], nullptr, 0) : 0u;
    if (data_xor) {  // re-map the keys (e.g. 0x80000000: top digit 128..255 instead of 0..127)
        std::vector<uint32_t> h(n);
        CK(hipMemcpy(h.data(), in, n * 4, hipMemcpyDeviceToHost));
        for (auto &x : h) x ^= data_xor;
        CK(hipMemcpy(in, h.data(), n * 4, hipMemcpyHostToDevice));
    }
    CK(launch_tile_counts(in, n, shift, false, tc, nullptr, s));
    CK(hipMemcpyAsync(tc_raw, tc, sweep_tiles(n) * kRadix * 4, hipMemcpyDeviceToDevice, s));
    CK(launch_scan_tiles(tc, n, (uint64_t *)gs, (uint64_t *)tot, (uint64_t *)bases, s));
    CK(hipStreamSynchronize(s));
    std::vector<uint32_t> h_in(n), h_out(n);
    CK(hipMemcpy(h_in.data(), in, n * 4, hipMemcpyDeviceToHost));
    uint64_t s_in = 0, x_in = 0;
    for (uint64_t i = 0; i < n; ++i) { uint64_t m = mix(h_in[i]); s_in += m; x_in ^= m; }
    std::vector<V> vs = {
        {"prod_stable_b512_i16", prod},
        {"u_A_b512_i16", run<512, 16, 0>},
        {"u_B_b512_i16", run<512, 16, 1>},
        {"u_B_b256_i32", run<256, 32, 1>},
        {"u_B_b1024_i8", run<1024, 8, 1>},
        {"u_A_b1024_i8", run<1024, 8, 0>},
        {"prod_partition", prod_u},
    };
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    for (int r = 0; r < rounds; ++r) {
        for (auto &v : vs) {
            CK(hipEventRecord(e0, s));
            v.fn(in, out, n, shift, tc_raw, tc, gs, bases, s);
            CK(hipEventRecord(e1, s));
            CK(hipEventSynchronize(e1));
            float m;
            CK(hipEventElapsedTime(&m, e0, e1));
            v.t.push_back(m);
            if (r == 0 && v.check) {
                CK(hipMemcpy(h_out.data(), out, n * 4, hipMemcpyDeviceToHost));
                uint64_t so = 0, xo = 0, bad = 0;
                for (uint64_t i = 0; i < n; ++i) {
                    uint64_t mm = mix(h_out[i]); so += mm; xo ^= mm;
                    if (i && ((h_out[i] >> shift) & 255u) < ((h_out[i - 1] >> shift) & 255u)) ++bad;
                }
                if (so != s_in || xo != x_in || bad) {
                    printf("FAIL %s bad=%llu\n", v.name, (unsigned long long)bad);
                    return 1;
                }
            }
        }
    }
    {   // the MSD level-3 sequence exactly as msd_sort issues it: int32 input, flipped counts
        std::vector<float> tk1, tk3;
        for (int r = 0; r < rounds; ++r) {
            CK(hipEventRecord(e0, s));
            CK(launch_tile_counts(in, n, 24, true, tc, nullptr, s));
            CK(launch_scan_tiles(tc, n, (uint64_t *)gs, (uint64_t *)tot, (uint64_t *)bases, s));
            hipEvent_t e2 = e1;
            CK(hipEventRecord(e2, s));
            CK(hipEventSynchronize(e2));
            float m;
            CK(hipEventElapsedTime(&m, e0, e2));
            tk1.push_back(m);
            CK(hipEventRecord(e0, s));
            CK(launch_partition(in, out, n, 24, tc, (const uint64_t *)gs, (const uint64_t *)bases,
                                true, s));
            CK(hipEventRecord(e1, s));
            CK(hipEventSynchronize(e1));
            CK(hipEventElapsedTime(&m, e0, e1));
            tk3.push_back(m);
        }
        std::sort(tk1.begin(), tk1.end());
        std::sort(tk3.begin(), tk3.end());
        printf("{\"variant\": \"msd_level3_k1k2_flip\", \"ms\": %.4f}\n", tk1[tk1.size() / 2]);
        printf("{\"variant\": \"msd_level3_partition_flip\", \"ms\": %.4f, \"GBps\": %.1f}\n",
               tk3[tk3.size() / 2], n * 8.0 / (tk3[tk3.size() / 2] * 1e-3) / 1e9);
    }
    for (auto &v : vs) {
        std::sort(v.t.begin(), v.t.end());
        const float m = v.t[v.t.size() / 2];
        printf("{\"variant\": \"%s\", \"ms\": %.4f, \"GBps\": %.1f}\n", v.name, m,
               n * 8.0 / (m * 1e-3) / 1e9);
    }
    return 0;
}
