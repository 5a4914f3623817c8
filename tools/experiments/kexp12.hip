// kexp12.hip -- the two-level plan front end (K1h, K12h, K3a) in isolation (development tool):
// checks K1h's tile counts and K12h's child starts / tile plan against a host count, then the
// level-2 output of K3a bucket by bucket, and times K1h / K12h / K3a against K1 / K3u.
//   run: kexp12 [case=0] [rounds=5]
//   case 0: 256 values x 9000 copies, sorted; 1: 2^28 uniform 31-bit; 2: 1200 x 8190 sorted
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
// ---- K1h variants: 0 product form, 1 olds checked after the 8 atomics, 2 no-return h16
// atomics (no wrap repair; timing only), 3 no h16 histogram (tile counts only, same LDS)
template <int V>
__global__ __launch_bounds__(1024) void k1h_var(const uint32_t *__restrict__ in, uint64_t n,
                                                uint32_t *__restrict__ tcounts,
                                                uint32_t *__restrict__ part,
                                                unsigned long long *__restrict__ fix) {
    constexpr int BLOCK = 1024, ITEMS = 8;
    constexpr uint32_t kWords = kBuckets16 / 2;
    __shared__ uint32_t s_h[kWords];
    __shared__ uint32_t s_t[kRadix];
    const uint32_t tid = threadIdx.x;
    for (uint32_t i = tid; i < kWords; i += BLOCK) s_h[i] = 0;
    if (tid < kRadix) s_t[tid] = 0;
    const uint64_t ntiles = (n + kSweepTile - 1) / kSweepTile;
    uint32_t k[ITEMS];
    if (blockIdx.x < ntiles) {
        const uint64_t t0 = (uint64_t)blockIdx.x * kSweepTile;
        const uint32_t len = (uint32_t)min(n - t0, (uint64_t)kSweepTile);
        load_tile<BLOCK, ITEMS, true>(in + t0 + tid, len == (uint32_t)kSweepTile, len, k);
    }
    for (uint64_t t = blockIdx.x; t < ntiles; t += gridDim.x) {
        __syncthreads();
        const uint32_t len = (uint32_t)min(n - t * kSweepTile, (uint64_t)kSweepTile);
        const uint64_t tn = t + gridDim.x;
        uint32_t kn[ITEMS];
        if (tn < ntiles) {
            const uint64_t t0 = tn * kSweepTile;
            const uint32_t lenn = (uint32_t)min(n - t0, (uint64_t)kSweepTile);
            load_tile<BLOCK, ITEMS, true>(in + t0 + tid, lenn == (uint32_t)kSweepTile, lenn, kn);
        }
        if (V == 1) {
            uint32_t old[ITEMS];
#pragma unroll
            for (int i = 0; i < ITEMS; ++i) {
                old[i] = 0;
                if ((uint32_t)(i * BLOCK) + tid < len) {
                    atomicAdd(&s_t[k[i] >> 24], 1u);
                    const uint32_t b = k[i] >> 16, sh = (b & 1u) << 4;
                    old[i] = atomicAdd(&s_h[b >> 1], 1u << sh);
                }
            }
            bool any = false;
#pragma unroll
            for (int i = 0; i < ITEMS; ++i) {
                const uint32_t sh = ((k[i] >> 16) & 1u) << 4;
                any |= ((old[i] >> sh) & 0xffffu) == 0xffffu && (uint32_t)(i * BLOCK) + tid < len;
            }
            if (any) {
#pragma unroll
                for (int i = 0; i < ITEMS; ++i) {
                    const uint32_t b = k[i] >> 16, sh = (b & 1u) << 4;
                    if (((old[i] >> sh) & 0xffffu) == 0xffffu && (uint32_t)(i * BLOCK) + tid < len)
                        h16_wrap(fix, b, old[i]);
                }
            }
        } else {
#pragma unroll
            for (int i = 0; i < ITEMS; ++i) {
                if ((uint32_t)(i * BLOCK) + tid < len) {
                    atomicAdd(&s_t[k[i] >> 24], 1u);
                    const uint32_t b = k[i] >> 16, sh = (b & 1u) << 4;
                    if (V == 0) {
                        const uint32_t old = atomicAdd(&s_h[b >> 1], 1u << sh);
                        if (((old >> sh) & 0xffffu) == 0xffffu) h16_wrap(fix, b, old);
                    } else if (V == 2 || V == 4) {
                        atomicAdd(&s_h[b >> 1], 1u << sh);
                    }
                }
            }
        }
        __syncthreads();
        if (tid < kRadix) {
            tcounts[t * kRadix + tid] = s_t[tid];
            s_t[tid] = 0;
        }
        if (V == 4 && ((t - blockIdx.x) / gridDim.x) % 7 == 6) {
            for (uint32_t i = tid; i < kWords; i += BLOCK) {
                const uint32_t wv = s_h[i];
                if ((wv & 0xe000e000u) != 0) {
                    atomicAdd(&fix[2 * i], (unsigned long long)(wv & 0xffffu));
                    atomicAdd(&fix[2 * i + 1], (unsigned long long)(wv >> 16));
                    s_h[i] = 0;
                }
            }
        }
#pragma unroll
        for (int i = 0; i < ITEMS; ++i) k[i] = kn[i];
    }
    __syncthreads();
    uint32_t *dst = part + (uint64_t)blockIdx.x * kWords;
    for (uint32_t i = tid; i < kWords; i += BLOCK) dst[i] = s_h[i];
}

// ---- K3a variants: 0 u64 atomic (product; records the reservations in rec), 1 u32 atomic
// relative to the bucket start, 3 reservations read from rec (no atomics), 4 read from rec and
// the atomics issued but not waited for
template <int M>
__global__ __launch_bounds__(1024) void k3a_var(const uint32_t *__restrict__ in,
                                                uint32_t *__restrict__ out,
                                                const uint32_t *__restrict__ tpfx,
                                                const unsigned long long *__restrict__ bases,
                                                const unsigned long long *__restrict__ totals,
                                                unsigned long long *__restrict__ cur,
                                                unsigned long long *__restrict__ rec) {
    constexpr int BLOCK = 1024, ITEMS = 8, TILE = 8192;
    __shared__ uint32_t s_keys[TILE];
    __shared__ uint32_t s_cur[kRadix];
    __shared__ uint32_t *s_dst[kRadix];
    __shared__ uint32_t s_wsum[kRadix / 64];
    __shared__ uint32_t s_tp[kRadix + 1];
    const uint32_t tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    if (tid <= kRadix) s_tp[tid] = tpfx[tid];
    __syncthreads();
    const uint32_t t = xcd_tile(blockIdx.x, gridDim.x);
    if (t >= s_tp[kRadix]) return;
    uint32_t lo = 0, hi = kRadix;
    while (hi - lo > 1) {
        const uint32_t mid = (lo + hi) >> 1;
        if (s_tp[mid] <= t) lo = mid;
        else hi = mid;
    }
    const uint64_t b0 = bases[lo], end = b0 + totals[lo];
    const uint64_t t0 = b0 + (uint64_t)(t - s_tp[lo]) * TILE;
    const uint32_t len = (uint32_t)(end - t0 < (uint64_t)TILE ? end - t0 : (uint64_t)TILE);
    const bool full = len == (uint32_t)TILE;
    const int shift = 16;
    if (tid < kRadix) s_cur[tid] = 0;
    uint32_t k[ITEMS];
    load_tile<BLOCK, ITEMS, false>(in + t0 + tid, full, len, k);
    __syncthreads();
    uint32_t r[ITEMS];
#pragma unroll
    for (int i = 0; i < ITEMS; ++i)
        if (full || (uint32_t)(i * BLOCK + tid) < len)
            r[i] = atomicAdd(&s_cur[(k[i] >> shift) & 255u], 1u);
    __syncthreads();
    uint32_t c = 0, excl = 0;
    unsigned long long pos = 0;
    if (tid < kRadix) {
        c = s_cur[tid];
        unsigned int *c32 = reinterpret_cast<unsigned int *>(cur);
        if (M == 0 && c) { pos = atomicAdd(&cur[lo * kRadix + tid], (unsigned long long)c); rec[(uint64_t)t * kRadix + tid] = pos; }
        if (M == 1 && c) pos = b0 + atomicAdd(&c32[lo * kRadix + tid], c);
        if (M == 3 || M == 4) pos = rec[(uint64_t)t * kRadix + tid];
        if (M == 4 && c) atomicAdd(&c32[65536 * 2 + lo * kRadix + tid], c);
        uint32_t v = c;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const uint32_t tt = __shfl_up(v, o);
            if (lane >= o) v += tt;
        }
        if (lane == 63) s_wsum[w] = v;
        excl = v - c;
    }
    __syncthreads();
    if (tid < kRadix) {
        for (int ww = 0; ww < (int)w; ++ww) excl += s_wsum[ww];
        s_cur[tid] = excl;
    }
    __syncthreads();
#pragma unroll
    for (int i = 0; i < ITEMS; ++i)
        if (full || (uint32_t)(i * BLOCK + tid) < len)
            s_keys[s_cur[(k[i] >> shift) & 255u] + r[i]] = k[i];
    if (tid < kRadix) s_dst[tid] = out + pos - excl;
    __syncthreads();
#pragma unroll
    for (int i = 0; i < ITEMS; ++i) {
        const uint32_t j = (uint32_t)(i * BLOCK + tid);
        if (full || j < len) {
            const uint32_t key = s_keys[j];
            s_dst[(key >> shift) & 255u][j] = key;
        }
    }
}

__global__ void k_cur32(const unsigned long long *cstart, const unsigned long long *bases,
                        unsigned int *c32) {
    const uint32_t i = blockIdx.x * 256 + threadIdx.x;
    c32[i] = (unsigned int)(cstart[i] - bases[i >> 8]);
    c32[65536 * 2 + i] = 0;
}
}  // namespace

int main(int argc, char **argv) {
    const int cs = argc > 1 ? atoi(argv[1]) : 0;
    const int rounds = argc > 2 ? atoi(argv[2]) : 5;
    std::vector<int32_t> h;
    if (cs == 0) {
        for (int v = 0; v < 256; ++v) h.insert(h.end(), 9000, v * 65536);
    } else if (cs == 2) {
        for (int v = -600; v < 600; ++v) h.insert(h.end(), 8190, v * 65536);
    } else {
        h.resize(1u << 28);
        uint64_t z = 42;
        for (auto &x : h) {
            z += 0x9E3779B97F4A7C15ULL;
            uint64_t y = z;
            y = (y ^ (y >> 30)) * 0xBF58476D1CE4E5B9ULL;
            y = (y ^ (y >> 27)) * 0x94D049BB133111EBULL;
            y ^= y >> 31;
            x = (int32_t)(y >> 33);
        }
    }
    const uint64_t n = h.size(), tiles = sweep_tiles(n);
    printf("case %d n %llu tiles %llu\n", cs, (unsigned long long)n, (unsigned long long)tiles);
    // host reference: tile top-digit counts, 16-bit counts
    std::vector<uint32_t> tc(tiles * 256, 0);
    std::vector<uint64_t> c16(65536, 0);
    for (uint64_t i = 0; i < n; ++i) {
        const uint32_t u = (uint32_t)h[i] ^ 0x80000000u;
        tc[(i / kSweepTile) * 256 + (u >> 24)]++;
        c16[u >> 16]++;
    }
    std::vector<uint64_t> cs16(65537, 0);
    for (int i = 0; i < 65536; ++i) cs16[i + 1] = cs16[i] + c16[i];

    uint32_t *d_in, *d_tmp, *d_out, *d_tc, *d_part, *d_tpfx;
    uint64_t *d_fix, *d_gsum, *d_small, *d_cstart, *d_cur, *d_lists;
    CK(hipMalloc(&d_in, n * 4));
    CK(hipMalloc(&d_tmp, n * 4));
    CK(hipMalloc(&d_out, n * 4));
    CK(hipMalloc(&d_tc, tiles * 256 * 4 + 4096));
    CK(hipMalloc(&d_part, (size_t)kH16Blocks * kH16PartWords * 4));
    CK(hipMalloc(&d_tpfx, 257 * 4));
    CK(hipMalloc(&d_fix, 65536 * 8));
    CK(hipMalloc(&d_gsum, (scan_groups(n) + 1) * 256 * 8));
    CK(hipMalloc(&d_small, 4096 * 8));
    CK(hipMalloc(&d_cstart, 65537 * 8));
    CK(hipMalloc(&d_cur, 65536 * 8));
    CK(hipMalloc(&d_lists, 8 * 65536 * 16));
    CK(hipMemcpy(d_in, h.data(), n * 4, hipMemcpyHostToDevice));
    uint64_t *totals = d_small, *bases = d_small + 256, *ctr = d_small + 1024;
    WorkLists wl2, wl3;
    for (int k = 0; k < 4; ++k) {
        wl2.list[k] = d_lists + (size_t)k * 65536 * 2;
        wl3.list[k] = d_lists + (size_t)(4 + k) * 65536 * 2;
    }
    wl2.ctr = ctr;
    wl3.ctr = ctr + 16;
    wl2.force_next = wl3.force_next = false;
    hipEvent_t ev[6];
    for (auto &x : ev) CK(hipEventCreate(&x));
    float t_k1h = 0, t_plan = 0, t_l3 = 0, t_l2 = 0;
    for (int r = 0; r < rounds; ++r) {
        uint32_t nblk = 0;
        CK(hipMemset(d_fix, 0, 65536 * 8));
        CK(hipMemset(ctr, 0, 64 * 8));
        CK(hipEventRecord(ev[0], 0));
        CK(launch_counts_h16(d_in, n, true, d_tc, d_part, d_fix, &nblk, 0));
        CK(hipEventRecord(ev[1], 0));
        if (r == 0) {
            std::vector<uint32_t> g(tiles * 256);
            CK(hipMemcpy(g.data(), d_tc, tiles * 256 * 4, hipMemcpyDeviceToHost));
            uint64_t bad = 0;
            for (uint64_t i = 0; i < tiles * 256; ++i)
                if (g[i] != tc[i] && bad++ < 5)
                    printf("tcount tile %llu d %llu: got %u want %u\n", (unsigned long long)(i / 256),
                           (unsigned long long)(i % 256), g[i], tc[i]);
            printf("tcounts bad %llu (nblk %u)\n", (unsigned long long)bad, nblk);
        }
        CK(launch_scan_tiles(d_tc, n, d_gsum, totals, bases, 0));
        CK(launch_plan_h16(d_part, nblk, d_fix, bases, totals, n, false, d_cstart, reinterpret_cast<uint32_t *>(d_cur), d_tpfx,
                           wl2, wl3, 0));
        CK(hipEventRecord(ev[2], 0));
        CK(launch_partition(d_in, d_tmp, n, 24, d_tc, d_gsum, bases, true, 0));
        CK(hipEventRecord(ev[3], 0));
        CK(launch_partition_h16(d_tmp, d_out, nullptr, n, d_tpfx, bases, totals, reinterpret_cast<uint32_t *>(d_cur), 0));
        CK(hipEventRecord(ev[4], 0));
        CK(hipDeviceSynchronize());
        float a, b, c, d;
        CK(hipEventElapsedTime(&a, ev[0], ev[1]));
        CK(hipEventElapsedTime(&b, ev[1], ev[2]));
        CK(hipEventElapsedTime(&c, ev[2], ev[3]));
        CK(hipEventElapsedTime(&d, ev[3], ev[4]));
        if (r > 0) { t_k1h += a; t_plan += b; t_l3 += c; t_l2 += d; }
        if (r == 0) {
            std::vector<uint64_t> g(65537);
            CK(hipMemcpy(g.data(), d_cstart, 65537 * 8, hipMemcpyDeviceToHost));
            uint64_t bad = 0;
            for (int i = 0; i <= 65536; ++i)
                if (g[i] != cs16[i] && bad++ < 5)
                    printf("cstart %d: got %llu want %llu\n", i, (unsigned long long)g[i],
                           (unsigned long long)cs16[i]);
            printf("cstart bad %llu\n", (unsigned long long)bad);
            std::vector<uint32_t> tp(257);
            CK(hipMemcpy(tp.data(), d_tpfx, 257 * 4, hipMemcpyDeviceToHost));
            printf("tpfx[256] %u\n", tp[256]);
            std::vector<uint32_t> o(n);
            CK(hipMemcpy(o.data(), d_out, n * 4, hipMemcpyDeviceToHost));
            uint64_t badk = 0;
            for (int b16 = 0; b16 < 65536; ++b16)
                for (uint64_t i = cs16[b16]; i < cs16[b16 + 1]; ++i)
                    if ((o[i] >> 16) != (uint32_t)b16 && badk++ < 5)
                        printf("out[%llu] = %08x not in bucket %04x\n", (unsigned long long)i, o[i],
                               b16);
            printf("level-2 misplaced %llu\n", (unsigned long long)badk);
            uint64_t hc[48];
            CK(hipMemcpy(hc, ctr, sizeof(hc), hipMemcpyDeviceToHost));
            printf("wl2 ctr:");
            for (int i = 0; i < 12; ++i) printf(" %llu", (unsigned long long)hc[i]);
            printf("\nwl3 ctr:");
            for (int i = 16; i < 28; ++i) printf(" %llu", (unsigned long long)hc[i]);
            printf("\n");
        }
    }
    const int m = std::max(rounds - 1, 1);

    {
        // K1h variants
        uint32_t nblk = std::min<uint64_t>(tiles, kH16Blocks);
        for (int v = 0; v < 5; ++v) {
            float tot = 0;
            for (int r = 0; r < rounds; ++r) {
                CK(hipMemset(d_fix, 0, 65536 * 8));
                CK(hipEventRecord(ev[0], 0));
                if (v == 0) k1h_var<0><<<nblk, 1024>>>(d_in, n, d_tc, d_part, reinterpret_cast<unsigned long long *>(d_fix));
                if (v == 1) k1h_var<1><<<nblk, 1024>>>(d_in, n, d_tc, d_part, reinterpret_cast<unsigned long long *>(d_fix));
                if (v == 2) k1h_var<2><<<nblk, 1024>>>(d_in, n, d_tc, d_part, reinterpret_cast<unsigned long long *>(d_fix));
                if (v == 3) k1h_var<3><<<nblk, 1024>>>(d_in, n, d_tc, d_part, reinterpret_cast<unsigned long long *>(d_fix));
                if (v == 4) k1h_var<4><<<nblk, 1024>>>(d_in, n, d_tc, d_part, reinterpret_cast<unsigned long long *>(d_fix));
                CK(hipEventRecord(ev[1], 0));
                CK(hipDeviceSynchronize());
                float a;
                CK(hipEventElapsedTime(&a, ev[0], ev[1]));
                if (r) tot += a;
            }
            printf("{\"k1h_variant\": %d, \"ms\": %.4f}\n", v, tot / m);
        }
        // restore a correct plan for the K3a variants
        uint32_t nb2 = 0;
        CK(hipMemset(d_fix, 0, 65536 * 8));
        CK(launch_counts_h16(d_in, n, true, d_tc, d_part, d_fix, &nb2, 0));
        CK(launch_scan_tiles(d_tc, n, d_gsum, totals, bases, 0));
        CK(launch_plan_h16(d_part, nb2, d_fix, bases, totals, n, false, d_cstart, reinterpret_cast<uint32_t *>(d_cur), d_tpfx,
                           wl2, wl3, 0));
        CK(launch_partition(d_in, d_tmp, n, 24, d_tc, d_gsum, bases, true, 0));
        unsigned long long *rec;
        CK(hipMalloc(&rec, (tiles + 256) * 256 * 8));
        unsigned long long *cur2;
        CK(hipMalloc(&cur2, 65536 * 8 * 2));
        const unsigned g = (unsigned)(tiles + 256);
        auto ull = [](uint64_t *p) { return reinterpret_cast<unsigned long long *>(p); };
        for (int v : {0, 1, 3, 4}) {
            float tot = 0;
            for (int r = 0; r < rounds; ++r) {
                CK(hipMemcpy(cur2, d_cstart, 65536 * 8, hipMemcpyDeviceToDevice));
                if (v == 1 || v == 4)
                    k_cur32<<<256, 256>>>(ull(d_cstart), ull(bases), reinterpret_cast<unsigned int *>(cur2));
                CK(hipEventRecord(ev[0], 0));
                if (v == 0) k3a_var<0><<<g, 1024>>>(d_tmp, d_out, d_tpfx, ull(bases), ull(totals), cur2, rec);
                if (v == 1) k3a_var<1><<<g, 1024>>>(d_tmp, d_out, d_tpfx, ull(bases), ull(totals), cur2, rec);
                if (v == 3) k3a_var<3><<<g, 1024>>>(d_tmp, d_out, d_tpfx, ull(bases), ull(totals), cur2, rec);
                if (v == 4) k3a_var<4><<<g, 1024>>>(d_tmp, d_out, d_tpfx, ull(bases), ull(totals), cur2, rec);
                CK(hipEventRecord(ev[1], 0));
                CK(hipDeviceSynchronize());
                float a;
                CK(hipEventElapsedTime(&a, ev[0], ev[1]));
                if (r) tot += a;
            }
            printf("{\"k3a_variant\": %d, \"ms\": %.4f}\n", v, tot / m);
        }
    }
    printf("{\"ms_k1h\": %.4f, \"ms_scan_plan\": %.4f, \"ms_l3\": %.4f, \"ms_k3a\": %.4f}\n",
           t_k1h / m, t_plan / m, t_l3 / m, t_l2 / m);
    return 0;
}
