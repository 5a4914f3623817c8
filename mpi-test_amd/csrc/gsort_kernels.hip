// gsort_kernels.hip -- hand-written CDNA4 (gfx950) kernels of the distributed sorter.
//
// Keys are int32; every kernel that compares digits works on the order-preserving map
// u = key ^ 0x80000000 (unsigned order of u == signed order of key).  The local sort is an
// 8-bit LSD radix sort in "onesweep" form: one read builds all four digit histograms (K1),
// then each pass (K3) ranks a tile with wave64 ballots, takes its global digit offsets from a
// single-pass decoupled lookback, and scatters through LDS so the global stores come out in
// digit runs.  Algorithmic traffic: 4 B/key for K1 + 8 B/key per pass.
//
// Reference hot loops these replace (cites /root/reference/...):
//   K1/K3  mpi_radix_sort.c:144-147 (number_digit_at + bucket_push per key), :54-58, :33-43;
//          and the local qsort of mpi_sample_sort.c:85 and :174
//   K4     mpi_sample_sort.c:89-105 regular sampling
//   K5     mpi_sample_sort.c:109-125 sort samples at the root, pick splitters
//   K6     mpi_sample_sort.c:148-155 bucket partition (here: bounds on the sorted block)
//   K8     mpi_radix_sort.c:164-192 per-pass placement (receive side of the exchange)
#include "gsort_kernels.h"

namespace gsort {
namespace {

constexpr uint32_t kFlip = 0x80000000u;
constexpr uint64_t kGolden = 0x9E3779B97F4A7C15ULL;
constexpr uint64_t kCountMask = (1ULL << 46) - 1;

__device__ __forceinline__ uint64_t mix64(uint64_t z) {
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
    return z ^ (z >> 31);
}

__device__ __forceinline__ uint64_t ld_agent(const unsigned long long *p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_agent(unsigned long long *p, uint64_t v) {
    __hip_atomic_store(p, (unsigned long long)v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ uint64_t pack_status(uint32_t epoch, uint64_t flag, uint64_t cnt) {
    return ((uint64_t)epoch << 48) | (flag << 46) | cnt;
}

// ---------------------------------------------------------------------------------------
// K10: canonical splitmix64 stream; identical to oracle.c orc_gen_one.
// ---------------------------------------------------------------------------------------
__global__ void k_generate(int dist, uint64_t seed, uint64_t start, uint64_t n, int32_t *out) {
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
        const uint64_t z = mix64(seed + (start + i + 1) * kGolden);
        int32_t key;
        if (dist == 0) {
            key = (int32_t)(z >> 33);
        } else {
            const double u = (double)((z >> 11) + 1) * 0x1p-53;
            const double uu = __dmul_rn(u, u);
            double k = floor(__ddiv_rn(1.0, uu));
            if (k > 2147483647.0) k = 2147483647.0;
            key = (int32_t)k;
        }
        out[i] = key;
    }
}

// ---------------------------------------------------------------------------------------
// K1: all four digit histograms in one read.  Per-wave private LDS bins (4 x 256 per wave)
// absorb the contention of duplicate-heavy inputs; one global atomic per non-zero bin.
// ---------------------------------------------------------------------------------------
template <int BLOCK, bool VEC>
__global__ __launch_bounds__(BLOCK) void k_hist4(const uint32_t *__restrict__ in, uint64_t n,
                                                 unsigned long long *__restrict__ hist) {
    constexpr int WAVES = BLOCK / 64;
    __shared__ uint32_t sh[WAVES * 4 * kRadix];
    for (int i = threadIdx.x; i < WAVES * 4 * kRadix; i += BLOCK) sh[i] = 0;
    __syncthreads();
    uint32_t *my = sh + (threadIdx.x >> 6) * 4 * kRadix;
    auto count = [&](uint32_t u) {
        u ^= kFlip;
        atomicAdd(&my[u & 255u], 1u);
        atomicAdd(&my[kRadix + ((u >> 8) & 255u)], 1u);
        atomicAdd(&my[2 * kRadix + ((u >> 16) & 255u)], 1u);
        atomicAdd(&my[3 * kRadix + (u >> 24)], 1u);
    };
    const uint64_t stride = (uint64_t)gridDim.x * BLOCK;
    const uint64_t t0 = (uint64_t)blockIdx.x * BLOCK + threadIdx.x;
    uint64_t done = 0;
    if (VEC) {
        const uint64_t nv = n / 4;
        const uint4 *in4 = reinterpret_cast<const uint4 *>(in);
        for (uint64_t v = t0; v < nv; v += stride) {
            const uint4 q = in4[v];
            count(q.x); count(q.y); count(q.z); count(q.w);
        }
        done = nv * 4;
    }
    for (uint64_t i = done + t0; i < n; i += stride) count(in[i]);
    __syncthreads();
    for (int b = threadIdx.x; b < 4 * kRadix; b += BLOCK) {
        uint32_t s = 0;
#pragma unroll
        for (int w = 0; w < WAVES; ++w) s += sh[w * 4 * kRadix + b];
        if (s) atomicAdd(&hist[b], (unsigned long long)s);
    }
}

// ---------------------------------------------------------------------------------------
// Decoupled lookback for digit d of `tile` (one thread): W predecessor status words are in
// flight per round trip (MI355X cross-XCD sc1 loads cost ~1 us under load, so a one-word walk
// over the tiles still in flight was the pass's bottleneck).  Sums AGGREGATEs back to the
// first INCLUSIVE; on a not-yet-published word it sleeps and re-polls from there.  Bounded:
// gives up (sets *err) instead of hanging.
// ---------------------------------------------------------------------------------------
#ifdef GSORT_KBENCH_STAMPS
// Diagnostic build only (tools/kbench.hip defines the macro; the product never does): per-tile
// phase timestamps (s_memrealtime, 100 MHz) and digit-0 lookback round trips / spins.
__device__ unsigned long long *g_stamps;
#define GSORT_STAMP(slot) \
    if (threadIdx.x == 0) g_stamps[(uint64_t)tile * 8 + (slot)] = __builtin_amdgcn_s_memrealtime()
#else
#define GSORT_STAMP(slot)
#endif
// rounds / spins report the round trips and not-ready re-polls (diagnostics; dead otherwise)
template <int W>
__device__ __forceinline__ uint64_t lookback(const unsigned long long *status, uint32_t tile,
                                             int d, uint32_t epoch, uint32_t *err,
                                             uint32_t &rounds, uint32_t &spins_out) {
    uint64_t prefix = 0;
    int64_t t = (int64_t)tile - 1;  // nearest predecessor not yet consumed
    uint32_t spins = 0;
    while (t >= 0) {
        uint64_t wv[W];
#pragma unroll
        for (int j = 0; j < W; ++j)
            wv[j] = (t - j >= 0) ? ld_agent(status + (uint64_t)(t - j) * kRadix + d)
                                 : pack_status(epoch, kFlagInc, 0);
        int consumed = 0;
        bool stop = false, fin = false;
#pragma unroll
        for (int j = 0; j < W; ++j) {
            if (!stop) {
                const uint32_t ep = (uint32_t)(wv[j] >> 48);
                const uint64_t fl = (wv[j] >> 46) & 3u;
                if (ep != epoch || fl == 0) {
                    stop = true;
                } else {
                    prefix += wv[j] & kCountMask;
                    ++consumed;
                    if (fl == kFlagInc) stop = fin = true;
                }
            }
        }
        ++rounds;
        if (fin) break;
        t -= consumed;
        if (consumed < W) {
            if (++spins > (1u << 22)) {
                atomicOr(err, 1u);
                break;
            }
            __builtin_amdgcn_s_sleep(1);
        }
    }
    spins_out = spins;
    return prefix;
}

// ---------------------------------------------------------------------------------------
// K3: one stable onesweep LSD pass.
//   tile = BLOCK * ITEMS keys; wave w owns keys [w*64*ITEMS, (w+1)*64*ITEMS) of the tile,
//   round i of the wave holds keys i*64 + lane, so (round, lane) order == memory order.
//   1. rank: for each round, 8 ballots give each lane the mask of lanes sharing its digit
//      (per bit: v_bfe_i32, v_cmp, two v_bitop3); rank = (wave's running count of the digit)
//      + (#peers below the lane); every peer writes the same advanced count (branch-free).
//   2. per-digit tile counts -> publish AGGREGATE; block-exclusive digit starts folded into
//      the per-wave offset table.
//   3. scatter keys into LDS in block-sorted order (stable); meanwhile one thread per digit
//      runs the decoupled lookback over previous tiles' status words -> global offsets.
//   4. stream LDS out in order: consecutive lanes hit consecutive addresses within a digit.
// Tile ids come from an atomic counter, so every tile a lookback waits on is already running.
// LB_EARLY runs the lookback right after publishing the aggregate (so this tile's inclusive
// prefix is published as early as possible) instead of after the LDS scatter.
// NO_LOOKBACK is an ablation switch for timing-only builds (tools/kbench.hip): it skips the
// lookback wait (prefix = 0, wrong output) and is never set in the product.
// ---------------------------------------------------------------------------------------
template <int BLOCK, int ITEMS, bool FIN, bool FOUT, bool NO_LOOKBACK = false,
          bool LB_EARLY = true, int LB_W = 8>
__global__ __launch_bounds__(BLOCK) void k_onesweep(const uint32_t *__restrict__ in,
                                                    uint32_t *__restrict__ out, uint64_t n,
                                                    int shift,
                                                    const unsigned long long *__restrict__ base,
                                                    unsigned long long *status,
                                                    uint32_t *tile_ctr, uint32_t *err,
                                                    uint32_t epoch) {
    constexpr int WAVES = BLOCK / 64;
    constexpr int TILE = BLOCK * ITEMS;
    static_assert(BLOCK >= kRadix, "one thread per digit in the scan/lookback");
    static_assert(TILE <= 65536, "ranks are packed as 16 bits");
    __shared__ uint32_t s_keys[TILE];
    __shared__ uint32_t s_wofs[WAVES * kRadix];  // per-wave counts, then per-wave tile offsets
    __shared__ uint32_t *s_dst[kRadix];          // out + global offset - tile start, by digit
    __shared__ uint32_t s_wsum[kRadix / 64];
    __shared__ uint32_t s_tile;

    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int w = tid >> 6;
    if (tid == 0) s_tile = atomicAdd(tile_ctr, 1u);
    for (int i = tid; i < WAVES * kRadix; i += BLOCK) s_wofs[i] = 0;
    __syncthreads();
    const uint32_t tile = s_tile;
    const uint64_t tbase = (uint64_t)tile * TILE;
    const bool full = tbase + TILE <= n;
    GSORT_STAMP(0);

    uint32_t k[ITEMS];
    {
        const uint32_t *src = in + tbase + (uint64_t)w * 64 * ITEMS + lane;
        if (full) {
#pragma unroll
            for (int i = 0; i < ITEMS; ++i) k[i] = FIN ? (src[i * 64] ^ kFlip) : src[i * 64];
        } else {
            const uint64_t lim = n - tbase;  // valid keys in this tile
            const uint64_t o = (uint64_t)w * 64 * ITEMS + lane;
#pragma unroll
            for (int i = 0; i < ITEMS; ++i) {
                // sentinels sort after every valid key of digit 255 (they are last in order)
                k[i] = (o + i * 64 < lim) ? (FIN ? (src[i * 64] ^ kFlip) : src[i * 64])
                                          : 0xFFFFFFFFu;
            }
        }
    }

    // 1. wave-level stable ranking
    uint32_t rk[(ITEMS + 1) / 2];  // two 16-bit ranks per register
    uint32_t *wc = s_wofs + w * kRadix;
#pragma unroll
    for (int i = 0; i < ITEMS; ++i) {
        const uint32_t d = (k[i] >> shift) & 255u;
        uint32_t plo = ~0u, phi = ~0u;
#pragma unroll
        for (int b = 0; b < 8; ++b) {
            // 4 VALU per bit: m = sign-extended bit (v_bfe_i32), ballot of m (v_cmp, asm so
            // hipcc does not re-derive the bit), peers &= ~(ballot ^ m) (v_bitop3 0x90)
            const uint32_t m = (uint32_t)__builtin_amdgcn_sbfe((int32_t)d, b, 1);
            uint64_t bal;
            asm("v_cmp_ne_u32_e64 %0, 0, %1" : "=s"(bal) : "v"(m));
            plo = __builtin_amdgcn_bitop3_b32(plo, (uint32_t)bal, m, 0x90);
            phi = __builtin_amdgcn_bitop3_b32(phi, (uint32_t)(bal >> 32), m, 0x90);
        }
        const uint32_t below =
            __builtin_amdgcn_mbcnt_hi(phi, __builtin_amdgcn_mbcnt_lo(plo, 0u));
        const uint32_t prev = wc[d];
        const uint32_t r = prev + below;
        wc[d] = prev + (uint32_t)(__popc(plo) + __popc(phi));  // same value from every peer
        if (i & 1) rk[i >> 1] |= r << 16; else rk[i >> 1] = r;
    }
    __syncthreads();
    GSORT_STAMP(1);

    // 2. per-digit tile counts; publish the aggregate; (early) lookback; digit starts
    uint32_t tcount = 0, excl = 0, lb_rounds = 0, lb_spins = 0;
    uint64_t prefix = 0;
    uint32_t c[WAVES];
    if (tid < kRadix) {
#pragma unroll
        for (int ww = 0; ww < WAVES; ++ww) {
            c[ww] = s_wofs[ww * kRadix + tid];
            tcount += c[ww];
        }
        st_agent(status + (uint64_t)tile * kRadix + tid,
                 pack_status(epoch, tile == 0 ? kFlagInc : kFlagAgg, tcount));
        if (LB_EARLY && tile > 0 && !NO_LOOKBACK) {
            prefix = lookback<LB_W>(status, tile, tid, epoch, err, lb_rounds, lb_spins);
            st_agent(status + (uint64_t)tile * kRadix + tid,
                     pack_status(epoch, kFlagInc, prefix + tcount));
        }
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
    uint32_t start = 0;
    if (tid < kRadix) {
        start = excl;
        for (int ww = 0; ww < w; ++ww) start += s_wsum[ww];
        uint32_t off = start;
#pragma unroll
        for (int ww = 0; ww < WAVES; ++ww) {
            s_wofs[ww * kRadix + tid] = off;
            off += c[ww];
        }
    }
    __syncthreads();

    // 3a. stable scatter into LDS (block-sorted order)
#pragma unroll
    for (int i = 0; i < ITEMS; ++i) {
        const uint32_t d = (k[i] >> shift) & 255u;
        const uint32_t r = (i & 1) ? (rk[i >> 1] >> 16) : (rk[i >> 1] & 0xFFFFu);
        s_keys[wc[d] + r] = k[i];
    }
    // 3b. (late) lookback, one thread per digit; global destination base per digit
    if (tid < kRadix) {
        if (!LB_EARLY && tile > 0 && !NO_LOOKBACK) {
            prefix = lookback<LB_W>(status, tile, tid, epoch, err, lb_rounds, lb_spins);
            st_agent(status + (uint64_t)tile * kRadix + tid,
                     pack_status(epoch, kFlagInc, prefix + tcount));
        }
        s_dst[tid] = out + (base[tid] + prefix) - start;
    }
    __syncthreads();
    GSORT_STAMP(2);
#ifdef GSORT_KBENCH_STAMPS
    if (tid == 0) {
        g_stamps[(uint64_t)tile * 8 + 4] = lb_rounds;
        g_stamps[(uint64_t)tile * 8 + 5] = lb_spins;
        uint32_t hw;
        asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(hw));
        g_stamps[(uint64_t)tile * 8 + 6] = hw & 0xF;
    }
#endif

    // 4. ordered write-out
    const uint32_t lim = full ? (uint32_t)TILE : (uint32_t)(n - tbase);
#pragma unroll
    for (int i = 0; i < ITEMS; ++i) {
        const uint32_t j = (uint32_t)(i * BLOCK + tid);
        if (full || j < lim) {
            const uint32_t key = s_keys[j];
            s_dst[(key >> shift) & 255u][j] = FOUT ? (key ^ kFlip) : key;
        }
    }
    GSORT_STAMP(3);
}

// ---------------------------------------------------------------------------------------
// K8: receive-side placement of a distributed pass.  segs[3*i] = {src_off, dst_off, len},
// sorted by src_off and covering the receive buffer.  Each block copies one contiguous tile
// of the receive buffer and, if asked, histograms the NEXT pass's digit of what it placed
// (so the next pass needs no separate histogram read).
// ---------------------------------------------------------------------------------------
template <int BLOCK, int ITEMS>
__global__ __launch_bounds__(BLOCK) void k_place(const uint32_t *__restrict__ recv,
                                                 uint32_t *__restrict__ out,
                                                 const unsigned long long *__restrict__ segs,
                                                 int nseg, uint64_t n,
                                                 unsigned long long *__restrict__ hist,
                                                 int next_shift, uint32_t out_xor) {
    constexpr int TILE = BLOCK * ITEMS;
    __shared__ uint32_t sh[kRadix];
    __shared__ int s_first;
    const uint64_t a = (uint64_t)blockIdx.x * TILE;
    const uint64_t e = a + TILE < n ? a + TILE : n;
    if (hist)
        for (int i = threadIdx.x; i < kRadix; i += BLOCK) sh[i] = 0;
    if (threadIdx.x == 0) {
        int lo = 0, hi = nseg;  // last segment with src_off <= a
        while (hi - lo > 1) {
            const int mid = (lo + hi) / 2;
            if (segs[3 * mid] <= a) lo = mid; else hi = mid;
        }
        s_first = lo;
    }
    __syncthreads();
    for (int s = s_first; s < nseg; ++s) {
        const uint64_t so = segs[3 * s], dofs = segs[3 * s + 1], len = segs[3 * s + 2];
        if (so >= e) break;
        const uint64_t x = so > a ? so : a;
        const uint64_t y = so + len < e ? so + len : e;
        for (uint64_t p = x + threadIdx.x; p < y; p += BLOCK) {
            const uint32_t key = recv[p];
            out[dofs + (p - so)] = key ^ out_xor;
            if (hist) atomicAdd(&sh[(key >> next_shift) & 255u], 1u);
        }
    }
    if (hist) {
        __syncthreads();
        for (int i = threadIdx.x; i < kRadix; i += BLOCK)
            if (sh[i]) atomicAdd(&hist[i], (unsigned long long)sh[i]);
    }
}

// ---------------------------------------------------------------------------------------
// K9: fingerprint (sum / xor of mix64(u32 key)) and descent count.
// ---------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_fingerprint(const int32_t *__restrict__ a, uint64_t n,
                                                     unsigned long long *acc) {
    __shared__ unsigned long long s_sum[4], s_xor[4], s_desc[4];
    uint64_t sum = 0, xr = 0, desc = 0;
    const uint64_t stride = (uint64_t)gridDim.x * 256;
    for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += stride) {
        const int32_t v = a[i];
        const uint64_t m = mix64((uint64_t)(uint32_t)v);
        sum += m;
        xr ^= m;
        if (i > 0 && a[i - 1] > v) ++desc;
    }
    for (int o = 32; o > 0; o >>= 1) {
        sum += __shfl_down(sum, o);
        xr ^= __shfl_down(xr, o);
        desc += __shfl_down(desc, o);
    }
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    if (lane == 0) { s_sum[w] = sum; s_xor[w] = xr; s_desc[w] = desc; }
    __syncthreads();
    if (threadIdx.x == 0) {
        for (int i = 1; i < 4; ++i) { sum += s_sum[i]; xr ^= s_xor[i]; desc += s_desc[i]; }
        atomicAdd(&acc[0], (unsigned long long)sum);
        atomicXor(&acc[1], (unsigned long long)xr);
        atomicAdd(&acc[2], (unsigned long long)desc);
    }
}

// K4: regular samples of a sorted block.
__global__ void k_regular_sample(const int32_t *sorted, uint64_t interval, int k, int32_t *out) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < k) out[i] = sorted[(uint64_t)i * interval];
}

// K5: rank-sort m <= 1024 samples in LDS (stable: ties broken by position), pick splitters.
__global__ __launch_bounds__(1024) void k_select_splitters(const int32_t *samples, int m, int k,
                                                           int nsplit, int32_t *splitters) {
    __shared__ int32_t s_in[1024], s_sorted[1024];
    const int i = threadIdx.x;
    if (i < m) s_in[i] = samples[i];
    __syncthreads();
    if (i < m) {
        const int32_t v = s_in[i];
        int rank = 0;
        for (int j = 0; j < m; ++j) {
            const int32_t u = s_in[j];
            rank += (u < v) || (u == v && j < i);
        }
        s_sorted[rank] = v;
    }
    __syncthreads();
    if (i < nsplit) splitters[i] = s_sorted[(i + 1) * k];
}

// K6: bucket bounds on a sorted block, one wave per splitter: 64-way search steps narrow the
// range 64x per dependent load, then one sweep of <= 64 keys.  bounds[j] = #keys <= s[j].
__global__ __launch_bounds__(64) void k_bucket_bounds(const int32_t *__restrict__ a, uint64_t n,
                                                      const int32_t *__restrict__ spl,
                                                      unsigned long long *bounds) {
    const int j = blockIdx.x;
    const int lane = threadIdx.x;
    const int32_t s = spl[j];
    uint64_t lo = 0, hi = n;  // answer (first index with a[i] > s) lies in [lo, hi]
    while (hi - lo > 64) {
        const uint64_t step = (hi - lo) / 64;
        const uint64_t pos = lo + (uint64_t)lane * step;
        const uint64_t m = __ballot(a[pos] <= s);
        const int c = __popcll(m);  // sorted: the true lanes are a prefix
        if (c == 0) { hi = lo; break; }
        const uint64_t nlo = lo + (uint64_t)(c - 1) * step + 1;
        if (c < 64) hi = lo + (uint64_t)c * step;
        lo = nlo;
    }
    const uint64_t pos = lo + lane;
    const uint64_t m = __ballot(pos < hi && a[pos] <= s);
    if (lane == 0) bounds[j] = lo + (uint64_t)__popcll(m);
}

__global__ void k_copy(const uint32_t *__restrict__ in, uint32_t *__restrict__ out, uint64_t n) {
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride)
        out[i] = in[i];
}

unsigned grid_for(uint64_t n, unsigned block, unsigned cap) {
    uint64_t g = (n + block - 1) / block;
    if (g < 1) g = 1;
    return (unsigned)(g < cap ? g : cap);
}

}  // namespace

hipError_t launch_generate(int dist, uint64_t seed, uint64_t start, uint64_t n, int32_t *out,
                           hipStream_t s) {
    if (n == 0) return hipSuccess;
    k_generate<<<grid_for(n, 256, 4096), 256, 0, s>>>(dist, seed, start, n, out);
    return hipGetLastError();
}

hipError_t launch_hist4(const uint32_t *in, uint64_t n, uint64_t *hist, hipStream_t s) {
    if (n == 0) return hipSuccess;
    constexpr int B = 512;
    const unsigned g = grid_for(n / 16 + 1, B, 1024);
    auto *h = reinterpret_cast<unsigned long long *>(hist);
    if ((reinterpret_cast<uintptr_t>(in) & 15) == 0)
        k_hist4<B, true><<<g, B, 0, s>>>(in, n, h);
    else
        k_hist4<B, false><<<g, B, 0, s>>>(in, n, h);
    return hipGetLastError();
}

hipError_t launch_onesweep(const uint32_t *in, uint32_t *out, uint64_t n, int shift,
                           const uint64_t *base, uint64_t *status, uint32_t *tile_ctr,
                           uint32_t *err, uint32_t epoch, bool flip_in, bool flip_out,
                           hipStream_t s) {
    if (n == 0) return hipSuccess;
    const unsigned g = (unsigned)sweep_tiles(n);
    auto *b = reinterpret_cast<const unsigned long long *>(base);
    auto *st = reinterpret_cast<unsigned long long *>(status);
    constexpr int B = kSweepBlock, I = kSweepItems;
    if (flip_in && flip_out)
        k_onesweep<B, I, true, true><<<g, B, 0, s>>>(in, out, n, shift, b, st, tile_ctr, err, epoch);
    else if (flip_in)
        k_onesweep<B, I, true, false><<<g, B, 0, s>>>(in, out, n, shift, b, st, tile_ctr, err, epoch);
    else if (flip_out)
        k_onesweep<B, I, false, true><<<g, B, 0, s>>>(in, out, n, shift, b, st, tile_ctr, err, epoch);
    else
        k_onesweep<B, I, false, false><<<g, B, 0, s>>>(in, out, n, shift, b, st, tile_ctr, err, epoch);
    return hipGetLastError();
}

hipError_t launch_place(const uint32_t *recv, uint32_t *out, const uint64_t *segs, int nseg,
                        uint64_t n_out, uint64_t *hist, int next_shift, bool flip_out,
                        hipStream_t s) {
    if (n_out == 0 || nseg == 0) return hipSuccess;
    constexpr int B = 256, I = 16;
    const unsigned g = (unsigned)((n_out + B * I - 1) / (B * I));
    k_place<B, I><<<g, B, 0, s>>>(recv, out, reinterpret_cast<const unsigned long long *>(segs),
                                  nseg, n_out, reinterpret_cast<unsigned long long *>(hist),
                                  next_shift, flip_out ? kFlip : 0u);
    return hipGetLastError();
}

hipError_t launch_fingerprint(const int32_t *keys, uint64_t n, unsigned long long *acc,
                              hipStream_t s) {
    if (n == 0) return hipSuccess;
    k_fingerprint<<<grid_for(n, 256, 2048), 256, 0, s>>>(keys, n, acc);
    return hipGetLastError();
}

hipError_t launch_regular_sample(const int32_t *sorted, uint64_t interval, int k, int32_t *out,
                                 hipStream_t s) {
    k_regular_sample<<<1, 64 * ((k + 63) / 64), 0, s>>>(sorted, interval, k, out);
    return hipGetLastError();
}

hipError_t launch_select_splitters(const int32_t *samples, int m, int k, int nsplit,
                                   int32_t *splitters, hipStream_t s) {
    if (m > 1024 || nsplit <= 0) return nsplit <= 0 ? hipSuccess : hipErrorInvalidValue;
    k_select_splitters<<<1, 1024, 0, s>>>(samples, m, k, nsplit, splitters);
    return hipGetLastError();
}

hipError_t launch_bucket_bounds(const int32_t *sorted, uint64_t n, const int32_t *splitters,
                                int nsplit, uint64_t *bounds, hipStream_t s) {
    if (nsplit <= 0) return hipSuccess;
    k_bucket_bounds<<<nsplit, 64, 0, s>>>(sorted, n, splitters,
                                          reinterpret_cast<unsigned long long *>(bounds));
    return hipGetLastError();
}

hipError_t launch_copy(const uint32_t *in, uint32_t *out, uint64_t n, hipStream_t s) {
    if (n == 0) return hipSuccess;
    k_copy<<<grid_for(n, 256, 8192), 256, 0, s>>>(in, out, n);
    return hipGetLastError();
}

}  // namespace gsort
