// gsort_kernels.hip -- hand-written CDNA4 (gfx950) kernels of the distributed sorter.
//
// Keys are int32; every kernel that compares digits works on the order-preserving map
// u = key ^ 0x80000000 (unsigned order of u == signed order of key).  The local sort is an
// 8-bit LSD radix sort; each pass counts digits per tile (K1; the first pass also builds all
// four global digit histograms), scans the tile offsets (K2), then ranks every tile with
// wave64 ballots and scatters it through LDS so the global stores come out in digit runs
// (K3).  Algorithmic traffic: 4 B/key (K1) + 8 B/key (K3) per pass.
//
// Reference hot loops these replace (cites /root/reference/...):
//   K1/K3  mpi_radix_sort.c:144-147 (number_digit_at + bucket_push per key), :54-58, :33-43;
//          and the local qsort of mpi_sample_sort.c:85 and :174
//   K4     mpi_sample_sort.c:89-105 regular sampling
//   K5     mpi_sample_sort.c:109-125 sort samples at the root, pick splitters
//   K6     mpi_sample_sort.c:148-155 bucket partition (here: bounds on the sorted block)
//   K8     mpi_radix_sort.c:164-192 per-pass placement (receive side of the exchange)
#include <hip/hip_ext.h>

#include <algorithm>

#include "gsort_kernels.h"

namespace gsort {
namespace {

constexpr uint32_t kFlip = 0x80000000u;

constexpr uint64_t kGolden = 0x9E3779B97F4A7C15ULL;

__device__ __forceinline__ uint64_t mix64(uint64_t z) {
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
    return z ^ (z >> 31);
}

// Wave-wide inclusive scans through DPP (row shifts 1/2/4/8, then the row-15 and row-31
// broadcasts): VALU only, where __shfl_up costs an LDS-crossbar op per step.
template <int CTRL, int ROWS = 0xf>
__device__ __forceinline__ uint32_t dpp0(uint32_t x) {  // lanes outside the pattern read 0
    return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, CTRL, ROWS, 0xf, true);
}
__device__ __forceinline__ uint32_t wave_incl_add(uint32_t x) {
    x += dpp0<0x111>(x);
    x += dpp0<0x112>(x);
    x += dpp0<0x114>(x);
    x += dpp0<0x118>(x);
    x += dpp0<0x142, 0xa>(x);
    x += dpp0<0x143, 0xc>(x);
    return x;
}
__device__ __forceinline__ uint32_t wave_incl_max(uint32_t x) {
    x = max(x, dpp0<0x111>(x));
    x = max(x, dpp0<0x112>(x));
    x = max(x, dpp0<0x114>(x));
    x = max(x, dpp0<0x118>(x));
    x = max(x, dpp0<0x142, 0xa>(x));
    x = max(x, dpp0<0x143, 0xc>(x));
    return x;
}

// ---------------------------------------------------------------------------------------
// Duplicate-aggregated LDS counter atomics.  Skewed inputs (sorted runs, many equal keys, the
// top digits of a Zipf stream) send most lanes of a wave to ONE counter, and same-address LDS
// atomics serialize lane by lane (an all-equal 2^28-key sort ran 4.5x slower than a uniform
// one, tools/dist_probe.py).  So the lanes whose counter equals the first active lane's add
// their total with one atomic from that lane (the others of them add 0 to their own spare
// word), and every lane gets back the value it would have seen had the adds been serialized in
// lane order -- which is the order the hardware serializes same-address lanes in, so the
// stable per-wave ranks of K11 stay stable.  Other lanes add as before.
// spare: 64 words, one per lane (distinct banks).
// ---------------------------------------------------------------------------------------
constexpr int kAggSpare = 64;

__device__ __forceinline__ uint32_t lane_rank(uint64_t m) {  // set bits of m below this lane
    return __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
}

// Rank on ctr[idx] (+1 per lane); returns the lane's rank among the adds to ctr[idx].
__device__ __forceinline__ uint32_t agg_rank(uint32_t *ctr, uint32_t idx, uint32_t *spare) {
    const uint32_t idx0 = __builtin_amdgcn_readfirstlane(idx);
    const bool eq = idx == idx0;
    const uint64_t m = __ballot(eq);
    const uint32_t lr = lane_rank(m);
    uint32_t *a = !eq ? ctr + idx : lr == 0 ? ctr + idx0 : spare + (threadIdx.x & 63);
    const uint32_t v = !eq ? 1u : lr == 0 ? (uint32_t)__popcll(m) : 0u;
    const uint32_t old = atomicAdd(a, v);
    return eq ? __builtin_amdgcn_readfirstlane(old) + lr : old;
}

// K1h's packed pair counters: word w = b >> 1 gains 1 << (16 * (b & 1)) per lane.  The lanes on
// the first active lane's WORD (either half) add their sum with one atomic; each gets the word
// value of the lane-order serialization (so the wrap test and repair see a consistent order).
__device__ __forceinline__ uint32_t agg_add_pair(uint32_t *words, uint32_t b, uint32_t *spare) {
    const uint32_t w = b >> 1, w0 = __builtin_amdgcn_readfirstlane(w);
    const bool eq = w == w0;
    const uint64_t m = __ballot(eq), mhi = __ballot(eq && (b & 1u));
    const uint64_t mlo = m & ~mhi;
    const uint32_t lr = lane_rank(m);
    const uint32_t inc = 1u << ((b & 1u) << 4);
    uint32_t *a = !eq ? words + w : lr == 0 ? words + w0 : spare + (threadIdx.x & 63);
    const uint32_t v = !eq ? inc
                     : lr == 0 ? (uint32_t)__popcll(mlo) + ((uint32_t)__popcll(mhi) << 16) : 0u;
    const uint32_t old = atomicAdd(a, v);
    return eq ? __builtin_amdgcn_readfirstlane(old) + lane_rank(mlo) + (lane_rank(mhi) << 16)
              : old;
}

// agg_add_pair on a given word w0 (wave-uniform): the lanes on w0 add their sum with one atomic
// from the first of them, every other lane adds its own increment.
__device__ __forceinline__ uint32_t agg_add_pair_at(uint32_t *words, uint32_t b, uint32_t w0,
                                                    uint32_t *spare, bool valid = true) {
    // (valid false: the lane adds 0 -- every lane issues its atomic, no divergent branch)
    const uint32_t w = b >> 1;
    const bool eq = valid && w == w0;
    const uint64_t m = __ballot(eq), mhi = __ballot(eq && (b & 1u));
    const uint64_t mlo = m & ~mhi;
    const uint32_t lr = lane_rank(m);
    const uint32_t inc = valid ? 1u << ((b & 1u) << 4) : 0u;
    uint32_t *a = !eq ? words + w : lr == 0 ? words + w0 : spare + (threadIdx.x & 63);
    const uint32_t v = !eq ? inc
                     : lr == 0 ? (uint32_t)__popcll(mlo) + ((uint32_t)__popcll(mhi) << 16) : 0u;
    const uint32_t old = atomicAdd(a, v);
    const uint32_t o0 = m ? (uint32_t)__builtin_amdgcn_readlane((int)old, (int)__builtin_ctzll(m)) : 0u;
    return eq ? o0 + lane_rank(mlo) + (lane_rank(mhi) << 16) : old;
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
// One LSD pass = K1 (per-tile digit counts) + K2 (two-level scan of the tile offsets) + K3
// (rank + stable scatter).  A single-pass "onesweep" with a decoupled lookback was measured
// first: on MI355X a cross-XCD status round trip costs ~1.35 us under streaming
// load, so at the tile rate an HBM-bound pass needs (~90 tiles/us) every tile walked ~40
// predecessors and read more status bytes than key bytes.  Counting first costs 4 B/key more
// per pass but makes K3 free of inter-workgroup communication.
// ---------------------------------------------------------------------------------------

// K1: digit counts of every kSweepTile-key tile (tcounts[tile][256], u32).  ALL4 (first pass,
// digit 0) also accumulates the four global digit histograms (hist4[4][256]) in the same read;
// they decide which passes are trivial and, in the distributed sort, are all-gathered.
template <int BLOCK, bool ALL4, bool VEC>
__global__ __launch_bounds__(BLOCK) void k_tile_counts(const uint32_t *__restrict__ in,
                                                       uint64_t n, int shift, uint32_t flip,
                                                       uint32_t *__restrict__ tcounts,
                                                       unsigned long long *__restrict__ hist4,
                                                       uint32_t ntiles) {
    constexpr int WAVES = BLOCK / 64;
    __shared__ uint32_t s_t[kRadix];
    __shared__ uint32_t s_h[ALL4 ? WAVES * 3 * kRadix : 1];  // digits 1..3, per wave
    const int tid = threadIdx.x;
    uint32_t *hw = s_h + (ALL4 ? (tid >> 6) * 3 * kRadix : 0);
    if (ALL4)
        for (int i = tid; i < WAVES * 3 * kRadix; i += BLOCK) s_h[i] = 0;
    uint64_t acc0 = 0;  // ALL4: this thread's digit of hist4[0] (= sum of its tile counts)
    auto count = [&](uint32_t u) {
        u ^= flip;
        atomicAdd(&s_t[(u >> shift) & 255u], 1u);
        if (ALL4) {
            atomicAdd(&hw[(u >> 8) & 255u], 1u);
            atomicAdd(&hw[kRadix + ((u >> 16) & 255u)], 1u);
            atomicAdd(&hw[2 * kRadix + (u >> 24)], 1u);
        }
    };
    for (uint32_t tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
        if (tid < kRadix) s_t[tid] = 0;
        __syncthreads();
        const uint64_t t0 = (uint64_t)tile * kSweepTile;
        if (VEC && t0 + kSweepTile <= n) {
            const uint4 *p = reinterpret_cast<const uint4 *>(in + t0);
#pragma unroll
            for (int j = 0; j < kSweepTile / 4 / BLOCK; ++j) {
                const uint4 q = p[j * BLOCK + tid];
                count(q.x); count(q.y); count(q.z); count(q.w);
            }
        } else {
            const uint64_t t1 = t0 + kSweepTile < n ? t0 + kSweepTile : n;
            for (uint64_t i = t0 + tid; i < t1; i += BLOCK) count(in[i]);
        }
        __syncthreads();
        if (tid < kRadix) {
            tcounts[(uint64_t)tile * kRadix + tid] = s_t[tid];
            acc0 += s_t[tid];
        }
    }
    if (ALL4) {
        __syncthreads();
        if (tid < kRadix && acc0) atomicAdd(&hist4[tid], (unsigned long long)acc0);
        for (int b = tid; b < 3 * kRadix; b += BLOCK) {
            uint32_t s = 0;
#pragma unroll
            for (int w = 0; w < WAVES; ++w) s += s_h[w * 3 * kRadix + b];
            if (s) atomicAdd(&hist4[kRadix + b], (unsigned long long)s);
        }
    }
}

// K2a: group-local exclusive scan over the kScanGroup tiles of group g, one thread per digit
// (all 32 loads of a thread in flight at once): tcounts[t][d] becomes the offset of tile t's
// digit-d keys inside its group; gsum[g][d] = the group's total.
__global__ __launch_bounds__(kRadix) void k_scan_tiles(uint32_t *__restrict__ tcounts,
                                                       uint32_t ntiles,
                                                       unsigned long long *__restrict__ gsum) {
    const uint32_t g = blockIdx.x, d = threadIdx.x;
    const uint32_t t0 = g * kScanGroup;
    uint32_t c[kScanGroup];
#pragma unroll
    for (int j = 0; j < kScanGroup; ++j)
        c[j] = t0 + j < ntiles ? tcounts[(uint64_t)(t0 + j) * kRadix + d] : 0u;
    uint32_t run = 0;
#pragma unroll
    for (int j = 0; j < kScanGroup; ++j) {
        if (t0 + j < ntiles) tcounts[(uint64_t)(t0 + j) * kRadix + d] = run;
        run += c[j];
    }
    gsum[(uint64_t)g * kRadix + d] = run;
}

// K2b: one workgroup per digit: exclusive scan of gsum[.][d] over the groups (in place) and
// totals[d] = the pass's count of digit d.
__global__ __launch_bounds__(1024) void k_scan_groups(unsigned long long *__restrict__ gsum,
                                                      uint32_t ngroups,
                                                      unsigned long long *__restrict__ totals) {
    __shared__ unsigned long long s_w[16];
    const uint32_t d = blockIdx.x, tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const uint32_t per = (ngroups + 1023) / 1024;
    const uint32_t g0 = tid * per;
    unsigned long long sum = 0;
    for (uint32_t j = 0; j < per; ++j)
        if (g0 + j < ngroups) sum += gsum[(uint64_t)(g0 + j) * kRadix + d];
    unsigned long long v = sum;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const unsigned long long t = __shfl_up(v, o);
        if (lane >= o) v += t;
    }
    if (lane == 63) s_w[w] = v;
    __syncthreads();
    unsigned long long run = v - sum;
    for (uint32_t ww = 0; ww < w; ++ww) run += s_w[ww];
    if (tid == 1023) {
        unsigned long long tot = 0;
        for (int ww = 0; ww < 16; ++ww) tot += s_w[ww];
        totals[d] = tot;
    }
    for (uint32_t j = 0; j < per; ++j)
        if (g0 + j < ngroups) {
            const unsigned long long c = gsum[(uint64_t)(g0 + j) * kRadix + d];
            gsum[(uint64_t)(g0 + j) * kRadix + d] = run;
            run += c;
        }
}

// K2c: bases[d] = exclusive scan of the digit totals (where digit d starts in the output).
__global__ __launch_bounds__(kRadix) void k_scan_digits(const unsigned long long *__restrict__ totals,
                                                        unsigned long long *__restrict__ bases) {
    __shared__ unsigned long long s_w[kRadix / 64];
    const int d = threadIdx.x, lane = d & 63, w = d >> 6;
    const unsigned long long tot = totals[d];
    unsigned long long v = tot;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const unsigned long long t = __shfl_up(v, o);
        if (lane >= o) v += t;
    }
    if (lane == 63) s_w[w] = v;
    __syncthreads();
    unsigned long long run = v - tot;
    for (int ww = 0; ww < w; ++ww) run += s_w[ww];
    bases[d] = run;
}

// XCD-aware tile order: workgroups are dealt round-robin over the 8 XCDs (MI355X_MICROARCH.md,
// dispatch), so workgroup b runs on XCD b % 8.  Giving each XCD a contiguous range of tiles
// keeps the partial 128-B lines shared by neighbouring tiles' digit runs in one L2, where they
// merge before write-back.  Bijective for any tile count; speed only, never correctness.
// Items of a packed register array: item i in the low (even i) or high (odd i) half of word i/2
// (values below 2^16: ranks, positions and keys of a tile whose keys share their top half).
template <int BLOCK, int ITEMS>
struct Pack16 {  // item i of a packed register array
    static constexpr int NP = (ITEMS + 1) / 2;
    __device__ static uint32_t get(const uint32_t (&a)[NP], int i) {
        return (i & 1) ? a[i >> 1] >> 16 : a[i >> 1] & 0xFFFFu;
    }
    // the packed words as opaque values: without this the compiler keeps every key (rank)
    // unpacked until its last use and packs late -- 33 live registers instead of 17
    __device__ static void pin(uint32_t (&a)[NP]) {
#pragma unroll
        for (int q = 0; q < NP; ++q) asm volatile("" : "+v"(a[q]));
    }
    __device__ static void set(uint32_t (&a)[NP], int i, uint32_t v) {
        a[i >> 1] = (i & 1) ? __builtin_amdgcn_perm(v, a[i >> 1], 0x05040100u)   // v.lo : a.lo
                            : __builtin_amdgcn_perm(a[i >> 1], v, 0x07060100u);  // a.hi : v.lo
    }
};

// A store through a pointer kept in LDS (a digit's output run) as a global, not flat, access:
// flat stores also count against the LDS wait counter, so every later LDS wait waited on them
template <typename T>
__device__ __forceinline__ void st_global(T *p, T v) {
    *reinterpret_cast<__attribute__((address_space(1))) T *>(reinterpret_cast<uintptr_t>(p)) = v;
}

__device__ __forceinline__ uint32_t xcd_tile(uint32_t b, uint32_t ntiles) {
    const uint32_t q = ntiles >> 3, r = ntiles & 7, x = b & 7, i = b >> 3;
    return x < r ? x * (q + 1) + i : r * (q + 1) + (x - r) * q + i;
}

// ---------------------------------------------------------------------------------------
// K3: rank + stable scatter of one tile (no inter-workgroup communication).
//   tile = BLOCK * ITEMS keys; wave w owns keys [w*64*ITEMS, (w+1)*64*ITEMS) of the tile,
//   round i of the wave holds keys i*64 + lane, so (round, lane) order == memory order.
//   1. rank: for each round, 8 ballots give each lane the mask of lanes sharing its digit
//      (per bit: v_bfe_i32, v_cmp, two v_bitop3); rank = (wave's running count of the digit)
//      + (#peers below the lane); every peer writes the same advanced count (branch-free).
//   2. block-exclusive digit starts + per-wave counts -> per-wave tile offsets.
//   3. scatter keys into LDS in block-sorted order (stable); the tile's global destination
//      per digit = digit base (K2c) + group prefix (K2b) + in-group tile offset (K2a), loaded
//      at kernel start.  Tiles are assigned to workgroups XCD-contiguously (xcd_tile).
//   4. stream LDS out in order: consecutive lanes hit consecutive addresses within a digit.
// ---------------------------------------------------------------------------------------
//   KV (the reference-compat sort, gsort_set_ref_compat): every key carries a 32-bit value
//   (vin -> vout), scattered through LDS beside it, so the pass is a stable key-value pass.
template <int BLOCK, int ITEMS, bool FIN, bool FOUT, bool KV = false>
__global__ __launch_bounds__(BLOCK) void k_scatter(const uint32_t *__restrict__ in,
                                                   uint32_t *__restrict__ out, uint64_t n,
                                                   int shift,
                                                   const uint32_t *__restrict__ toff,
                                                   const unsigned long long *__restrict__ gpfx,
                                                   const unsigned long long *__restrict__ bases,
                                                   const uint32_t *__restrict__ vin = nullptr,
                                                   uint32_t *__restrict__ vout = nullptr) {
    constexpr int WAVES = BLOCK / 64;
    constexpr int TILE = BLOCK * ITEMS;
    static_assert(TILE == kSweepTile, "K1/K2 count tiles of kSweepTile keys");
    static_assert(BLOCK >= kRadix, "one thread per digit in the scan");
    static_assert(TILE <= 65536, "ranks are packed as 16 bits");
    __shared__ uint32_t s_keys[TILE];
    __shared__ uint32_t s_vals[KV ? TILE : 1];
    __shared__ uint32_t s_wofs[WAVES * kRadix];  // per-wave counts, then per-wave tile offsets
    __shared__ uint32_t *s_dst[kRadix];          // out + global offset - tile start, by digit
    __shared__ uint32_t s_wsum[kRadix / 64];

    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int w = tid >> 6;
    const uint32_t tile = xcd_tile(blockIdx.x, gridDim.x);
    const uint64_t tbase = (uint64_t)tile * TILE;
    const bool full = tbase + TILE <= n;
    for (int i = tid; i < WAVES * kRadix; i += BLOCK) s_wofs[i] = 0;
    // this tile's global base per digit, fetched early (latency hidden behind the ranking)
    uint32_t *dst_base = nullptr;
    if (tid < kRadix)
        dst_base = out + bases[tid] + gpfx[(uint64_t)(tile / kScanGroup) * kRadix + tid] +
                   toff[(uint64_t)tile * kRadix + tid];

    uint32_t k[ITEMS];
    uint32_t v[KV ? ITEMS : 1];
    {
        const uint64_t o = (uint64_t)w * 64 * ITEMS + lane;
        const uint32_t *src = in + tbase + o;
        if (full) {
#pragma unroll
            for (int i = 0; i < ITEMS; ++i) k[i] = FIN ? (src[i * 64] ^ kFlip) : src[i * 64];
            if constexpr (KV) {
#pragma unroll
                for (int i = 0; i < ITEMS; ++i) v[i] = vin[tbase + o + i * 64];
            }
        } else {
            const uint64_t lim = n - tbase;  // valid keys in this tile
#pragma unroll
            for (int i = 0; i < ITEMS; ++i) {
                // sentinels sort after every valid key of digit 255 (they are last in order)
                k[i] = (o + i * 64 < lim) ? (FIN ? (src[i * 64] ^ kFlip) : src[i * 64])
                                          : 0xFFFFFFFFu;
            }
            if constexpr (KV) {
#pragma unroll
                for (int i = 0; i < ITEMS; ++i)
                    v[i] = (o + i * 64 < lim) ? vin[tbase + o + i * 64] : 0u;
            }
        }
    }
    __syncthreads();

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

    // 2. per-wave tile offsets = block-exclusive digit start + counts of earlier waves
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

    // 3. stable scatter into LDS (block-sorted order)
#pragma unroll
    for (int i = 0; i < ITEMS; ++i) {
        const uint32_t d = (k[i] >> shift) & 255u;
        const uint32_t r = (i & 1) ? (rk[i >> 1] >> 16) : (rk[i >> 1] & 0xFFFFu);
        s_keys[wc[d] + r] = k[i];
        if constexpr (KV) s_vals[wc[d] + r] = v[i];
    }
    __syncthreads();

    // 4. ordered write-out
    const uint32_t lim = full ? (uint32_t)TILE : (uint32_t)(n - tbase);
#pragma unroll
    for (int i = 0; i < ITEMS; ++i) {
        const uint32_t j = (uint32_t)(i * BLOCK + tid);
        if (full || j < lim) {
            const uint32_t key = s_keys[j];
            uint32_t *dst = s_dst[(key >> shift) & 255u] + j;
            st_global(dst, FOUT ? (key ^ kFlip) : key);
            if constexpr (KV) vout[dst - out] = s_vals[j];
        }
    }
}

// ---------------------------------------------------------------------------------------
// Reference-compat key map (gsort_set_ref_compat).  The reference
// radix sort orders keys by base-P digits of |v| (mpi_radix_sort.c:54-58), number_digits(max)
// of them (:48-52, :100), one stable pass per digit (:133-195): a stable sort of the values by
// the mixed-radix number of those digits, which is |v| mod P^loop for in-range moduli.
// K20 finds the min / max key (loop needs the max; INT_MIN has no |v|), K19 writes that
// composite key for every value; the stable key-value LSD passes (k_scatter<.., KV>) then sort
// the values by it.
// ---------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_minmax(const int32_t *__restrict__ a, uint64_t n,
                                                int *__restrict__ mm) {
    int lo = 2147483647, hi = -2147483647 - 1;
    const uint64_t stride = (uint64_t)gridDim.x * 256;
    for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += stride) {
        const int v = a[i];
        lo = min(lo, v);
        hi = max(hi, v);
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        lo = min(lo, __shfl_xor(lo, o));
        hi = max(hi, __shfl_xor(hi, o));
    }
    if ((threadIdx.x & 63) == 0) {
        atomicMin(&mm[0], lo);
        atomicMax(&mm[1], hi);
    }
}

// K19: key[i] = sum over d = 1..loop of digit_d(|v|) * P^(d-1), digit_d = x86_dtoi(rem / scale[d])
// with rem = |v| % mod[d] (mod[d] = x86_dtoi(P^d), the reference's (int)pow; 0 or -1: 0).
// bad[0] counts keys whose digit falls outside [0, P) or whose key does not fit 32 bits (the
// reference indexes outside its buckets there).  The caller rejects INT_MIN beforehand.
constexpr int kCompatMaxDigits = 64;
struct CompatDigits {
    int P, loop;
    int mod[kCompatMaxDigits];
    double scale[kCompatMaxDigits];
    unsigned long long weight[kCompatMaxDigits];  // P^(d-1), saturated
};

__device__ __forceinline__ int x86_dtoi(double x) {
    return (x > -2147483649.0 && x < 2147483648.0) ? (int)x : (-2147483647 - 1);
}

__global__ __launch_bounds__(256) void k_compat_keys(const int32_t *__restrict__ a, uint64_t n,
                                                     CompatDigits cd, uint32_t *__restrict__ key,
                                                     unsigned long long *__restrict__ bad) {
    const uint64_t stride = (uint64_t)gridDim.x * 256;
    uint32_t nbad = 0;
    for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += stride) {
        const int v = a[i];
        const int mag = v < 0 ? -v : v;
        unsigned long long k = 0;
        bool ok = mag >= 0;
        for (int d = 0; d < cd.loop; ++d) {
            const int m = cd.mod[d];
            const int rem = (m == 0 || m == -1) ? 0 : mag % m;
            const int dig = x86_dtoi(__ddiv_rn((double)rem, cd.scale[d]));
            ok &= dig >= 0 && dig < cd.P;
            if (dig > 0) k += (unsigned long long)dig * cd.weight[d];
        }
        ok &= k < (1ull << 32);
        key[i] = (uint32_t)k;
        nbad += !ok;
    }
    if (nbad) atomicAdd(bad, (unsigned long long)nbad);
}

// ---------------------------------------------------------------------------------------
// K12p: publish n u64 counters to pinned host memory, then seq to *flag with a system-scope
// release, so the host reads the MSD work-list counters by polling (no copy, no event on the
// stream).  One workgroup of 64 threads.
// ---------------------------------------------------------------------------------------
__global__ __launch_bounds__(64) void k_publish(const unsigned long long *__restrict__ src,
                                                uint32_t n, unsigned long long *dst,
                                                unsigned long long *flag,
                                                unsigned long long seq) {
    for (uint32_t i = threadIdx.x; i < n; i += 64) dst[i] = src[i];
    __threadfence_system();
    __syncthreads();
    if (threadIdx.x == 0)
        __hip_atomic_store(flag, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
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

// K13: out[i] = #keys of the sorted int32 block `a` whose ordered u32 form is < xs[i] (u64:
// 2^32 counts every key).  One thread per threshold, binary search.  Radix select of the exact
// global splitters of the distributed radix sort (gsort_runtime.cpp, radix_dist).
__global__ __launch_bounds__(256) void k_count_below(const int32_t *__restrict__ a, uint64_t n,
                                                     const unsigned long long *__restrict__ xs,
                                                     int m, unsigned long long *__restrict__ out) {
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i >= m) return;
    const uint64_t x = xs[i];
    uint64_t lo = 0, hi = n;
    while (lo < hi) {
        const uint64_t mid = (lo + hi) >> 1;
        if ((uint64_t)((uint32_t)a[mid] ^ kFlip) < x) lo = mid + 1; else hi = mid;
    }
    out[i] = lo;
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
                                                      unsigned long long *bounds, int strict) {
    // strict: count keys < s (lower bound) as keys <= s - 1; s = INT_MIN has none
    const int j = blockIdx.x;
    const int lane = threadIdx.x;
    if (strict && spl[j] == (int32_t)0x80000000) {
        if (lane == 0) bounds[j] = 0;
        return;
    }
    const int32_t s = strict ? spl[j] - 1 : spl[j];
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

// Streaming copy ceiling (bench reference, not on the sort path): one 256-thread block per
// contiguous 16 KiB chunk, four 16-B loads in flight per lane, nontemporal stores.  The best of
// the variants measured in tools/experiments/copy_ceiling.hip (grid-strided loops, wider
// unrolls, 1024-thread blocks, nontemporal loads, hipMemcpyAsync): 5.76 TB/s over 1 GiB,
// 6.0 TB/s over 4 GiB (MI355X_MICROARCH.md quotes 6.29 TB/s for a float4 copy).
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
__global__ __launch_bounds__(256) void k_stream_copy(const u32x4 *__restrict__ in,
                                                     u32x4 *__restrict__ out, uint64_t n16) {
    constexpr int U = 4;
    const uint64_t base = (uint64_t)blockIdx.x * (U * 256);
    u32x4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
        const uint64_t j = base + u * 256 + threadIdx.x;
        if (j < n16) v[u] = in[j];
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
        const uint64_t j = base + u * 256 + threadIdx.x;
        if (j < n16) __builtin_nontemporal_store(v[u], out + j);
    }
}

__global__ void k_copy(const uint32_t *__restrict__ in, uint32_t *__restrict__ out, uint64_t n) {
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride)
        out[i] = in[i];
}

// =======================================================================================
// MSD partition sort (keys only).  A keys-only sort does not need stable partitions: an MSD
// pass only has to put every key into its digit's bucket, and the buckets are then sorted on
// the remaining digits.  So the partition passes rank keys with one LDS atomic each (no ballot
// matching), and buckets small enough for one workgroup (<= kLocalMax keys) are finished in
// LDS by K11 -- one HBM read + one write for all their remaining digits.
//   level 3: K1 + K2 (global tiles) + K3u  -> 256 buckets
//   level L<3: K12 plan/map, K1s, K2s-a, K2s-b, K3u over the oversized buckets of level L+1
//   K11: buckets <= kLocalMax keys, remaining digits sorted in LDS (first digit unstable by
//        LDS atomics, the others stable by wave64 ballot ranks), written back flipped to int32
// Segment descriptors are u64 pairs {start, len}.  Segment tile ranges are NOT padded: group
// G of segment s covers its tiles [32 (G - gpfx[s]), +32) counted from the segment's first.
// =======================================================================================

// Block-strided tile load: k[i] = src[i * BLOCK] (src already offset by threadIdx.x) for the
// first len keys of the tile, 0 beyond.  All loads are issued before any use: a per-key branch
// around a load AND its use (e.g. the int32 flip) makes the compiler wait on every load.
template <int BLOCK, int ITEMS, bool FIN>
__device__ __forceinline__ void load_tile(const uint32_t *__restrict__ src, bool full,
                                          uint32_t len, uint32_t (&k)[ITEMS]) {
    if (full) {
#pragma unroll
        for (int i = 0; i < ITEMS; ++i) k[i] = src[i * BLOCK];
    } else {
#pragma unroll
        for (int i = 0; i < ITEMS; ++i)
            k[i] = (uint32_t)(i * BLOCK + threadIdx.x) < len ? src[i * BLOCK] : 0u;
    }
    if (FIN) {
#pragma unroll
        for (int i = 0; i < ITEMS; ++i) k[i] ^= kFlip;
    }
}

// Buffer descriptor over n_bytes at p (wave-uniform p and n_bytes): loads past the end return
// 0 and stores past it are dropped, so partial buckets need no per-key bound.
__device__ __forceinline__ __amdgpu_buffer_rsrc_t bucket_rsrc(const void *p, uint32_t n_bytes) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void *>(p), 0, (int)n_bytes, 0x00020000);
}

// K11 bucket load: k[i] = src[i * BLOCK + threadIdx.x] below len, 0 past it.
template <int BLOCK, int ITEMS, bool FIN>
__device__ __forceinline__ void load_bucket(const uint32_t *src, uint32_t len,
                                            uint32_t (&k)[ITEMS]) {
    const __amdgpu_buffer_rsrc_t rs = bucket_rsrc(src, len * 4u);
#pragma unroll
    for (int i = 0; i < ITEMS; ++i)
        k[i] = __builtin_amdgcn_raw_buffer_load_b32(rs, (i * BLOCK + (int)threadIdx.x) * 4, 0, 0);
    if (FIN) {
#pragma unroll
        for (int i = 0; i < ITEMS; ++i) k[i] ^= kFlip;
    }
}

// Shared K3u body: unstable partition of one tile [t0, t0 + len) of `in` by digit `shift`.
// dst_base (tid < 256) = out + global start of this tile's digit-tid keys.
// OT = uint16_t stores only the low 16 bits of every key (the packed send buffer of the
// distributed radix, whose groups are the top 16 bits).
// resv != nullptr (K3a): the tile reserves its digit runs instead, one returning device-scope
// atomicAdd on resv[digit] (a u32 cursor into out, relative to out) per non-empty digit, issued
// as soon as the tile's counts are known and consumed only after the LDS scatter; dst_base is
// then ignored.
template <int BLOCK, int ITEMS, bool FIN, bool FOUT, typename OT = uint32_t>
__device__ __forceinline__ void partition_tile(const uint32_t *__restrict__ in, uint64_t t0,
                                               uint32_t len, int shift, OT *dst_base,
                                               uint32_t *s_keys, uint32_t *s_cur,
                                               OT **s_dst, uint32_t *s_wsum,
                                               uint32_t *resv = nullptr,
                                               OT *out = nullptr) {
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    constexpr int TILE = BLOCK * ITEMS;
    const bool full = len == (uint32_t)TILE;
    if (tid < kRadix) s_cur[tid] = 0;
    uint32_t k[ITEMS];
    load_tile<BLOCK, ITEMS, FIN>(in + t0 + tid, full, len, k);
    __syncthreads();
    uint32_t r[ITEMS];
#pragma unroll
    for (int i = 0; i < ITEMS; ++i)
        if (full || (uint32_t)(i * BLOCK + tid) < len)
            r[i] = agg_rank(s_cur, (k[i] >> shift) & 255u, s_cur + kRadix);
    __syncthreads();
    uint32_t c = 0, excl = 0;
    unsigned long long pos = 0;
    if (tid < kRadix) {
        c = s_cur[tid];
        if (resv && c) pos = atomicAdd(&resv[tid], c);
        uint32_t v = c;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const uint32_t t = __shfl_up(v, o);
            if (lane >= o) v += t;
        }
        if (lane == 63) s_wsum[w] = v;
        excl = v - c;
    }
    __syncthreads();
    if (tid < kRadix) {
        for (int ww = 0; ww < w; ++ww) excl += s_wsum[ww];
        s_cur[tid] = excl;
    }
    __syncthreads();
#pragma unroll
    for (int i = 0; i < ITEMS; ++i)
        if (full || (uint32_t)(i * BLOCK + tid) < len)
            s_keys[s_cur[(k[i] >> shift) & 255u] + r[i]] = k[i];
    if (tid < kRadix) s_dst[tid] = (resv ? out + pos : dst_base) - excl;
    __syncthreads();
#pragma unroll
    for (int i = 0; i < ITEMS; ++i) {
        const uint32_t j = (uint32_t)(i * BLOCK + tid);
        if (full || j < len) {
            const uint32_t key = s_keys[j];
            st_global(s_dst[(key >> shift) & 255u] + j, (OT)(FOUT ? (key ^ kFlip) : key));
        }
    }
}

// K3u (level 3, global tiles): offsets from K1/K2 exactly as K3.
template <int BLOCK, int ITEMS, bool FIN>
__global__ __launch_bounds__(BLOCK) void k_partition(const uint32_t *__restrict__ in,
                                                     uint32_t *__restrict__ out, uint64_t n,
                                                     int shift, const uint32_t *__restrict__ toff,
                                                     const unsigned long long *__restrict__ gpfx,
                                                     const unsigned long long *__restrict__ bases) {
    constexpr int TILE = BLOCK * ITEMS;
    static_assert(TILE == kSweepTile, "K1/K2 count tiles of kSweepTile keys");
    __shared__ uint32_t s_keys[TILE];
    __shared__ uint32_t s_cur[kRadix + kAggSpare];  // + agg_rank spare words
    __shared__ uint32_t *s_dst[kRadix];
    __shared__ uint32_t s_wsum[kRadix / 64];
    const uint32_t tile = xcd_tile(blockIdx.x, gridDim.x);
    const uint64_t t0 = (uint64_t)tile * TILE;
    const uint32_t len = (uint32_t)(n - t0 < (uint64_t)TILE ? n - t0 : (uint64_t)TILE);
    uint32_t *dst_base = nullptr;
    if (threadIdx.x < kRadix)
        dst_base = out + bases[threadIdx.x] +
                   gpfx[(uint64_t)(tile / kScanGroup) * kRadix + threadIdx.x] +
                   toff[(uint64_t)tile * kRadix + threadIdx.x];
    partition_tile<BLOCK, ITEMS, FIN, false>(in, t0, len, shift, dst_base, s_keys, s_cur, s_dst,
                                             s_wsum);
}

// Tile -> segment geometry of a segmented pass.
struct SegTile {
    uint32_t seg;    // segment index
    uint32_t group;  // global scan-group index
    uint64_t t0;     // first key
    uint32_t len;    // keys in this tile (0: tile beyond the last segment)
};
__device__ __forceinline__ SegTile seg_tile(uint32_t t, const unsigned long long *segs,
                                            const uint32_t *tpfx, const uint32_t *gpfx,
                                            const uint32_t *segmap, uint32_t nseg) {
    SegTile st{0, 0, 0, 0};
    if (t >= tpfx[nseg]) return st;
    const uint32_t s = segmap[t];
    const uint32_t j = t - tpfx[s];
    const uint64_t a = segs[2 * s] + (uint64_t)j * kSweepTile;
    const uint64_t e = segs[2 * s] + segs[2 * s + 1];
    st.seg = s;
    st.group = gpfx[s] + j / kScanGroup;
    st.t0 = a;
    st.len = (uint32_t)(e - a < (uint64_t)kSweepTile ? e - a : (uint64_t)kSweepTile);
    return st;
}

// K12a: tpfx[s] / gpfx[s] = tiles / scan groups before segment s (one 1024-thread block).
__global__ __launch_bounds__(1024) void k_seg_plan(const unsigned long long *__restrict__ segs,
                                                   uint32_t nseg, uint32_t *__restrict__ tpfx,
                                                   uint32_t *__restrict__ gpfx) {
    __shared__ uint32_t s_t[16], s_g[16];
    const uint32_t tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const uint32_t per = (nseg + 1023) / 1024, s0 = tid * per;
    uint32_t st = 0, sg = 0;
    for (uint32_t j = 0; j < per && s0 + j < nseg; ++j) {
        const uint32_t nt = (uint32_t)((segs[2 * (s0 + j) + 1] + kSweepTile - 1) / kSweepTile);
        st += nt;
        sg += (nt + kScanGroup - 1) / kScanGroup;
    }
    uint32_t vt = st, vg = sg;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t a = __shfl_up(vt, o), b = __shfl_up(vg, o);
        if (lane >= o) { vt += a; vg += b; }
    }
    if (lane == 63) { s_t[w] = vt; s_g[w] = vg; }
    __syncthreads();
    uint32_t rt = vt - st, rg = vg - sg;
    for (uint32_t ww = 0; ww < w; ++ww) { rt += s_t[ww]; rg += s_g[ww]; }
    for (uint32_t j = 0; j < per && s0 + j < nseg; ++j) {
        tpfx[s0 + j] = rt;
        gpfx[s0 + j] = rg;
        const uint32_t nt = (uint32_t)((segs[2 * (s0 + j) + 1] + kSweepTile - 1) / kSweepTile);
        rt += nt;
        rg += (nt + kScanGroup - 1) / kScanGroup;
    }
    if (tid == 1023) {
        uint32_t tt = 0, tg = 0;
        for (int ww = 0; ww < 16; ++ww) { tt += s_t[ww]; tg += s_g[ww]; }
        tpfx[nseg] = tt;
        gpfx[nseg] = tg;
    }
}

// K12b: segmap[t] = segment of tile t, groupmap[G] = segment of scan group G (block = segment).
__global__ __launch_bounds__(256) void k_seg_map(const uint32_t *__restrict__ tpfx,
                                                 const uint32_t *__restrict__ gpfx,
                                                 uint32_t *__restrict__ segmap,
                                                 uint32_t *__restrict__ groupmap) {
    const uint32_t s = blockIdx.x;
    for (uint32_t t = tpfx[s] + threadIdx.x; t < tpfx[s + 1]; t += 256) segmap[t] = s;
    for (uint32_t g = gpfx[s] + threadIdx.x; g < gpfx[s + 1]; g += 256) groupmap[g] = s;
}

// K1s: digit counts of one tile per block: SEG=false, global tile t = [t*kSweepTile, ...);
// SEG=true, tile t of the segment plan (grid may exceed the tiles).  Block-strided dword
// loads (segments start anywhere), all issued before the first LDS atomic.
template <int BLOCK, bool SEG, bool FIN>
__global__ __launch_bounds__(BLOCK) void k_seg_counts(const uint32_t *__restrict__ in,
                                                      uint64_t n,
                                                      const unsigned long long *__restrict__ segs,
                                                      const uint32_t *__restrict__ tpfx,
                                                      const uint32_t *__restrict__ gpfx,
                                                      const uint32_t *__restrict__ segmap,
                                                      uint32_t nseg, int shift,
                                                      uint32_t *__restrict__ tcounts) {
    constexpr int ITEMS = kSweepTile / BLOCK;
    __shared__ uint32_t s_h[kRadix + kAggSpare];
    const uint32_t t = blockIdx.x, tid = threadIdx.x;
    uint64_t t0;
    uint32_t len;
    if (SEG) {
        const SegTile st = seg_tile(t, segs, tpfx, gpfx, segmap, nseg);
        if (st.len == 0) return;
        t0 = st.t0;
        len = st.len;
    } else {
        t0 = (uint64_t)t * kSweepTile;
        len = (uint32_t)(n - t0 < (uint64_t)kSweepTile ? n - t0 : (uint64_t)kSweepTile);
    }
    for (uint32_t b = tid; b < kRadix; b += BLOCK) s_h[b] = 0;
    uint32_t k[ITEMS];
    load_tile<BLOCK, ITEMS, FIN>(in + t0 + tid, len == (uint32_t)kSweepTile, len, k);
    __syncthreads();
#pragma unroll
    for (int i = 0; i < ITEMS; ++i)
        if ((uint32_t)(i * BLOCK) + tid < len) agg_rank(s_h, (k[i] >> shift) & 255u, s_h + kRadix);
    __syncthreads();
    for (uint32_t b = tid; b < kRadix; b += BLOCK) tcounts[(uint64_t)t * kRadix + b] = s_h[b];
}

// K2s-a: group-local exclusive scan of the tile counts of each scan group (group = block).
__global__ __launch_bounds__(kRadix) void k_seg_scan_tiles(uint32_t *__restrict__ tcounts,
                                                           const uint32_t *__restrict__ tpfx,
                                                           const uint32_t *__restrict__ gpfx,
                                                           const uint32_t *__restrict__ groupmap,
                                                           uint32_t nseg,
                                                           unsigned long long *__restrict__ gsum) {
    const uint32_t g = blockIdx.x, d = threadIdx.x;
    if (g >= gpfx[nseg]) return;
    const uint32_t s = groupmap[g];
    const uint32_t t0 = tpfx[s] + (g - gpfx[s]) * kScanGroup;
    const uint32_t nt = min((uint32_t)kScanGroup, tpfx[s + 1] - t0);
    uint32_t c[kScanGroup];
#pragma unroll
    for (int j = 0; j < kScanGroup; ++j)
        c[j] = (uint32_t)j < nt ? tcounts[(uint64_t)(t0 + j) * kRadix + d] : 0u;
    uint32_t run = 0;
#pragma unroll
    for (int j = 0; j < kScanGroup; ++j) {
        if ((uint32_t)j < nt) tcounts[(uint64_t)(t0 + j) * kRadix + d] = run;
        run += c[j];
    }
    gsum[(uint64_t)g * kRadix + d] = run;
}

// Child buckets -> work lists (WorkLists, gsort_kernels.h): > kLocalMax keys to the next
// level, the rest to K11's size classes.  Called by all kRadix threads of a block (one child
// each): the block reserves its entries with one global atomic per list, so the counters see
// a few atomics per block, not one per child.
// merge (the block's children are consecutive buckets of one parent, in key order): runs of
// small children (<= kMergeWin keys each) are merged into one K11 entry of <= 2 kMergeWin keys
// -- children whose starts fall in one kMergeWin-aligned window of the parent -- sorted with one
// more digit (the digit that split them), flagged in the entry's high word.  Dense or sorted
// inputs otherwise end in ~256-key buckets, one K11 workgroup each at a few % of its slots
// (a sorted 2^28-key input spent 2.1 ms in K11, tools/dist_probe.py).
constexpr uint64_t kMergeWin = kLocalCap[2] / 2;

__device__ __forceinline__ void classify_block(uint64_t start, uint64_t len, const WorkLists &wl,
                                               bool merge = false) {
    constexpr int NL = kLocalClasses + 1;
    __shared__ unsigned int s_n[NL];
    __shared__ unsigned long long s_keys[NL], s_max[NL], s_base[NL];
    __shared__ unsigned long long s_gsum[kRadix], s_gkey[kRadix], s_wx[kRadix / 64];
    __shared__ unsigned int s_gcnt[kRadix], s_wl[kRadix / 64];
    const uint32_t tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    if (tid < NL) { s_n[tid] = 0; s_keys[tid] = 0; s_max[tid] = 0; }
    uint32_t extra = 0;  // digits the K11 entry sorts beyond its list's
    bool absorbed = false;
    merge = merge && !wl.force_next;
    if (merge) {
        // exclusive prefix of the children's lengths (block scan)
        unsigned long long x = len;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const unsigned long long t = __shfl_up(x, o);
            if ((int)lane >= o) x += t;
        }
        if (lane == 63) s_wx[w] = x;
        s_gsum[tid] = 0;
        s_gcnt[tid] = 0;
        __syncthreads();
        unsigned long long excl = x - len;
        for (uint32_t ww = 0; ww < w; ++ww) excl += s_wx[ww];
        const bool small = len > 0 && len <= kMergeWin;
        const unsigned long long g = excl / kMergeWin;
        s_gkey[tid] = small ? g : ~0ull;
        __syncthreads();
        // the group's first child: the nearest child at or before this one opening group g
        // (an inclusive max-scan of the opening children's indices)
        const bool opens = small && (tid == 0 || s_gkey[tid - 1] != g);
        uint32_t lead = opens ? tid : 0u;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const uint32_t t = __shfl_up(lead, o);
            if ((int)lane >= o) lead = max(lead, t);
        }
        if (lane == 63) s_wl[w] = lead;
        __syncthreads();
        for (uint32_t ww = 0; ww < w; ++ww) lead = max(lead, s_wl[ww]);
        if (small) {
            atomicAdd(&s_gsum[lead], len);
            atomicAdd(&s_gcnt[lead], 1u);
        }
        __syncthreads();
        if (small) {
            if (!opens) {
                absorbed = true;
            } else {
                len = s_gsum[tid];
                extra = s_gcnt[tid] > 1 ? 1u : 0u;
            }
        }
    } else {
        __syncthreads();
    }
    int which = -1;
    if (len > 0 && !absorbed) {
        which = 0;
        if (!wl.force_next)
            for (int k = 1; k < NL; ++k)
                if (len <= kLocalCap[k]) { which = k; break; }
    }
    unsigned int idx = 0;
    if (which >= 0) {
        idx = atomicAdd(&s_n[which], 1u);
        atomicAdd(&s_keys[which], (unsigned long long)len);
        atomicMax(&s_max[which], (unsigned long long)len);
    }
    __syncthreads();
    if (tid < NL && s_n[tid]) {
        unsigned long long *ctr = reinterpret_cast<unsigned long long *>(wl.ctr) + 3 * tid;
        s_base[tid] = atomicAdd(&ctr[0], (unsigned long long)s_n[tid]);
        atomicAdd(&ctr[1], s_keys[tid]);
        atomicMax(&ctr[2], s_max[tid]);
    }
    __syncthreads();
    if (which >= 0) {
        unsigned long long *list = reinterpret_cast<unsigned long long *>(wl.list[which]);
        const unsigned long long i = s_base[which] + idx;
        list[2 * i] = start;
        list[2 * i + 1] = len | ((unsigned long long)extra << 32);
    }
}

// K2s-b: per segment (block) and digit (thread): exclusive scan over the segment's scan
// groups (in place), then the child bucket starts; classify the children.
__global__ __launch_bounds__(kRadix) void k_seg_scan_groups(
    unsigned long long *__restrict__ gsum, const unsigned long long *__restrict__ segs,
    const uint32_t *__restrict__ gpfx, unsigned long long *__restrict__ cstart, WorkLists wl) {
    __shared__ unsigned long long s_w[kRadix / 64];
    const uint32_t s = blockIdx.x, d = threadIdx.x, lane = d & 63, w = d >> 6;
    const uint32_t g0 = gpfx[s], g1 = gpfx[s + 1];
    unsigned long long run = 0;
    for (uint32_t g = g0; g < g1; g += 16) {
        unsigned long long v[16];
#pragma unroll
        for (int j = 0; j < 16; ++j) v[j] = g + j < g1 ? gsum[(uint64_t)(g + j) * kRadix + d] : 0ull;
#pragma unroll
        for (int j = 0; j < 16; ++j) {
            if (g + j < g1) gsum[(uint64_t)(g + j) * kRadix + d] = run;
            run += v[j];
        }
    }
    unsigned long long x = run;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const unsigned long long t = __shfl_up(x, o);
        if (lane >= o) x += t;
    }
    if (lane == 63) s_w[w] = x;
    __syncthreads();
    unsigned long long excl = x - run;
    for (uint32_t ww = 0; ww < w; ++ww) excl += s_w[ww];
    const uint64_t start = segs[2 * s] + excl;
    cstart[(uint64_t)s * kRadix + d] = start;
    if (wl.ctr) classify_block(start, run, wl, true);
}

// Level-3 children: the 256 buckets of the global pass.
__global__ __launch_bounds__(kRadix) void k_classify_buckets(
    const unsigned long long *__restrict__ bases, const unsigned long long *__restrict__ totals,
    WorkLists wl) {
    const uint32_t d = threadIdx.x;
    classify_block(bases[d], totals[d], wl, true);
}

// K3u (segmented): one block per segment tile.
template <int BLOCK, int ITEMS, bool FOUT, typename OT = uint32_t, bool FIN = false>
__global__ __launch_bounds__(BLOCK) void k_seg_partition(
    const uint32_t *__restrict__ in, OT *__restrict__ out, int shift,
    const uint32_t *__restrict__ toff, const unsigned long long *__restrict__ gpfx64,
    const unsigned long long *__restrict__ cstart, const unsigned long long *__restrict__ segs,
    const uint32_t *__restrict__ tpfx, const uint32_t *__restrict__ gpfx,
    const uint32_t *__restrict__ segmap, uint32_t nseg) {
    constexpr int TILE = BLOCK * ITEMS;
    static_assert(TILE == kSweepTile, "segment tiles are kSweepTile keys");
    __shared__ uint32_t s_keys[TILE];
    __shared__ uint32_t s_cur[kRadix + kAggSpare];  // + agg_rank spare words
    __shared__ OT *s_dst[kRadix];
    __shared__ uint32_t s_wsum[kRadix / 64];
    const uint32_t t = xcd_tile(blockIdx.x, gridDim.x);
    const SegTile st = seg_tile(t, segs, tpfx, gpfx, segmap, nseg);
    if (st.len == 0) return;
    OT *dst_base = nullptr;
    if (threadIdx.x < kRadix)
        dst_base = out + cstart[(uint64_t)st.seg * kRadix + threadIdx.x] +
                   gpfx64[(uint64_t)st.group * kRadix + threadIdx.x] +
                   toff[(uint64_t)t * kRadix + threadIdx.x];
    partition_tile<BLOCK, ITEMS, FIN, FOUT, OT>(in, st.t0, st.len, shift, dst_base, s_keys, s_cur,
                                              s_dst, s_wsum);
}

// =======================================================================================
// Two-level plan (default MSD front end): levels 3 and 2 without per-tile counting passes.
//   K1h  histogram of the top 16 bits of every key (one returning LDS atomic per key)
//   K12a the 65536 level-2 child counts, and each level-3 bucket's count per shard
//   K12b bucket bases, child starts, the level-3 (per shard) and level-2 cursors, the K11
//        work lists and the K3a tile plan -- all before level 3 runs
//   K3r  level 3: every pair of input tiles reserves its 256 digit runs with one atomicAdd per
//        digit on its shard's bucket cursors (an MSD level only needs every key in its
//        bucket, not a stable order), then scatters through LDS
//   K3a  level 2: the same over the tiles of every level-3 bucket, on its child cursors
// A shard is one XCD's share of the tiles: tile pair p is processed by workgroup p of K1h's
// and K3r's grids, which runs on XCD p % 8 (workgroups are dealt round-robin over the 8
// XCDs), and counts / reserves under shard p % 8.  So every cursor takes 1/8 of a bucket's
// reservations (a single device-scope counter saturates near 88 M atomics/s,
// MI355X_MICROARCH.md 'dequeue'), and consecutive runs of a bucket share one XCD's L2.
// Replaced (v0-v8): K1 + K2 tile counts and scans for level 3, and a second LDS atomic per key
// in K1h for them.  Level 3 + 2 + K11 = 4 + 8 + 8 + 8 = 28 B/key.
// =======================================================================================
constexpr uint32_t kShards = kH16Shards;

// A u16 half of K1h's packed LDS counters that wraps is seen by exactly one thread, whose
// returning atomic read 0xffff in that half, and repaired through fix[] (u64, zeroed by the
// caller): a wrapped low half lost 65536 and carried one into the high half; a carry out of
// the whole word (a high half wrapping, or a low add on 0xffffffff) lost 65536 of the high bin.
// Hence count[h] = sum_b half_h(part[b]) + fix[h] (mod 2^64), per shard.
__device__ __forceinline__ void h16_wrap(unsigned long long *fix, uint32_t b, uint32_t old) {
    atomicAdd(&fix[b], 65536ull);
    if (!(b & 1u)) {
        atomicAdd(&fix[b | 1u], ~0ull);  // -1: the carry into the high half
        if (old == 0xffffffffu) atomicAdd(&fix[b | 1u], 65536ull);
    }
}

// K1h: per workgroup, a histogram of the top 16 bits (ordered u32) of its tiles, as 32768
// packed u16 pairs in LDS (128 KiB: one 1024-thread workgroup per CU), stored to
// part[blockIdx.x][.] at the end.  Workgroup b takes the tile pairs p = b, b + G, b + 2G, ..
// (G = gridDim.x, a multiple of kShards, so shard p % 8 == b % 8) and prefetches its next tile
// while it counts the current one.  Wraps go to fix[b % 8][.].
template <int BLOCK, bool FIN>
__global__ __launch_bounds__(BLOCK) void k_hist16(const uint32_t *__restrict__ in, uint64_t n,
                                                  uint32_t *__restrict__ part,
                                                  unsigned long long *__restrict__ fix) {
    constexpr int ITEMS = kSweepTile / BLOCK;
    constexpr uint32_t kWords = kBuckets16 / 2;
    __shared__ uint32_t s_h[kWords + kAggSpare];
    uint32_t *spare = s_h + kWords;
    const uint32_t tid = threadIdx.x;
    for (uint32_t i = tid; i < kWords; i += BLOCK) s_h[i] = 0;
    // tile lengths in 32-bit scalar arithmetic (tools/isa_scc_check.py: the u64 min() form was
    // miscompiled by ROCm 7.2 and loaded a full tile past the input's end)
    const uint32_t ntiles = (uint32_t)((n + kSweepTile - 1) / kSweepTile);
    const uint32_t last_len = (uint32_t)(n - (uint64_t)(ntiles - 1) * kSweepTile);
    auto tile_len = [&](uint32_t t) -> uint32_t {
        return t == ntiles - 1 ? last_len : (uint32_t)kSweepTile;
    };
    auto tile_of = [&](uint32_t i) -> uint32_t {  // this workgroup's i-th tile
        return 2 * (blockIdx.x + (i >> 1) * gridDim.x) + (i & 1);
    };
    unsigned long long *fx = fix + (uint64_t)(blockIdx.x % kShards) * kBuckets16;
    uint32_t t = tile_of(0);
    uint32_t k[ITEMS];
    if (t < ntiles) {
        const uint32_t len = tile_len(t);
        load_tile<BLOCK, ITEMS, FIN>(in + (uint64_t)t * kSweepTile + tid,
                                     len == (uint32_t)kSweepTile, len, k);
    }
    __syncthreads();  // zeroing done
    for (uint32_t i = 1; t < ntiles; ++i) {
        const uint32_t len = tile_len(t);
        const uint32_t tn = tile_of(i);
        uint32_t kn[ITEMS];
        if (tn < ntiles) {
            const uint32_t lenn = tile_len(tn);
            load_tile<BLOCK, ITEMS, FIN>(in + (uint64_t)tn * kSweepTile + tid,
                                         lenn == (uint32_t)kSweepTile, lenn, kn);
        }
        // all returning atomics in flight before the first wrap test; every tile but the
        // input's last is full, and its atomics and wrap tests go without per-key bounds
        // (tools/experiments/kexp13.hip: the bounded form cost 12 %)
        uint32_t old[ITEMS];
        bool wrap = false;
        // skewed wave (its first item's keys all in one packed word: duplicates, sorted runs,
        // Zipf): aggregated adds; otherwise plain ones (the aggregation's VALU would cost the
        // uniform case ~25 %)
        const uint32_t w0 = __builtin_amdgcn_readfirstlane(k[0] >> 17);
        const bool skew = __ballot((k[0] >> 17) == w0) == __builtin_amdgcn_read_exec();
        if (len == (uint32_t)kSweepTile && skew) {
#pragma unroll
            for (int j = 0; j < ITEMS; ++j) old[j] = agg_add_pair(s_h, k[j] >> 16, spare);
#pragma unroll
            for (int j = 0; j < ITEMS; ++j)
                wrap |= ((old[j] >> (((k[j] >> 16) & 1u) << 4)) & 0xffffu) == 0xffffu;
        } else if (len == (uint32_t)kSweepTile) {
#pragma unroll
            for (int j = 0; j < ITEMS; ++j) {
                const uint32_t b = k[j] >> 16;
                old[j] = atomicAdd(&s_h[b >> 1], 1u << ((b & 1u) << 4));
            }
#pragma unroll
            for (int j = 0; j < ITEMS; ++j)
                wrap |= ((old[j] >> (((k[j] >> 16) & 1u) << 4)) & 0xffffu) == 0xffffu;
        } else {
#pragma unroll
            for (int j = 0; j < ITEMS; ++j) {
                old[j] = 0;
                if ((uint32_t)(j * BLOCK) + tid < len) old[j] = agg_add_pair(s_h, k[j] >> 16, spare);
            }
#pragma unroll
            for (int j = 0; j < ITEMS; ++j)
                wrap |= (uint32_t)(j * BLOCK) + tid < len &&
                        ((old[j] >> (((k[j] >> 16) & 1u) << 4)) & 0xffffu) == 0xffffu;
        }
        if (__builtin_expect(wrap, 0)) {
#pragma unroll
            for (int j = 0; j < ITEMS; ++j) {
                const uint32_t b = k[j] >> 16;
                if ((uint32_t)(j * BLOCK) + tid < len &&
                    ((old[j] >> ((b & 1u) << 4)) & 0xffffu) == 0xffffu)
                    h16_wrap(fx, b, old[j]);
            }
        }
#pragma unroll
        for (int j = 0; j < ITEMS; ++j) k[j] = kn[j];
        t = tn;
    }
    __syncthreads();
    uint32_t *dst = part + (uint64_t)blockIdx.x * kWords;
    for (uint32_t i = tid; i < kWords; i += BLOCK) dst[i] = s_h[i];
}

// Level-3 bucket s goes through level 2 (K3a) when it is too large for K11, or -- force, the
// grouping of the distributed sender -- whenever it is non-empty.
__device__ __forceinline__ bool level2_bucket(unsigned long long tot, int force) {
    return force ? tot > 0 : tot > kLocalMax;
}

// Block-wide (kRadix threads) exclusive scan of one u64 per thread; *total = the sum.
__device__ __forceinline__ unsigned long long block_excl_scan(unsigned long long v,
                                                              unsigned long long *s_w,
                                                              unsigned long long *total) {
    const uint32_t tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    unsigned long long x = v;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const unsigned long long t = __shfl_up(x, o);
        if (lane >= o) x += t;
    }
    __syncthreads();
    if (lane == 63) s_w[w] = x;
    __syncthreads();
    unsigned long long excl = x - v, all = 0;
    for (uint32_t ww = 0; ww < kRadix / 64; ++ww) {
        if (ww < w) excl += s_w[ww];
        all += s_w[ww];
    }
    *total = all;
    return excl;
}

// block_excl_scan of values whose wave sums stay below 2^32 (counts of one block's <= 2^31 keys):
// the wave scan in DPP (no LDS round trip per step, as __shfl_up's bpermute costs), the
// cross-wave sums in 64 bits as above
__device__ __forceinline__ unsigned long long block_excl_scan32(uint32_t v, unsigned long long *s_w,
                                                                unsigned long long *total) {
    const uint32_t tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const uint32_t x = wave_incl_add(v);
    __syncthreads();
    if (lane == 63) s_w[w] = x;
    __syncthreads();
    unsigned long long excl = x - v, all = 0;
    for (uint32_t ww = 0; ww < kRadix / 64; ++ww) {
        if (ww < w) excl += s_w[ww];
        all += s_w[ww];
    }
    *total = all;
    return excl;
}

// K12a: block s = level-3 digit, thread e = level-2 digit.  The count of child (s, e) in shard
// x = the e-half of word s*128 + e/2 summed over the partials b = x (mod 8), + fix[x][s*256+e].
// Writes ccount[s*256+e] (all shards), t3[x*256+s] (bucket s in shard x) and tot[s].
// nblk is a multiple of kShards.
// K12a also leaves fix[] zeroed for the next K1h (each entry is read by one thread, then
// cleared) and block 0 zeroes the nzero work-list counters at zero (K12b's atomics follow), so
// a sort needs no memset before K1h.
__global__ __launch_bounds__(kRadix) void k_plan16_count(const uint32_t *__restrict__ part,
                                                         uint32_t nblk,
                                                         unsigned long long *__restrict__ fix,
                                                         unsigned long long *__restrict__ ccount,
                                                         unsigned long long *__restrict__ t3,
                                                         unsigned long long *__restrict__ tot,
                                                         unsigned long long *__restrict__ zero,
                                                         uint32_t nzero) {
    constexpr uint32_t kWords = kBuckets16 / 2;
    __shared__ uint32_t s_lo[kShards][kRadix / 2], s_hi[kShards][kRadix / 2];
    __shared__ unsigned long long s_red[kShards][kRadix / 64];
    const uint32_t s = blockIdx.x, e = threadIdx.x, lane = e & 63, wv = e >> 6;
    // this thread: word s*128 + (e & 127) over the partials b = par (mod 2), i.e. the shards
    // par, par + 2, par + 4, par + 6 (b, b + 2, b + 4, b + 6 of every group of eight)
    const uint32_t par = e >> 7, word = s * (kRadix / 2) + (e & 127u);
    uint32_t lo[4] = {0, 0, 0, 0}, hi[4] = {0, 0, 0, 0};
    // U groups of eight partials per round, all 4 U loads in flight (a round per group left
    // nblk / 8 dependent HBM round trips: K12a 41 us at 256 partials)
    constexpr uint32_t U = 8;
    for (uint32_t b0 = par; b0 < nblk; b0 += kShards * U) {
        uint32_t v[U][4];
#pragma unroll
        for (uint32_t u = 0; u < U; ++u) {
            const uint32_t b = b0 + u * kShards;  // (b < nblk: b + 6 < nblk too, nblk % 8 == 0)
#pragma unroll
            for (int j = 0; j < 4; ++j)
                v[u][j] = b < nblk ? part[(uint64_t)(b + 2 * j) * kWords + word] : 0u;
        }
#pragma unroll
        for (uint32_t u = 0; u < U; ++u)
#pragma unroll
            for (int j = 0; j < 4; ++j) { lo[j] += v[u][j] & 0xffffu; hi[j] += v[u][j] >> 16; }
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        s_lo[par + 2 * j][e & 127u] = lo[j];
        s_hi[par + 2 * j][e & 127u] = hi[j];
    }
    __syncthreads();
    const uint32_t w2 = e >> 1;
    unsigned long long c = 0, cx[kShards];
#pragma unroll
    for (uint32_t x = 0; x < kShards; ++x) {
        unsigned long long *f = &fix[(uint64_t)x * kBuckets16 + s * kRadix + e];
        cx[x] = (unsigned long long)((e & 1u) ? s_hi[x][w2] : s_lo[x][w2]) + *f;
        *f = 0;
        c += cx[x];
    }
    ccount[s * kRadix + e] = c;
    if (s == 0 && e < nzero) zero[e] = 0;
#pragma unroll
    for (uint32_t x = 0; x < kShards; ++x) {
        unsigned long long r = cx[x];
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) r += __shfl_xor(r, o);
        if (lane == 0) s_red[x][wv] = r;
    }
    __syncthreads();
    if (e < kShards) {
        unsigned long long r = 0;
        for (uint32_t ww = 0; ww < kRadix / 64; ++ww) r += s_red[e][ww];
        t3[e * kRadix + s] = r;
    }
    if (e == kShards) {
        unsigned long long r = 0;
        for (uint32_t x = 0; x < kShards; ++x)
            for (uint32_t ww = 0; ww < kRadix / 64; ++ww) r += s_red[x][ww];
        tot[s] = r;
    }
}

// K12b: block s, thread e.  bases[s] = the keys of level-3 buckets < s; child (s, e) starts at
// cstart[s*256+e] = bases[s] + its exclusive scan over e (the 65536 bucket bounds of the top 16
// bits; cstart[65536] = n); a level-2 bucket's child cursors cur[s*256+e] (u32, from bases[s])
// and the child in wl2 (K11 classes / next level); any other non-empty bucket s whole in wl3
// (K11 on three digits); the level-3 cursors cur3[x*256+s] = the keys of bucket s in shards
// < x (u32, from bases[s]).  Block 0 also writes bases / totals (256 u64 each) and tpfx[0..256],
// the K3a tiles before each level-2 bucket.
__global__ __launch_bounds__(kRadix) void k_plan16_place(
    const unsigned long long *__restrict__ ccount, const unsigned long long *__restrict__ t3,
    const unsigned long long *__restrict__ tot, uint64_t n, int force,
    unsigned long long *__restrict__ bases, unsigned long long *__restrict__ totals,
    unsigned long long *__restrict__ cstart, uint32_t *__restrict__ cur,
    uint32_t *__restrict__ cur3, uint32_t *__restrict__ tpfx, WorkLists wl2, WorkLists wl3,
    uint32_t *__restrict__ flags) {
    __shared__ unsigned long long s_w[kRadix / 64];
    __shared__ unsigned long long s_base;
    const uint32_t s = blockIdx.x, e = threadIdx.x;
    const unsigned long long te = tot[e];
    unsigned long long all;
    const unsigned long long be = block_excl_scan(te, s_w, &all);
    if (e == s) s_base = be;
    if (s == 0) { bases[e] = be; totals[e] = te; }
    __syncthreads();
    const unsigned long long b0 = s_base, ts = tot[s];
    const unsigned long long c = ccount[s * kRadix + e];
    // trivial levels (zeroed by K12a): bit 0 = bucket s holds every key, bit 1 = child (s, e)
    if (flags && n > 0) {
        if (e == 0 && ts == n) atomicOr(flags, 1u);
        if (c == n) atomicOr(flags, 2u);
    }
    unsigned long long sum;
    const unsigned long long excl = block_excl_scan(c, s_w, &sum);
    const unsigned long long st = b0 + excl;
    cstart[s * kRadix + e] = st;
    if (s == 0 && e == 0) cstart[kBuckets16] = n;
    if (e == 0) {
        unsigned long long r = 0;
        for (uint32_t x = 0; x < kShards; ++x) {
            cur3[x * kRadix + s] = (uint32_t)r;
            r += t3[x * kRadix + s];
        }
    }
    if (level2_bucket(ts, force)) {
        cur[s * kRadix + e] = (uint32_t)excl;
        if (wl2.ctr) classify_block(st, c, wl2, true);
    } else if (wl3.ctr) {
        classify_block(e == 0 ? b0 : 0ull, e == 0 ? ts : 0ull, wl3);
    }
    if (s == 0) {
        const unsigned long long nt =
            level2_bucket(te, force) ? (te + kSweepTile - 1) / kSweepTile : 0ull;
        unsigned long long ntall;
        const unsigned long long tx = block_excl_scan(nt, s_w, &ntall);
        tpfx[e] = (uint32_t)tx;
        if (e == 0) tpfx[kRadix] = (uint32_t)ntall;
    }
}

// K12c: the K3a tile descriptors, one thread per level-2 tile t < tpfx[256]: its bucket s
// (tpfx[s] <= t < tpfx[s+1]), first key and length.  K3a then reaches its keys after one
// (scalar) load instead of a tpfx load, an LDS binary search and two dependent loads of the
// bucket bounds -- a chain every one of its ~16K single-pair workgroups exposed.
// The sampled plan's words in the pinned host mailbox (relative to the `mail` pointer the
// runtime passes): the status {eflag, ovf} and its sequence after K12g, the same after K12e
// (eligibility only), the 15 work-list counters after K12g.
constexpr uint32_t kMailStatus = 0, kMailSeq = 1, kMailElig = 2, kMailEligSeq = 3,
                   kMailChildren = 4, kMailVary = 5, kMailLo = 6, kMailHi = 7, kMailCtr = 8,
                   kMailMaxChild = 23;

__device__ __forceinline__ void mail_release(unsigned long long *flag, unsigned long long seq) {
    __threadfence_system();
    __hip_atomic_store(flag, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

// The eligibility word and the count of sampled children for the host (K12e has completed).
__device__ __forceinline__ void publish_elig(unsigned long long *mail, const uint32_t *eflag,
                                             unsigned long long seq) {
    if (threadIdx.x == 0) {
        mail[kMailElig] = *reinterpret_cast<const unsigned long long *>(eflag);
        mail[kMailChildren] = eflag[4];
        mail[kMailVary] = eflag[5];
        mail[kMailLo] = eflag[6];
        mail[kMailHi] = eflag[7];
        mail[kMailMaxChild] = eflag[8];
        mail_release(mail + kMailEligSeq, seq);
    }
}

constexpr uint32_t kStraddle = 0x80000000u;  // K12f: a K3a tile across level-3 pieces
struct TileDesc {
    unsigned long long t0;
    uint32_t len, seg;
};
__global__ __launch_bounds__(256) void k_tile_desc(const uint32_t *__restrict__ tpfx,
                                                   const unsigned long long *__restrict__ bases,
                                                   const unsigned long long *__restrict__ totals,
                                                   uint32_t max_tiles,
                                                   TileDesc *__restrict__ desc) {
    __shared__ uint32_t s_tp[kRadix + 1];
    for (uint32_t i = threadIdx.x; i <= kRadix; i += 256) s_tp[i] = tpfx[i];
    __syncthreads();
    const uint32_t t = blockIdx.x * 256 + threadIdx.x;
    if (t >= max_tiles || t >= s_tp[kRadix]) return;
    uint32_t lo = 0, hi = kRadix;  // s_tp[lo] <= t < s_tp[hi]
    while (hi - lo > 1) {
        const uint32_t mid = (lo + hi) >> 1;
        if (s_tp[mid] <= t) lo = mid;
        else hi = mid;
    }
    const unsigned long long b0 = bases[lo], end = b0 + totals[lo];
    const unsigned long long t0 = b0 + (unsigned long long)(t - s_tp[lo]) * kSweepTile;
    const unsigned long long rem = end - t0;
    desc[t] = {t0, (rem >> 13) ? (uint32_t)kSweepTile : (uint32_t)rem, lo};
}

// Phase stamps (diagnostic build only: make VARIANT=stamps EXTRA=-DGSORT_STAMPS lib; never in
// the product).  Thread 0 of every K3r / K3a (sampled plan) workgroup writes s_memrealtime
// (100 MHz) at 7 points -- kernel entry (6), tile known (0), loads landed, ranked, reservations
// returned, scattered into LDS, stores completed (5) -- each behind a workgroup barrier (and a
// vmcnt(0) wait where a phase ends in memory traffic), to
// g_stamps[(L3 ? 0 : 1) * kStampWGs + workgroup][8]
// (tools/k3_stamps.py).
#ifdef GSORT_STAMPS
constexpr uint32_t kStampWGs = 32768;
__device__ unsigned long long *g_stamps = nullptr;
// (kept in LDS until the workgroup's last stamp: a global pointer live across the kernel cost
// it SGPRs past 80 -- 7 waves per SIMD, one workgroup per CU, half the live workgroups)
#define K3_STAMP(p)                                                                            \
    do {                                                                                       \
        __syncthreads();                                                                       \
        if (EST && threadIdx.x == 0) s_stamp[p] = __builtin_amdgcn_s_memrealtime();            \
        if (EST && (p) == 5 && threadIdx.x < 8 && g_stamps && blockIdx.x < kStampWGs)          \
            g_stamps[((L3 ? 0ull : 1ull) * kStampWGs + blockIdx.x) * 8 + threadIdx.x] =        \
                s_stamp[threadIdx.x]; /* (lanes of wave 0: lane 0's LDS write is visible) */   \
    } while (0)
#define K3_STAMP_DECL __shared__ unsigned long long s_stamp[8]
#define K3_STAMP_WAIT() asm volatile("s_waitcnt vmcnt(0)" ::: "memory")
#else
#define K3_STAMP(p) do { } while (0)
#define K3_STAMP_DECL
#define K3_STAMP_WAIT() do { } while (0)
#endif

// K3r / K3a: one workgroup per PAIR of tiles.  Both tiles are ranked (one LDS atomic per key)
// before either reservation is needed, so the two reservations (one returning device-scope
// atomicAdd per non-empty digit) are in flight together and their round trip hides behind
// twice the LDS scan + scatter; LDS holds both tiles (2 x 32 KiB: two 1024-thread workgroups
// per CU).
//   L3 (K3r): level 3 of the input (int32, FIN flips to ordered u32): tile pair p = blockIdx.x,
//     tiles 2p and 2p+1; digit runs reserved on cur[(p % 8) * 256 + d] (K12b's cur3), placed
//     at bases[d] + the reservation.
//   !L3 (K3a): level 2 of every level-2 bucket (in = level 3's output, ordered u32): the
//     K12b tile plan tpfx maps tile t to bucket s (tpfx[s] <= t < tpfx[s+1]); pairs are dealt
//     XCD-contiguously (xcd_tile); runs reserved on cur[s * 256 + d], placed at bases[s] + the
//     reservation; out may be uint16_t (only the low 16 bits: the distributed sender's packed
//     send buffer).
// Trivial levels (flags != nullptr: K12b's word, bit 0 = one level-3 bucket holds every key,
// bit 1 = one 16-bit child does): K3r does nothing when bit 0 is set, and K3a then partitions
// the int32 input raw itself (flipping on load); K3a does nothing when bit 1 is set (the
// caller continues from level 1 on the input).  Each level that moved keys without changing
// their order cost a full pass (16-bit keys took four partitions).
// EST (the sampled plan, "Sampled plan" below): every cursor run must end below its limit
// lim[same index as cur] (the run's region, sized from a sample); a run that would not fits
// raises *ovf and goes to the TILE-key scratch `dump` instead (the caller then re-sorts on the
// exact plan).  flags bit 2 (the sample found the input ineligible): do nothing.
template <int BLOCK, int ITEMS, bool L3, bool FIN, typename OT = uint32_t, bool EST = false,
          int TILES = 2>
__global__ __launch_bounds__(BLOCK, TILES == 1 ? 6 : 1) void k_partition_res(
    const uint32_t *__restrict__ in, OT *__restrict__ out, uint64_t n,
    const uint32_t *__restrict__ tpfx, const TileDesc *__restrict__ desc,
    const unsigned long long *__restrict__ bases, uint32_t *__restrict__ cur,
    const uint32_t *__restrict__ flags, const uint32_t *__restrict__ raw,
    const uint32_t *__restrict__ lim = nullptr, uint32_t *__restrict__ ovf = nullptr,
    OT *__restrict__ dump = nullptr, const TileDesc *__restrict__ pieces = nullptr,
    unsigned long long *mail = nullptr, unsigned long long seq = 0, int sb = 0,
    uint32_t koff = 0) {
    constexpr int TILE = BLOCK * ITEMS;
    const int shift = (L3 ? 24 : 16) - (EST ? sb : 0);  // EST: digits sb bits lower
    static_assert(TILE == kSweepTile, "reservation tiles are kSweepTile keys");
    K3_STAMP_DECL;
    K3_STAMP(6);
    if (EST && L3 && mail && blockIdx.x == 0) publish_elig(mail, flags, seq);  // K12e is done
    uint32_t flip = 0;
    if (flags) {
        const uint32_t f = *flags;
        if (f & (L3 ? 5u : 6u)) return;
        if (EST && !L3 && ovf && *ovf) return;  // level 3 overflowed: the exact plan sorts again
        if (!L3 && (f & 1u)) { in = raw; flip = kFlip; }
    }
    static_assert(TILES == 1 || TILES == 2, "a tile or a pair per workgroup");
    __shared__ uint32_t s_keys[TILES][TILE];
    __shared__ uint32_t s_cur[TILES][kRadix];
    // each digit's run as a u32 index into out minus its LDS start (out holds < 2^32 keys): one
    // 4-B random LDS read per key on the way out instead of an 8-B pointer
    __shared__ uint32_t s_off[TILES][kRadix];
    __shared__ uint32_t s_wsum[TILES][kRadix / 64];
    __shared__ uint32_t s_spare[kAggSpare];
    __shared__ uint32_t s_ovf[TILES];  // EST: a run of this tile overflowed its region
    const uint32_t tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    uint32_t pr, ntile, last_len = 0;
    if (L3) {
        pr = blockIdx.x;
        ntile = (uint32_t)((n + TILE - 1) / TILE);
        last_len = (uint32_t)(n - (uint64_t)(ntile - 1) * TILE);
    } else {
        pr = xcd_tile(blockIdx.x, gridDim.x);
        ntile = tpfx[kRadix];
    }
    if (TILES * pr >= ntile) return;
    K3_STAMP(0);
    uint32_t seg[TILES], len[TILES];
    uint64_t t0[TILES];
    bool straddle[TILES];
#pragma unroll
    for (int h = 0; h < TILES; ++h) {
        const uint32_t t = TILES * pr + h;
        seg[h] = 0; len[h] = 0; t0[h] = 0; straddle[h] = false;
        if (t < ntile) {
            if (L3) {
                t0[h] = (uint64_t)t * TILE;
                len[h] = t == ntile - 1 ? last_len : (uint32_t)TILE;
            } else {
                const TileDesc d = desc[t];
                t0[h] = d.t0;
                len[h] = d.len;
                seg[h] = d.seg;
                if (EST && (d.seg & kStraddle)) { straddle[h] = true; seg[h] = d.seg & ~kStraddle; }
            }
        }
    }
    if (tid < kRadix)
        for (int h = 0; h < TILES; ++h) s_cur[h][tid] = 0;
    if (EST && tid < TILES) s_ovf[tid] = 0;
    uint32_t *cursor[TILES];
    uint32_t limv[TILES];  // EST: the region limits, loaded now (off the reservation path)
#pragma unroll
    for (int h = 0; h < TILES; ++h) {
        limv[h] = 0;
        // the shard of tile t is (t / 2) % 8, as K1h / K1e count it
        const uint32_t row = (L3 ? ((TILES * pr + h) / 2 % kShards) : seg[h]) * kRadix;
        cursor[h] = cur + row;
        if (EST && tid < kRadix) limv[h] = lim ? lim[row + tid] : ~0u;
    }
    uint32_t k[TILES][ITEMS], r[TILES][ITEMS];
#pragma unroll
    for (int h = 0; h < TILES; ++h) {
        if (EST && !L3 && straddle[h]) {  // a tile across pieces of bucket seg[h] (K12f)
            const TileDesc *pc = pieces + seg[h] * kShards;
            uint64_t pa[kShards];
            uint32_t pv[kShards];
#pragma unroll
            for (uint32_t x = 0; x < kShards; ++x) { pa[x] = pc[x].t0; pv[x] = pc[x].len; }
#pragma unroll
            for (int i = 0; i < ITEMS; ++i) {
                const uint32_t j = (uint32_t)(i * BLOCK) + tid, v = (uint32_t)t0[h] + j;
                uint32_t x = 0;
#pragma unroll
                for (uint32_t q = 1; q < kShards; ++q) x += v >= pv[q];
                k[h][i] = j < len[h] ? in[pa[x] + (v - pv[x])] : 0u;
            }
        } else {
            load_tile<BLOCK, ITEMS, FIN>(in + t0[h] + tid, len[h] == (uint32_t)TILE, len[h], k[h]);
        }
        if (!L3) {
#pragma unroll
            for (int i = 0; i < ITEMS; ++i) k[h][i] ^= flip;
        }
    }
    if (EST && L3 && koff) {  // the offset retry: keys relative to the block's minimum
#pragma unroll
        for (int h = 0; h < TILES; ++h)
#pragma unroll
            for (int i = 0; i < ITEMS; ++i) k[h][i] -= koff;
    }
    if (EST && L3 && sb) {  // the prefix the sampled digits skip must hold for every key
        const uint32_t pfx = ((in[0] ^ kFlip) - koff) >> (32 - sb);
        bool bad = false;
#pragma unroll
        for (int h = 0; h < TILES; ++h)
#pragma unroll
            for (int i = 0; i < ITEMS; ++i)
                bad |= (uint32_t)(i * BLOCK) + tid < len[h] && (k[h][i] >> (32 - sb)) != pfx;
        if (__ballot(bad) && (tid & 63) == 0) atomicOr(ovf, 1u);
    }
    K3_STAMP_WAIT();
    K3_STAMP(1);
    __syncthreads();  // s_cur zeroed
#pragma unroll
    for (int h = 0; h < TILES; ++h)
#pragma unroll
        for (int i = 0; i < ITEMS; ++i)
            if ((uint32_t)(i * BLOCK) + tid < len[h])
                r[h][i] = agg_rank(s_cur[h], (k[h][i] >> shift) & 255u, s_spare);
    __syncthreads();
    K3_STAMP(2);
    uint32_t excl[TILES], pos[TILES], cnt[TILES];
#pragma unroll
    for (int h = 0; h < TILES; ++h) excl[h] = pos[h] = cnt[h] = 0;
    // both tiles on one cursor row (always for K3r: one shard; for K3a when both tiles are in
    // one bucket): ONE reservation of both counts, tile 1's run right behind tile 0's, so the
    // pair writes one run of twice the length -- half the run boundaries, whose lines are
    // otherwise written partly by two workgroups (often on two XCDs)
    const bool merge = TILES == 2 && 2 * pr + 1 < ntile && cursor[0] == cursor[TILES - 1];
    if (tid < kRadix) {
        cnt[0] = s_cur[0][tid];
        cnt[TILES - 1] = s_cur[TILES - 1][tid];
        if (merge) {
            if (cnt[0] + cnt[TILES - 1]) {
                pos[0] = atomicAdd(&cursor[0][tid], cnt[0] + cnt[TILES - 1]);
                pos[TILES - 1] = pos[0] + cnt[0];
            }
        } else {
#pragma unroll
            for (int h = 0; h < TILES; ++h)
                if (cnt[h]) pos[h] = atomicAdd(&cursor[h][tid], cnt[h]);
        }
#pragma unroll
        for (int h = 0; h < TILES; ++h) {
            const uint32_t c = cnt[h];
            const uint32_t v = wave_incl_add(c);
            if (lane == 63) s_wsum[h][w] = v;
            excl[h] = v - c;
        }
    }
    K3_STAMP_WAIT();
    K3_STAMP(3);
    __syncthreads();
    if (tid < kRadix) {
#pragma unroll
        for (int h = 0; h < TILES; ++h) {
            for (uint32_t ww = 0; ww < w; ++ww) excl[h] += s_wsum[h][ww];
            s_cur[h][tid] = excl[h];
        }
    }
    __syncthreads();
#pragma unroll
    for (int h = 0; h < TILES; ++h)
#pragma unroll
        for (int i = 0; i < ITEMS; ++i)
            if ((uint32_t)(i * BLOCK) + tid < len[h])
                s_keys[h][s_cur[h][(k[h][i] >> shift) & 255u] + r[h][i]] = k[h][i];
    if (tid < kRadix) {
#pragma unroll
        for (int h = 0; h < TILES; ++h) {
            s_off[h][tid] = (uint32_t)((L3 ? bases[tid] : bases[seg[h]]) + pos[h]) - excl[h];
            if (EST && cnt[h] && (uint64_t)pos[h] + cnt[h] > limv[h]) {
                atomicOr(ovf, 1u);
                s_ovf[h] = 1;  // the block is re-sorted on the exact plan: the tile goes to dump
            }
        }
    }
    __syncthreads();
    K3_STAMP(4);
#pragma unroll
    for (int h = 0; h < TILES; ++h) {
        OT *o = out;
        bool to_dump = false;
        if (EST && s_ovf[h]) { o = dump; to_dump = true; }
#pragma unroll
        for (int i = 0; i < ITEMS; ++i) {
            const uint32_t j = (uint32_t)(i * BLOCK) + tid;
            if (j < len[h]) {
                const uint32_t key = s_keys[h][j];
                const uint32_t at = to_dump ? j : s_off[h][(key >> shift) & 255u] + j;
                o[at] = (OT)key;
            }
        }
    }
    K3_STAMP_WAIT();
    K3_STAMP(5);
}

// Stable wave-level rank of one round (64 keys, lane order = key order) against the wave's
// running digit counters wc[256] (u32): returns #earlier keys of the wave with this digit.
//   ATOMIC: one ds_add_rtn_u32 per lane.  The MI355X LDS serializes lanes of one instruction
//           that hit the same address in ascending lane order, so the returned counts are the
//           stable ranks (measured: tools/lds_order.hip; re-checked by gsort_create, which
//           selects BALLOT if the check fails -- DESIGN.md 5).
//   BALLOT: 8 ballots give each lane the mask of lanes sharing its digit (v_bfe, v_cmp, two
//           v_bitop3 per bit); rank = running count + peers below; 36 VALU per round.
template <bool ATOMIC>
__device__ __forceinline__ uint32_t wave_rank(uint32_t *wc, uint32_t d, bool valid) {
    if (ATOMIC) return valid ? atomicAdd(&wc[d], 1u) : 0u;
    uint32_t plo = ~0u, phi = ~0u;
#pragma unroll
    for (int b = 0; b < 8; ++b) {
        const uint32_t m = (uint32_t)__builtin_amdgcn_sbfe((int32_t)d, b, 1);
        uint64_t bal;
        asm("v_cmp_ne_u32_e64 %0, 0, %1" : "=s"(bal) : "v"(m));
        plo = __builtin_amdgcn_bitop3_b32(plo, (uint32_t)bal, m, 0x90);
        phi = __builtin_amdgcn_bitop3_b32(phi, (uint32_t)(bal >> 32), m, 0x90);
    }
    const uint64_t vm = __ballot(valid);  // invalid lanes neither rank nor count
    plo &= (uint32_t)vm;
    phi &= (uint32_t)(vm >> 32);
    const uint32_t below = __builtin_amdgcn_mbcnt_hi(phi, __builtin_amdgcn_mbcnt_lo(plo, 0u));
    const uint32_t prev = wc[d];
    if (valid) wc[d] = prev + (uint32_t)(__popc(plo) + __popc(phi));  // same from all peers
    return prev + below;
}

// Body of K11: the bucket's keys are in registers (k[i] = key i*BLOCK + threadIdx.x, ordered
// u32, valid below len); sort them on digits 0 .. ndigits-1 in LDS and store them flipped to
// int32 order at dst[0 .. len).  Digit 0 is ranked by block-wide LDS atomics (an LSD sort may
// order equal first digits arbitrarily); every later digit is ranked stably per wave
// (wave_rank) in (wave, round, lane) order over wave-contiguous chunks, then offset by the
// (digit, wave)-major exclusive scan of the per-wave counts.
// Keys past len are neither counted nor placed (a lane-level mask on wave-uniform bounds; a
// padding key per empty slot would put every such lane on one LDS counter, serialized).
// The caller zeroes s_wc[0 .. 255] before its barrier.
// K11's key array: TILE slots, one pad word after every 32 (slot j at word j + j / 32) --
// except the 32 768-key class, whose 1024 threads hold 32 keys + 32 ranks in 128 VGPRs and
// spill with the pad's addressing (children that large are rare; dense blocks make 4096-key
// children at 2^28)
constexpr bool lds_pad(int tile) { return tile < 32768; }
constexpr int lds_slots(int tile) { return lds_pad(tile) ? tile + tile / 32 : tile; }

// STORE16: dst holds u16 -- the sorted keys' low 16 bits are stored there (no flip): the
// distributed sender's boundary groups, sorted in place in the packed send buffer.
template <int BLOCK, int ITEMS, bool ATOMIC, bool STORE16 = false>
__device__ __forceinline__ void sort_bucket(uint32_t (&k)[ITEMS], uint32_t len, int ndigits,
                                            uint32_t *__restrict__ dst, uint32_t *s_a,
                                            uint32_t *s_wc, uint32_t koff = 0) {
    constexpr int WAVES = BLOCK / 64;
    constexpr int TILE = BLOCK * ITEMS;
    static_assert(TILE <= 65536, "ranks fit 16 bits");
    static_assert(BLOCK >= kRadix, "one thread per digit in the scans");
    // the digit scans run while every key is in registers, so their 4 wave sums borrow the
    // tail of s_a
    uint32_t *s_wsum = s_a + TILE - kRadix / 64;
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    uint32_t *cnt = s_wc;  // digit 0: block-wide counters, then digit starts
    // slot j of the key array at word j + j / 32: in a dense block (sorted / reversed input,
    // keys in steps of 16: every child holds 16 digit-0 values of 256 keys each) a digit's run
    // starts 256 slots after the previous digit's, so without the pad word the 32 lanes of a
    // scatter all land on one bank (reversed 2^28 keys: K11e 1.13 -> 0.49 ms, uniform +1 %,
    // profiles/r04_ab_k11_pad_lds.txt); sequential reads of 32 aligned slots stay on 32 banks
    auto at = [](uint32_t j) constexpr -> uint32_t { return lds_pad(TILE) ? j + (j >> 5) : j; };
    // keys of item i are valid for tid < lim(i) (a wave-uniform bound)
    auto lim = [&](int i) -> uint32_t {
        return len > (uint32_t)(i * BLOCK) ? len - (uint32_t)(i * BLOCK) : 0u;
    };

    auto block_scan = [&](uint32_t c) -> uint32_t {  // tid < 256: exclusive scan over digits
        const uint32_t v = wave_incl_add(c);  // DPP: no LDS-crossbar op per step
        if (lane == 63) s_wsum[w] = v;
        return v - c;
    };

    // digit 0: unstable counting sort into s_a
    {
        uint32_t r[ITEMS];
#pragma unroll
        for (int i = 0; i < ITEMS; ++i)
            if ((uint32_t)tid < lim(i)) r[i] = atomicAdd(&cnt[k[i] & 255u], 1u);
        __syncthreads();
        uint32_t excl = 0;
        if (tid < kRadix) excl = block_scan(cnt[tid]);
        __syncthreads();
        if (tid < kRadix) {
            for (int ww = 0; ww < w; ++ww) excl += s_wsum[ww];
            cnt[tid] = excl;
        }
        __syncthreads();
        // every digit start read before any key is written, and with no predicate (a slot past
        // len reads some start, harmlessly; its write below stays masked): interleaved, or each
        // read inside its own masked block, every write waited for its own read -- an LDS
        // round trip per key-slot (the compiler cannot move a read of cnt above a write to s_a;
        // K11e class 2 -1.5 %, profiles/r06_ab_batched_lds_reads.txt).  Not in the 32 768-key
        // class, whose 128 VGPRs then spill.
        if constexpr (lds_pad(TILE)) {
#pragma unroll
            for (int i = 0; i < ITEMS; ++i) r[i] += cnt[k[i] & 255u];
#pragma unroll
            for (int i = 0; i < ITEMS; ++i)
                if ((uint32_t)tid < lim(i)) s_a[at(r[i])] = k[i];
        } else {
#pragma unroll
            for (int i = 0; i < ITEMS; ++i)
                if ((uint32_t)tid < lim(i)) s_a[at(cnt[k[i] & 255u] + r[i])] = k[i];
        }
        __syncthreads();
    }

    // digits 1 .. ndigits-1: stable, wave-chunked (wave w owns [w*64*R, (w+1)*64*R))
    const uint32_t R = (len + 64 * WAVES - 1) / (64 * WAVES);
    for (int p = 1; p < ndigits; ++p) {
        const int shift = 8 * p;
        uint32_t *wc = s_wc + w * kRadix;
#pragma unroll
        for (int j = 0; j < kRadix / 64; ++j) wc[j * 64 + lane] = 0;
        const uint32_t base = (uint32_t)w * 64 * R;  // wave-uniform
        const uint32_t wlen = len > base ? len - base : 0u;  // keys of this wave's chunk
        // base is a multiple of 64: slot base + i * 64 + lane sits at at(base + lane) + i * at(64)
        const uint32_t *pa = s_a + at(base + lane);
#pragma unroll
        for (int i = 0; i < ITEMS; ++i)
            if ((uint32_t)i < R && (uint32_t)(i * 64 + lane) < wlen)
                k[i] = pa[i * at(64)];
        __syncthreads();
        uint32_t rk[ITEMS];
#pragma unroll
        for (int i = 0; i < ITEMS; ++i)
            if ((uint32_t)i < R)
                rk[i] = wave_rank<ATOMIC>(wc, (k[i] >> shift) & 255u, (uint32_t)(i * 64 + lane) < wlen);
        __syncthreads();
        uint32_t tcount = 0, excl = 0;
        if (tid < kRadix) {
#pragma unroll
            for (int ww = 0; ww < WAVES; ++ww) tcount += s_wc[ww * kRadix + tid];
            excl = block_scan(tcount);
        }
        __syncthreads();
        if (tid < kRadix) {
            uint32_t off = excl;
            for (int ww = 0; ww < w; ++ww) off += s_wsum[ww];
#pragma unroll
            for (int ww = 0; ww < WAVES; ++ww) {
                const uint32_t cw = s_wc[ww * kRadix + tid];
                s_wc[ww * kRadix + tid] = off;
                off += cw;
            }
        }
        __syncthreads();
        if constexpr (lds_pad(TILE)) {
#pragma unroll
            for (int i = 0; i < ITEMS; ++i)  // (starts first, unpredicated, then the keys: as digit 0)
                rk[i] += wc[(k[i] >> shift) & 255u];
#pragma unroll
            for (int i = 0; i < ITEMS; ++i)
                if ((uint32_t)i < R && (uint32_t)(i * 64 + lane) < wlen) s_a[at(rk[i])] = k[i];
        } else {
#pragma unroll
            for (int i = 0; i < ITEMS; ++i)
                if ((uint32_t)i < R && (uint32_t)(i * 64 + lane) < wlen)
                    s_a[at(wc[(k[i] >> shift) & 255u] + rk[i])] = k[i];
        }
        __syncthreads();
    }
    const __amdgpu_buffer_rsrc_t rs = bucket_rsrc(dst, len * (STORE16 ? 2u : 4u));  // stores past len dropped
    // the bucket is one contiguous run of out: nontemporal stores for the 9216-key classes and
    // up (K11e class 2: 472 -> 452-462 us; the 4608-key class measured 113 -> 115 us with them,
    // its runs' partial end lines then miss the neighbours' in L2; K3r / K3a's scattered digit
    // runs doubled -- profiles/r04_ab_nt_stores.txt)
    constexpr bool kNtFinal = TILE > 4608;
    static_assert(BLOCK % 32 == 0, "slot i * BLOCK + tid at at(tid) + i * at(BLOCK)");
    const uint32_t *fa = s_a + at((uint32_t)tid);
#pragma unroll
    for (int i = 0; i < ITEMS; ++i) {
        const uint32_t j = (uint32_t)(i * BLOCK + tid);
        if (STORE16)
            __builtin_amdgcn_raw_buffer_store_b16((uint16_t)fa[i * at(BLOCK)], rs, (int)(j * 2u), 0, 0);
        else
            __builtin_amdgcn_raw_buffer_store_b32((fa[i * at(BLOCK)] + koff) ^ kFlip, rs,
                                                  (int)(j * 4u), 0, kNtFinal ? 2 : 0);  // (2: nt)
    }
}

// sort_bucket for keys that share their top 16 bits (top): the low halves travel two to a
// register (kp[q] = key 2q | key 2q+1 << 16, ranks likewise) and one to an LDS slot, the two
// digits below top are sorted as in sort_bucket, and top | key is stored flipped at dst.  Half
// the VGPRs and LDS bytes of sort_bucket: a 16 896-key tile (K11g class 3) then fits three
// workgroups per CU instead of two (112 -> <= 80 VGPRs, 76 -> 44 KiB).

template <int BLOCK, int ITEMS, bool ATOMIC>
__device__ __forceinline__ void sort_bucket16(uint32_t (&kp)[(ITEMS + 1) / 2], uint32_t len,
                                              uint32_t top, uint32_t *__restrict__ dst,
                                              uint16_t *s_a, uint32_t *s_wc, int ndigits = 2,
                                              uint32_t koff = 0) {
    using PK = Pack16<BLOCK, ITEMS>;
    constexpr int NP = PK::NP;
    constexpr int WAVES = BLOCK / 64;
    constexpr int TILE = BLOCK * ITEMS;
    static_assert(TILE <= 65536 && TILE % 2 == 0, "ranks fit 16 bits; the wave sums' words align");
    static_assert(BLOCK >= kRadix, "one thread per digit in the scans");
    uint32_t *s_wsum = reinterpret_cast<uint32_t *>(s_a + TILE - 2 * (kRadix / 64));
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    uint32_t *cnt = s_wc;
    auto at = [](uint32_t j) constexpr -> uint32_t { return j + (j >> 5); };  // sort_bucket's pad
    auto lim = [&](int i) -> uint32_t {
        return len > (uint32_t)(i * BLOCK) ? len - (uint32_t)(i * BLOCK) : 0u;
    };
    auto block_scan = [&](uint32_t c) -> uint32_t {
        const uint32_t v = wave_incl_add(c);
        if (lane == 63) s_wsum[w] = v;
        return v - c;
    };
    PK::pin(kp);
    uint32_t rp[NP];
#pragma unroll
    for (int q = 0; q < NP; ++q) rp[q] = 0;
    // digit 0: unstable counting sort into s_a
#pragma unroll
    for (int i = 0; i < ITEMS; ++i)
        if ((uint32_t)tid < lim(i)) PK::set(rp, i, atomicAdd(&cnt[PK::get(kp, i) & 255u], 1u));
    PK::pin(rp);
    __syncthreads();
    {
        uint32_t excl = 0;
        if (tid < kRadix) excl = block_scan(cnt[tid]);
        __syncthreads();
        if (tid < kRadix) {
            for (int ww = 0; ww < w; ++ww) excl += s_wsum[ww];
            cnt[tid] = excl;
        }
        __syncthreads();
    }
#pragma unroll
    for (int i = 0; i < ITEMS; ++i)  // (interleaved: sort_bucket's batched start reads measured
        if ((uint32_t)tid < lim(i)) {  // +5 % on this body, profiles/r06_ab_batched_lds_reads.txt)
            const uint32_t x = PK::get(kp, i);
            s_a[at(cnt[x & 255u] + PK::get(rp, i))] = (uint16_t)x;
        }
    __syncthreads();
    // digit 1 (ndigits == 2): stable, wave-chunked (wave w owns [w*64*R, (w+1)*64*R))
    if (ndigits > 1) {
    const uint32_t R = (len + 64 * WAVES - 1) / (64 * WAVES);
    uint32_t *wc = s_wc + w * kRadix;
#pragma unroll
    for (int j = 0; j < kRadix / 64; ++j) wc[j * 64 + lane] = 0;
    const uint32_t base = (uint32_t)w * 64 * R;
    const uint32_t wlen = len > base ? len - base : 0u;
    const uint16_t *pa = s_a + at(base + lane);
#pragma unroll
    for (int i = 0; i < ITEMS; ++i)
        if ((uint32_t)i < R && (uint32_t)(i * 64 + lane) < wlen) PK::set(kp, i, pa[i * at(64)]);
    PK::pin(kp);
    __syncthreads();
#pragma unroll
    for (int i = 0; i < ITEMS; ++i)
        if ((uint32_t)i < R)
            PK::set(rp, i, wave_rank<ATOMIC>(wc, PK::get(kp, i) >> 8,
                                             (uint32_t)(i * 64 + lane) < wlen));
    PK::pin(rp);
    __syncthreads();
    {
        uint32_t tcount = 0, excl = 0;
        if (tid < kRadix) {
#pragma unroll
            for (int ww = 0; ww < WAVES; ++ww) tcount += s_wc[ww * kRadix + tid];
            excl = block_scan(tcount);
        }
        __syncthreads();
        if (tid < kRadix) {
            uint32_t off = excl;
            for (int ww = 0; ww < w; ++ww) off += s_wsum[ww];
#pragma unroll
            for (int ww = 0; ww < WAVES; ++ww) {
                const uint32_t cw = s_wc[ww * kRadix + tid];
                s_wc[ww * kRadix + tid] = off;
                off += cw;
            }
        }
        __syncthreads();
    }
#pragma unroll
    for (int i = 0; i < ITEMS; ++i)
        if ((uint32_t)i < R && (uint32_t)(i * 64 + lane) < wlen) {
            const uint32_t x = PK::get(kp, i);
            s_a[at(wc[x >> 8] + PK::get(rp, i))] = (uint16_t)x;
        }
    __syncthreads();
    }
    const __amdgpu_buffer_rsrc_t rs = bucket_rsrc(dst, len * 4u);  // stores past len dropped
    constexpr bool kNtFinal = TILE > 4608;  // (as sort_bucket)
    static_assert(BLOCK % 32 == 0, "slot i * BLOCK + tid at at(tid) + i * at(BLOCK)");
    const uint16_t *fa = s_a + at((uint32_t)tid);
#pragma unroll
    for (int i = 0; i < ITEMS; ++i)
        __builtin_amdgcn_raw_buffer_store_b32(((top | fa[i * at(BLOCK)]) + koff) ^ kFlip, rs,
                                              (i * BLOCK + tid) * 4, 0, kNtFinal ? 2 : 0);
}

// K11: sort each listed bucket {start, len} (<= BLOCK * ITEMS keys) of `in` on digits
// 0 .. ndigits-1 in LDS and write it back flipped to int32 order at the same position of out.
template <int BLOCK, int ITEMS, bool FIN, bool ATOMIC>
__global__ __launch_bounds__(BLOCK) void k_local_sort(const uint32_t *__restrict__ in,
                                                      uint32_t *__restrict__ out,
                                                      const unsigned long long *__restrict__ list,
                                                      int ndigits) {
    constexpr int WAVES = BLOCK / 64;
    constexpr int TILE = BLOCK * ITEMS;
    __shared__ uint32_t s_a[lds_slots(TILE)];
    __shared__ uint32_t s_wc[WAVES * kRadix];  // per-wave digit counts, then offsets
    const uint64_t start = list[2 * blockIdx.x];
    const uint64_t e = list[2 * blockIdx.x + 1];  // len | extra digits << 32 (merged children)
    const uint32_t len = (uint32_t)e;
    if (threadIdx.x < kRadix) s_wc[threadIdx.x] = 0;
    uint32_t k[ITEMS];
    load_bucket<BLOCK, ITEMS, FIN>(in + start, len, k);
    __syncthreads();
    sort_bucket<BLOCK, ITEMS, ATOMIC>(k, len, min(ndigits + (int)(e >> 32), 4), out + start, s_a,
                                      s_wc);
}

// Received runs are addressed as recv + offset where a rank's own piece, read in place from its
// send buffer, carries the offset of that buffer from recv (mod 2^64, made on the host from
// integer addresses): the address is formed as an integer, not by pointer arithmetic
// across allocations.
template <typename T>
__device__ __forceinline__ const T *run_ptr(const T *recv, uint64_t off) {
    return reinterpret_cast<const T *>(reinterpret_cast<uintptr_t>(recv) + off * sizeof(T));
}
// A load through a run pointer as a global (not flat) access: the integer-formed address hides
// the address space from the compiler, whose flat loads then keep a 64-bit address pair live
// per load in flight (K11g class 3's one-run path: 84 VGPRs; global: SGPR base + 32-bit offset)
template <typename T>
__device__ __forceinline__ T ld_run(const T *p) {
    return *reinterpret_cast<const __attribute__((address_space(1))) T *>(
        reinterpret_cast<uintptr_t>(p));
}
__device__ __forceinline__ uint4 ld_run(const uint4 *p) {  // (HIP's uint4 is a class type)
    typedef unsigned int v4 __attribute__((ext_vector_type(4)));
    const v4 x = *reinterpret_cast<const __attribute__((address_space(1))) v4 *>(
        reinterpret_cast<uintptr_t>(p));
    return make_uint4(x.x, x.y, x.z, x.w);
}

// K11g (receive side of the distributed sorts): bucket h of the 2^16 top-16-bit buckets of
// the P received sorted runs.  Its keys are the P pieces recv[roff[p] + pos[p][h] ..
// roff[p] + pos[p][h+1]) (int32); they are gathered, sorted on the low 16 bits in LDS and
// stored at out[bstart[h] ..).  List entries are {h, len}.
// A received key in ordered-u32 form: int32 payload (flip), or the low 16 bits of a key whose
// top 16 bits are the bucket h (the packed exchange of the distributed radix).
__device__ __forceinline__ uint32_t recv_key(int32_t x, uint32_t) { return (uint32_t)x ^ kFlip; }
__device__ __forceinline__ uint32_t recv_key(uint16_t x, uint32_t h) { return (h << 16) | x; }

// pieces up to which K11g loads every key straight into registers (a piece lookup of P - 1
// scalar compares per key); more pieces go through an LDS gather first
constexpr int kGatherDirectP = 8;

// K11g's loads of bucket h (entry: first output position dst, len keys) from its P pieces into
// v[i] = key i * BLOCK + tid (past len: the last key again).  P == 1: the one run's bucket
// offsets are the bucket starts, so the keys come straight from the entry (no pos load, no
// piece table, no barrier in front of the loads -- round 6).  P <= kGatherDirectP: every key
// straight into registers through the wave-uniform piece boundaries, all loads in flight.
// Otherwise returns false with the piece table (s_src, s_cum) filled: the caller gathers the
// pieces through LDS.
template <int BLOCK, int ITEMS, typename T>
__device__ __forceinline__ bool gather_direct(const T *recv, const unsigned long long *pos,
                                              const unsigned long long *roff, int P, uint64_t h,
                                              uint64_t dst, uint32_t len, uint64_t *s_src,
                                              uint64_t *s_delta, uint32_t *s_cum, T (&v)[ITEMS]) {
    const int tid = threadIdx.x;
    const uint32_t last = len ? len - 1 : 0u;
    if (P == 1) {
        const T *src = run_ptr(recv, roff[0] + dst);
#pragma unroll
        for (int i = 0; i < ITEMS; ++i) v[i] = ld_run(src + min((uint32_t)(i * BLOCK + tid), last));
        return true;
    }
    if (tid < 64) {  // lane p: piece p; wave scan of the piece lengths (DPP)
        uint64_t a = 0, b = 0;
        if (tid < P) {
            a = pos[(uint64_t)tid * (kBuckets16 + 1) + h];
            b = pos[(uint64_t)tid * (kBuckets16 + 1) + h + 1];
        }
        const uint32_t l = (uint32_t)(b - a);
        const uint32_t vs = wave_incl_add(l);
        if (tid < P) {
            s_src[tid] = roff[tid] + a;
            s_cum[tid] = vs - l;
            s_delta[tid] = roff[tid] + a - (vs - l);  // key j of piece p: recv[delta + j]
        }
        if (tid == P - 1) s_cum[P] = vs;
    }
    __syncthreads();
    if (P > kGatherDirectP) return false;
    // key j lies in piece p(j) = #{q >= 1 : j >= cum[q]} (the boundaries are wave-uniform scalars)
    uint32_t cum[kGatherDirectP];
#pragma unroll
    for (int q = 1; q < kGatherDirectP; ++q)
        cum[q] = q < P ? (uint32_t)__builtin_amdgcn_readfirstlane((int)s_cum[q]) : 0xFFFFFFFFu;
#pragma unroll
    for (int i = 0; i < ITEMS; ++i) {
        const uint32_t j = min((uint32_t)(i * BLOCK + tid), last);
        uint32_t q = 0;
#pragma unroll
        for (int b = 1; b < kGatherDirectP; ++b) q += j >= cum[b] ? 1u : 0u;
        v[i] = ld_run(run_ptr(recv, s_delta[q] + j));
    }
    return true;
}

// The pieces of bucket h into LDS slots 0 .. len (coalesced per piece, 8 loads in flight per
// thread), each key as conv(value).
template <int BLOCK, typename T, typename S, typename F>
__device__ __forceinline__ void gather_lds(const T *recv, int P, const uint64_t *s_src,
                                           const uint32_t *s_cum, S *s_a, F conv) {
    const int tid = threadIdx.x;
#pragma unroll 1
    for (int p = 0; p < P; ++p) {
        const T *src = run_ptr(recv, s_src[p]);
        const uint32_t c0 = s_cum[p], c1 = s_cum[p + 1];
#pragma unroll 1
        for (uint32_t b = c0; b < c1; b += 8 * BLOCK) {
            T v[8];
#pragma unroll
            for (int u = 0; u < 8; ++u) {
                const uint32_t j = b + u * BLOCK + tid;
                v[u] = j < c1 ? ld_run(src + (j - c0)) : T(0);
            }
#pragma unroll
            for (int u = 0; u < 8; ++u) {
                const uint32_t j = b + u * BLOCK + tid;
                if (j < c1) s_a[j] = conv(v[u]);
            }
        }
    }
    __syncthreads();
}

template <int BLOCK, int ITEMS, bool ATOMIC, typename T>
__global__ __launch_bounds__(BLOCK) void k_gather_sort(const T *__restrict__ recv,
                                                       const unsigned long long *__restrict__ pos,
                                                       const unsigned long long *__restrict__ roff,
                                                       int P,
                                                       const unsigned long long *__restrict__ bstart,
                                                       const unsigned long long *__restrict__ list,
                                                       uint32_t *__restrict__ out,
                                                       const uint32_t *__restrict__ ndev,
                                                       uint32_t first) {
    constexpr int WAVES = BLOCK / 64;
    constexpr int TILE = BLOCK * ITEMS;
    constexpr int MAXP = 64;
    // entry first + blockIdx.x; ndev: the list's length read on the device (a launch queued
    // before the host knew it -- the grid is a guess, the blocks past the length return)
    const uint32_t ei = first + blockIdx.x;
    if (ndev && ei >= *ndev) return;
    __shared__ uint32_t s_a[lds_slots(TILE)];
    __shared__ uint32_t s_wc[WAVES * kRadix];
    __shared__ uint64_t s_src[MAXP];  // piece p: first key in recv
    __shared__ uint64_t s_delta[MAXP];
    __shared__ uint32_t s_cum[MAXP + 1];
    const int tid = threadIdx.x;
    const uint64_t e0 = list[2 * ei];  // h | bstart[h] << 16 (k_classify_gather)
    const uint64_t h = e0 & 0xFFFFu, dst = e0 >> 16;
    const uint32_t len = (uint32_t)list[2 * ei + 1];
    if (tid < kRadix) s_wc[tid] = 0;
    uint32_t k[ITEMS];
    T v[ITEMS];
    if (gather_direct<BLOCK, ITEMS>(recv, pos, roff, P, h, dst, len, s_src, s_delta, s_cum, v)) {
#pragma unroll
        for (int i = 0; i < ITEMS; ++i) k[i] = recv_key(v[i], (uint32_t)h);
    } else {
        gather_lds<BLOCK>(recv, P, s_src, s_cum, s_a,
                          [&](T x) { return recv_key(x, (uint32_t)h); });
#pragma unroll
        for (int i = 0; i < ITEMS; ++i) {
            const uint32_t j = (uint32_t)(i * BLOCK + tid);
            k[i] = j < len ? s_a[j] : 0u;
        }
    }
    __syncthreads();
    sort_bucket<BLOCK, ITEMS, ATOMIC>(k, len, 2, out + dst, s_a, s_wc);
    (void)bstart;
}

// K11g over packed receive buckets (u16 low halves, the bucket's top 16 bits implied) with the
// two-to-a-register body sort_bucket16 -- the 16 896-key class (P = 2's 16 384-key buckets).
template <int BLOCK, int ITEMS, bool ATOMIC>
__global__ __launch_bounds__(BLOCK) void k_gather_sort16(const uint16_t *__restrict__ recv,
                                                         const unsigned long long *__restrict__ pos,
                                                         const unsigned long long *__restrict__ roff,
                                                         int P,
                                                         const unsigned long long *__restrict__ list,
                                                         uint32_t *__restrict__ out,
                                                         const uint32_t *__restrict__ ndev,
                                                         uint32_t first) {
    constexpr int WAVES = BLOCK / 64;
    constexpr int TILE = BLOCK * ITEMS;
    constexpr int MAXP = 64;
    constexpr int NP = (ITEMS + 1) / 2;
    const uint32_t ei = first + blockIdx.x;
    if (ndev && ei >= *ndev) return;
    __shared__ __attribute__((aligned(16))) uint16_t s_a[(lds_slots(TILE) + 1) & ~1];  // (s_wsum: u32 words in it)
    __shared__ uint32_t s_wc[WAVES * kRadix];
    __shared__ uint64_t s_src[MAXP];
    __shared__ uint64_t s_delta[MAXP];
    __shared__ uint32_t s_cum[MAXP + 1];
    const int tid = threadIdx.x;
    const uint64_t e0 = list[2 * ei];
    const uint64_t h = e0 & 0xFFFFu, dst = e0 >> 16;
    const uint32_t len = (uint32_t)list[2 * ei + 1];
    if (tid < kRadix) s_wc[tid] = 0;
    uint32_t kp[NP];
    {
        uint16_t v[ITEMS];
        if (gather_direct<BLOCK, ITEMS>(recv, pos, roff, P, h, dst, len, s_src, s_delta, s_cum, v)) {
#pragma unroll
            for (int q = 0; q < NP; ++q)
                kp[q] = (uint32_t)v[2 * q] | (2 * q + 1 < ITEMS ? (uint32_t)v[2 * q + 1] << 16 : 0u);
        } else {
            gather_lds<BLOCK>(recv, P, s_src, s_cum, s_a, [](uint16_t x) { return x; });
#pragma unroll
            for (int q = 0; q < NP; ++q) {
                const uint32_t j0 = (uint32_t)(2 * q * BLOCK + tid), j1 = j0 + BLOCK;
                kp[q] = (j0 < len ? (uint32_t)s_a[j0] : 0u) |
                        (2 * q + 1 < ITEMS && j1 < len ? (uint32_t)s_a[j1] << 16 : 0u);
            }
        }
    }
    __syncthreads();
    sort_bucket16<BLOCK, ITEMS, ATOMIC>(kp, len, (uint32_t)h << 16, out + dst, s_a, s_wc);
}

// Receive side, K11g bookkeeping.  pos[p][h] = keys of sorted run p whose top 16 bits (ordered
// u32) are < h, h = 0 .. 2^16 (binary search; one thread per (p, h)).
__global__ __launch_bounds__(256) void k_run_bounds(const int32_t *__restrict__ recv,
                                                    const unsigned long long *__restrict__ roff,
                                                    const unsigned long long *__restrict__ rlen,
                                                    int P, unsigned long long *__restrict__ pos) {
    const uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= (uint64_t)P * (kBuckets16 + 1)) return;
    const uint32_t p = (uint32_t)(i / (kBuckets16 + 1)), h = (uint32_t)(i % (kBuckets16 + 1));
    const int32_t *a = run_ptr(recv, roff[p]);
    const uint64_t x = (uint64_t)h << 16;
    uint64_t lo = 0, hi = rlen[p];
    while (lo < hi) {
        const uint64_t mid = (lo + hi) >> 1;
        if ((uint64_t)((uint32_t)ld_run(a + mid) ^ kFlip) < x) lo = mid + 1; else hi = mid;
    }
    pos[i] = lo;
}

// bsize[h] = sum_p pos[p][h+1] - pos[p][h] (one thread per bucket); then bstart = exclusive
// scan of bsize (one 1024-thread block, 64 buckets per thread); then the buckets are
// classified (one 256-thread block per 256 buckets, classify_block): the next-level list gets
// {bstart, len} (segments), the K11g lists get {h, len}.
__global__ __launch_bounds__(256) void k_bucket_sizes(const unsigned long long *__restrict__ pos,
                                                      int P,
                                                      unsigned long long *__restrict__ bsize) {
    const uint32_t h = blockIdx.x * 256 + threadIdx.x;
    unsigned long long c = 0;
    for (int p = 0; p < P; ++p)
        c += pos[(uint64_t)p * (kBuckets16 + 1) + h + 1] - pos[(uint64_t)p * (kBuckets16 + 1) + h];
    bsize[h] = c;
}

__global__ __launch_bounds__(kRadix) void k_classify_gather(
    const unsigned long long *__restrict__ bsize, const unsigned long long *__restrict__ bstart,
    WorkLists wl, uint32_t h0, uint32_t h1) {
    const uint32_t h = blockIdx.x * kRadix + threadIdx.x;
    const uint64_t b0 = bstart[h];
    const uint64_t len = h >= h0 && h < h1 ? (bsize ? bsize[h] : bstart[h + 1] - b0) : 0ull;
    // {bucket id | its output start << 16, len}: K11g classes, and list 0 (K18 or, past
    // kHxMax, the MSD levels).  The start rides in the entry so that K11g reaches its output
    // (and, at P = 1, its keys: the one run's offset of bucket h IS bstart[h]) without a
    // dependent load behind the entry's (round 6)
    classify_block((uint64_t)h | (b0 << 16), len, wl);
}

// K18 (receive side, buckets of kLocalMax < len <= kHxMax keys): a counting sort of the
// bucket's low 16 bits -- keys carry no payload, so the output is written straight from the
// counts.  Two halves of the value range, 32768 u32 counters in LDS each (one pad word per 32
// so that a thread's 32 consecutive counters sit in distinct banks during the scan):
// histogram the P pieces, scan, then bin b writes its count copies of key (h, b) at the
// running position; consecutive lanes take consecutive bins, so the stores coalesce.
template <typename T>
__global__ __launch_bounds__(1024) void k_hist_expand(const T *__restrict__ recv,
                                                      const unsigned long long *__restrict__ pos,
                                                      const unsigned long long *__restrict__ roff,
                                                      int P,
                                                      const unsigned long long *__restrict__ bstart,
                                                      const unsigned long long *__restrict__ list,
                                                      uint32_t *__restrict__ out) {
    constexpr uint32_t HB = 32768, NT = 1024, PER = HB / NT;
    __shared__ uint32_t s_c[HB + HB / 32];
    __shared__ uint64_t s_src[64];
    __shared__ uint32_t s_len[64];
    __shared__ uint32_t s_w[NT / 64];
    const uint32_t tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const uint32_t h = (uint32_t)list[2 * blockIdx.x] & 0xFFFFu;  // (bstart[h] above bit 16)
    if ((int)tid < P) {
        const uint64_t a = pos[(uint64_t)tid * (kBuckets16 + 1) + h];
        const uint64_t b = pos[(uint64_t)tid * (kBuckets16 + 1) + h + 1];
        s_src[tid] = roff[tid] + a;
        s_len[tid] = (uint32_t)(b - a);
    }
    uint32_t *dst = out + bstart[h];
    uint32_t base = 0;  // keys of the lower half
    auto pad = [](uint32_t b) { return b + (b >> 5); };
    for (uint32_t half = 0; half < 2; ++half) {
        for (uint32_t i = tid; i < HB + HB / 32; i += NT) s_c[i] = 0;
        __syncthreads();
#pragma unroll 1
        for (int p = 0; p < P; ++p) {
            const T *src = run_ptr(recv, s_src[p]);
            const uint32_t np = s_len[p];
#pragma unroll 1
            for (uint32_t j0 = 0; j0 < np; j0 += 8 * NT) {
                uint32_t v[8];
#pragma unroll
                for (int u = 0; u < 8; ++u) {
                    const uint32_t j = j0 + u * NT + tid;
                    v[u] = j < np ? (recv_key(ld_run(src + j), h) & 0xFFFFu) : 0x10000u;
                }
#pragma unroll
                for (int u = 0; u < 8; ++u)
                    if ((v[u] >> 15) == half) atomicAdd(&s_c[pad(v[u] & (HB - 1))], 1u);
            }
        }
        __syncthreads();
        // exclusive scan: thread t owns bins [PER t, PER (t + 1))
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
        // expand: bin b = j * NT + tid holds [s_c[b], s_c[b + 1]) (the last: base + total)
        const uint32_t end_all = base + total;
#pragma unroll 1
        for (uint32_t j = 0; j < PER; ++j) {
            const uint32_t b = j * NT + tid;
            const uint32_t st = s_c[pad(b)];
            const uint32_t en = b + 1 < HB ? s_c[pad(b + 1)] : end_all;
            const uint32_t key = ((h << 16) | (half << 15) | b) ^ kFlip;
            for (uint32_t q = st; q < en; ++q) dst[q] = key;
        }
        base = end_all;
        __syncthreads();
    }
}

// ---- K18c: one-read counting sort of a receive bucket's low 16 bits -----------------------
// Bin counters: 65 536 u16 halves in 32 768 words (128 KiB).  A half that wraps (>= 65 536
// copies of one value: buckets past 65 535 keys only) is seen by the one lane whose returning
// atomic read 0xffff; it records the correction (bin, delta): +65 536 for the wrapped bin,
// and for a low half the carry into its neighbour (-1, and +65 536 more if that carry wrapped
// the high half too).  kHxMax bounds the wraps: 3 entries per 65 536 keys at most.
constexpr uint32_t kCxWrapMax = 64;
static_assert(3 * (kHxMax >> 16) <= kCxWrapMax, "K18c wrap list too small for kHxMax");

template <bool WRAP, int CB = 16>
__device__ __forceinline__ void cx_count(uint32_t *s_h, uint32_t v, uint32_t *s_nw,
                                         uint32_t *s_wb, int32_t *s_wd) {
    if (CB == 8) {  // u8 bins: word v >> 2, byte v & 3 (a wrap is found by the total, not here)
        atomicAdd(s_h + (v >> 2), 1u << ((v & 3u) << 3));
        return;
    }
    // word v >> 1 (byte address (v << 1) & ~3), half v & 1: add 1 or 0x10000
    uint32_t *a = reinterpret_cast<uint32_t *>(reinterpret_cast<char *>(s_h) + ((v << 1) & 0x1FFFCu));
    const uint32_t inc = (v & 1u) * 0xFFFFu + 1u;  // one v_mad_u32_u24
    if (!WRAP) {
        atomicAdd(a, inc);
        return;
    }
    const uint32_t o = atomicAdd(a, inc);
    const uint32_t sh = (v & 1u) << 4;
    if (((o >> sh) & 0xFFFFu) == 0xFFFFu) {
        const bool lo = sh == 0, both = lo && (o >> 16) == 0xFFFFu;
        const uint32_t e = atomicAdd(s_nw, lo ? (both ? 3u : 2u) : 1u);
        if (e < kCxWrapMax) { s_wb[e] = v; s_wd[e] = 65536; }
        if (lo && e + 1 < kCxWrapMax) { s_wb[e + 1] = v + 1; s_wd[e + 1] = -1; }
        if (both && e + 2 < kCxWrapMax) { s_wb[e + 2] = v + 1; s_wd[e + 2] = 65536; }
    }
}

template <bool WRAP, typename T>
__device__ __forceinline__ void cx_count_piece(const T *src, uint32_t np, uint32_t *s_h,
                                               uint32_t *s_nw, uint32_t *s_wb, int32_t *s_wd) {
    constexpr uint32_t NT = 1024, E = 16 / sizeof(T), U = 8;
    const uint32_t tid = threadIdx.x;
    // elements before the first 16-B boundary, whole 16-B vectors, the rest
    const uint32_t mis = (uint32_t)((reinterpret_cast<uintptr_t>(src) / sizeof(T)) & (E - 1));
    const uint32_t head = min(mis ? E - mis : 0u, np);
    const uint32_t nv = (np - head) / E, t0 = head + nv * E;
    if (tid < head) cx_count<WRAP>(s_h, (uint32_t)src[tid] & 0xFFFFu, s_nw, s_wb, s_wd);
    if (tid < np - t0) cx_count<WRAP>(s_h, (uint32_t)src[t0 + tid] & 0xFFFFu, s_nw, s_wb, s_wd);
    if (nv == 0) return;
    const uint4 *vs = reinterpret_cast<const uint4 *>(src + head);
#pragma unroll 1
    for (uint32_t v0 = 0; v0 < nv; v0 += U * NT) {
        uint4 x[U];
#pragma unroll
        for (uint32_t u = 0; u < U; ++u) x[u] = vs[min(v0 + u * NT + tid, nv - 1)];  // all in flight
#pragma unroll
        for (uint32_t u = 0; u < U; ++u) {
            if (v0 + u * NT + tid >= nv) continue;
            const uint32_t w4[4] = {x[u].x, x[u].y, x[u].z, x[u].w};
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                if (sizeof(T) == 2) {
                    cx_count<WRAP>(s_h, w4[q] & 0xFFFFu, s_nw, s_wb, s_wd);
                    cx_count<WRAP>(s_h, w4[q] >> 16, s_nw, s_wb, s_wd);
                } else {
                    cx_count<WRAP>(s_h, w4[q] & 0xFFFFu, s_nw, s_wb, s_wd);
                }
            }
        }
    }
}

// K18c (receive side; list {h, len}): the bucket's keys are the P pieces
// recv[roff[p] + pos[p][h] .. roff[p] + pos[p][h + 1]); keys carry no payload, so sorting them
// is counting them.  Persistent: one 1024-thread workgroup per CU walks buckets
// blockIdx.x, + gridDim.x, ... (the 128 KiB of bin counters allow one per CU), and the next
// bucket's first 8 x 16 B per thread are loaded while this one is expanded -- so its reads
// overlap this one's stores and VALU work instead of following them.  Per bucket:
// 1) the 65 536 packed u16 bin counters count the prefetched vectors, any vectors past them and
//    the pieces' unaligned heads / tails (one LDS atomic per key);
// 2) wave w owns bins [4096 w, +4096) (u8 bins, 8 waves: [8192 w, +8192), 32 chunks; lane L
//    one word of 4 bins per chunk) (16 chunks of 256 bins, lane L the 4 bins of words
//    128 j + 2 L, +1); the waves' totals are scanned into their output runs;
// 3) each wave writes its run in windows of 256 slots aligned to 16 B in out: the bins of every
//    chunk starting in the window mark their first slot with their key (LDS; chunks streamed
//    through registers), lane L reads slots 4 L .. 4 L + 3 (ds_read_b128), a running max inside
//    the lane + a wave max-scan (DPP) give every slot its key (keys grow with the slot; 0 is
//    both "no mark" and the smallest key), and the lane stores 4 keys with ONE 16-B store.  A
//    frequent value is windows without marks (the key carried over).
// 2 B read (16-bit packed pieces; 4 B for int32 pieces) + 4 B written per key.
template <typename T>
struct CxTable {  // one bucket's pieces (LDS, double-buffered)
    uint64_t src[64];    // piece p's first element in recv (elements, mod 2^64)
    uint32_t len[64];    // its elements
    uint32_t head[64];   // elements before its first 16-B boundary
    uint32_t cumv[65];   // 16-B vectors of the pieces before p (vector space)
    uint64_t dst;        // bstart[h]
    uint32_t h, keys;    // bucket, keys (0: no bucket)
};

// (ent: the bucket's list entry {h, len}, null past the lists' end)
template <typename T>
__device__ __forceinline__ void cx_fill_table(CxTable<T> &t, const T *recv,
                                              const unsigned long long *pos,
                                              const unsigned long long *roff, int P,
                                              const unsigned long long *bstart,
                                              const unsigned long long *ent) {  // wave 0 only
    constexpr uint32_t E = 16 / sizeof(T);
    const uint32_t lane = threadIdx.x & 63;
    if (!ent) {
        if (lane == 0) t.keys = 0;
        return;
    }
    const uint64_t e0 = ld_run(ent), e1 = ld_run(ent + 1);  // (global loads: ent is a joined-list pointer)
    const uint32_t h = (uint32_t)e0 & 0xFFFFu;  // (bstart[h] rides above bit 16)
    // a bucket past kHxMax is not K18c's: left as an empty one (recv_sort counts it in place,
    // giant_sort) -- its bins' u16 counts could not hold it
    const bool giant = (uint32_t)e1 > (uint32_t)kHxMax;
    uint64_t a = 0, b = 0, src = 0;
    if ((int)lane < P && !giant) {
        a = pos[(uint64_t)lane * (kBuckets16 + 1) + h];
        b = pos[(uint64_t)lane * (kBuckets16 + 1) + h + 1];
        src = roff[lane] + a;
    }
    const uint32_t n = (uint32_t)(b - a);
    const uint32_t mis = (uint32_t)((reinterpret_cast<uintptr_t>(run_ptr(recv, src)) / sizeof(T)) & (E - 1));
    const uint32_t hd = min(mis ? E - mis : 0u, n);
    const uint32_t nv = (n - hd) / E;
    const uint32_t x = wave_incl_add(nv);
    if ((int)lane < P) {
        t.src[lane] = src;
        t.len[lane] = n;
        t.head[lane] = hd;
        t.cumv[lane] = x - nv;
    }
    if ((int)lane == P - 1) t.cumv[P] = x;
    if (lane == 0) {
        t.h = h;
        t.keys = giant ? 0u : (uint32_t)e1;
        t.dst = bstart[h];
    }
}

// The sampled plan's children past kLocalMax (K12g's list 0, entries {src in Y | the child's top
// 16 bits << 40, dst | len << 40}, as K11e's): one piece each, read from Y.
template <typename T>
__device__ __forceinline__ void cx_fill_table_est(CxTable<T> &t, const T *y,
                                                  const unsigned long long *ent) {  // wave 0 only
    constexpr uint32_t E = 16 / sizeof(T);
    const uint32_t lane = threadIdx.x & 63;
    if (!ent) {
        if (lane == 0) t.keys = 0;
        return;
    }
    if (lane == 0) {
        const uint64_t sw = ld_run(ent), e = ld_run(ent + 1);
        const uint64_t src = sw & ((1ull << 40) - 1);
        const uint32_t n = (uint32_t)(e >> 40);
        const uint32_t mis = (uint32_t)((reinterpret_cast<uintptr_t>(y + src) / sizeof(T)) & (E - 1));
        const uint32_t hd = min(mis ? E - mis : 0u, n);
        t.src[0] = src;
        t.len[0] = n;
        t.head[0] = hd;
        t.cumv[0] = 0;
        t.cumv[1] = (n - hd) / E;
        t.h = (uint32_t)(sw >> 40);
        t.keys = n;
        t.dst = e & ((1ull << 40) - 1);
    }
}

// piece of vector g: the last p with cumv[p] <= g (binary search, P <= 64)
template <typename T>
__device__ __forceinline__ uint32_t cx_piece(const CxTable<T> &t, int P, uint32_t g) {
    uint32_t lo = 0, hi = (uint32_t)P;
    while (hi - lo > 1) {
        const uint32_t mid = (lo + hi) >> 1;
        if (t.cumv[mid] <= g) lo = mid; else hi = mid;
    }
    return lo;
}

template <typename T>
__device__ __forceinline__ const uint4 *cx_vec(const T *recv, const CxTable<T> &t, int P,
                                               uint32_t g) {
    const uint32_t p = cx_piece(t, P, g);
    return reinterpret_cast<const uint4 *>(run_ptr(recv, t.src[p] + t.head[p])) + (g - t.cumv[p]);
}

template <bool WRAP, typename T, int CB = 16>
__device__ __forceinline__ void cx_count_vec(uint32_t *s_h, const uint4 &x, uint32_t *s_nw,
                                             uint32_t *s_wb, int32_t *s_wd) {
    const uint32_t w4[4] = {x.x, x.y, x.z, x.w};
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        cx_count<WRAP, CB>(s_h, w4[q] & 0xFFFFu, s_nw, s_wb, s_wd);
        if (sizeof(T) == 2) cx_count<WRAP, CB>(s_h, w4[q] >> 16, s_nw, s_wb, s_wd);
    }
}

template <bool WRAP, typename T, uint32_t PF, uint32_t NT = 1024, int CB = 16>
__device__ __forceinline__ void cx_count_bucket(const T *recv, const CxTable<T> &t, int P,
                                                const uint4 (&x)[PF], uint32_t *s_h,
                                                uint32_t *s_nw, uint32_t *s_wb, int32_t *s_wd) {
    constexpr uint32_t E = 16 / sizeof(T), U = 8;
    const uint32_t tid = threadIdx.x, nv = t.cumv[P];
#pragma unroll
    for (uint32_t u = 0; u < PF; ++u)
        if (u * NT + tid < nv) cx_count_vec<WRAP, T, CB>(s_h, x[u], s_nw, s_wb, s_wd);
    // vectors past the prefetch (buckets of more than PF * NT * E keys), U in flight
#pragma unroll 1
    for (uint32_t g0 = PF * NT; g0 < nv; g0 += U * NT) {
        uint4 y[U];
#pragma unroll
        for (uint32_t u = 0; u < U; ++u) y[u] = ld_run(cx_vec(recv, t, P, min(g0 + u * NT + tid, nv - 1)));
#pragma unroll
        for (uint32_t u = 0; u < U; ++u)
            if (g0 + u * NT + tid < nv) cx_count_vec<WRAP, T, CB>(s_h, y[u], s_nw, s_wb, s_wd);
    }
    // the pieces' unaligned heads and tails: < E elements each, one per thread
    for (uint32_t e = tid; e < (uint32_t)P * 2 * E; e += NT) {
        const uint32_t p = e / (2 * E), k = e % (2 * E);
        const uint32_t hd = t.head[p], n = t.len[p];
        const uint32_t body = hd + (t.cumv[p + 1] - t.cumv[p]) * E;
        uint32_t j = ~0u;
        if (k < E) { if (k < hd) j = k; }
        else if (body + (k - E) < n) j = body + (k - E);
        if (j != ~0u) cx_count<WRAP, CB>(s_h, (uint32_t)ld_run(run_ptr(recv, t.src[p] + j)) & 0xFFFFu, s_nw, s_wb, s_wd);
    }
}

// Lane's 4 bins of one 256-bin chunk whose first word is wd0 (u8: word wd0 + lane; u16: words
// wd0 + 2 lane, +1), with the u16 kernel's wrap corrections (nw entries) applied.
template <int CB>
__device__ __forceinline__ void cx_counts(const uint32_t *s_h, uint32_t wd0, uint32_t lane,
                                          uint32_t nw, const uint32_t *s_wb, const int32_t *s_wd,
                                          uint32_t (&c)[4]) {
    if (CB == 8) {
        const uint32_t y = s_h[wd0 + lane];
        c[0] = y & 255u;
        c[1] = (y >> 8) & 255u;
        c[2] = (y >> 16) & 255u;
        c[3] = y >> 24;
        return;
    }
    const uint32_t wd = wd0 + 2 * lane;
    const uint2 y = *reinterpret_cast<const uint2 *>(s_h + wd);
    c[0] = y.x & 0xFFFFu;
    c[1] = y.x >> 16;
    c[2] = y.y & 0xFFFFu;
    c[3] = y.y >> 16;
    for (uint32_t e = 0; e < nw; ++e) {
        const uint32_t b = s_wb[e] - 2 * wd;  // bin relative to the lane's first
        if (b < 4u) {
            const uint32_t dd = (uint32_t)s_wd[e];
            c[0] += b == 0 ? dd : 0u;
            c[1] += b == 1 ? dd : 0u;
            c[2] += b == 2 ? dd : 0u;
            c[3] += b == 3 ? dd : 0u;
        }
    }
}

// Words of bins each expanding wave owns: 2048 (u8: 8 waves x 8192 bins; u16: 16 x 4096)
constexpr uint32_t kCxWaveWords = 2048;

// One wave's expansion (K18c): its bins -- words w0 .. w0 + kCxWaveWords of s_h -- hold
// nkw keys, written as ONE run at d in windows of 256 slots aligned to 16 B; the chunks are
// streamed through registers (a window marks the bins of every chunk starting in it; the last
// chunk it touched carries over) and every bin word is zeroed after its read.  mk4: the wave's
// 80 uint4 of marks (256 window slots + 64 dummy words: a lane's marks outside the window).
// hk: the bucket's top 16 bits (flipped unless EST); EST stores add koff and flip.
template <int CB, bool EST>
__device__ __forceinline__ void cx_expand_wave(uint32_t *s_h, uint32_t w0, uint4 *mk4,
                                               uint32_t *d, uint32_t nkw, uint32_t hk,
                                               uint32_t koff, uint32_t nw,
                                               const uint32_t *s_wb, const int32_t *s_wd) {
    constexpr uint32_t BPW = 32 / CB;            // bins per word
    constexpr uint32_t CW = 256 / BPW;           // words per chunk: 4 bins per lane (8 per lane
                                                 // with u8 bins measured slower: r05_recv_u8_bins)
    constexpr uint32_t CH = kCxWaveWords / CW;   // chunks per wave (u8: 32, u16: 16)
    const uint32_t lane = threadIdx.x & 63;
    uint32_t *mk = reinterpret_cast<uint32_t *>(mk4);
    const uint32_t off = (uint32_t)(reinterpret_cast<uintptr_t>(d) >> 2) & 3u;
    // windows [ws, ws + 256) of the wave's run; chunk j's bins mark the windows they start in
    // (an empty bin is parked at 2^31, past every window), and a window is finished once the
    // chunk being marked reaches past it
    // (wave-uniform values kept scalar: the window loop below then stays a scalar loop -- with
    // them in VGPRs the compiler ran it as a divergent one)
    uint32_t ws = 0u - off, lo = 0, carry = 0;
    auto finish = [&]() {  // window ws: keys from the marks, stored; next window cleared
        __builtin_amdgcn_wave_barrier();
        const uint4 m = mk4[lane];
        const uint32_t a0 = m.x, a1 = max(a0, m.y), a2 = max(a1, m.z), a3 = max(a2, m.w);
        const uint32_t S = wave_incl_max(a3);
        // the lanes below: S of lane - 1 (DPP wave shift right by one; lane 0 reads 0)
        const uint32_t prev = max(carry, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)S, 0x138, 0xf, 0xf, true));
        carry = max(carry, (uint32_t)__builtin_amdgcn_readlane((int)S, 63));
        const uint32_t q = ws + 4 * lane;  // this lane's first slot
        uint4 v = make_uint4(max(prev, a0), max(prev, a1), max(prev, a2), max(prev, a3));
        if (EST) {  // relative ordered keys -> int32
            v.x = (v.x + koff) ^ kFlip;
            v.y = (v.y + koff) ^ kFlip;
            v.z = (v.z + koff) ^ kFlip;
            v.w = (v.w + koff) ^ kFlip;
        }
        if (q + 4 <= nkw && q < nkw) {
            *reinterpret_cast<uint4 *>(d + q) = v;  // 16-B aligned (nontemporal: slower, r04_ab_nt_stores)
        } else {
            if (q < nkw) d[q] = v.x;
            if (q + 1 < nkw) d[q + 1] = v.y;
            if (q + 2 < nkw) d[q + 2] = v.z;
            if (q + 3 < nkw) d[q + 3] = v.w;
        }
        __builtin_amdgcn_wave_barrier();
        mk4[lane] = make_uint4(0, 0, 0, 0);
        ws += 256;
    };
    mk4[lane] = make_uint4(0, 0, 0, 0);
#pragma unroll 1
    for (uint32_t j = 0; j < CH; ++j) {
        uint32_t c[4];
        cx_counts<CB>(s_h, w0 + CW * j, lane, nw, s_wb, s_wd, c);
        // the chunk's last read: its words are zeroed for the next bucket here
        if (CB == 8) s_h[w0 + CW * j + lane] = 0;
        else *reinterpret_cast<uint2 *>(s_h + w0 + CW * j + 2 * lane) = make_uint2(0, 0);
        const uint32_t tc = c[0] + c[1] + c[2] + c[3];
        const uint32_t y = wave_incl_add(tc);
        uint32_t sm[4], st = lo + y - tc;
        const uint32_t k0 = hk | (CB == 8 ? 4 * (w0 + CW * j + lane) : 2 * (w0 + CW * j + 2 * lane));
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            sm[q] = c[q] ? st : 0x80000000u;
            st += c[q];
        }
        const uint32_t hi = (uint32_t)__builtin_amdgcn_readfirstlane(
            (int)(lo + (uint32_t)__builtin_amdgcn_readlane((int)y, 63)));
#pragma unroll 1
        while (true) {
            __builtin_amdgcn_wave_barrier();
#pragma unroll
            for (int q = 0; q < 4; ++q) {  // no branch: a bin off the window marks the dummy
                const uint32_t r = sm[q] - ws;
                mk[r < 256u ? r : 256u + lane] = k0 + q;
            }
            if (hi - ws <= 256u) break;  // every bin of chunk j starts before ws + 256
            finish();
        }
        lo = hi;
    }
    while (ws + off < nkw + off) finish();
}

// EST: the sampled plan's oversized children (cx_fill_table_est: recv = Y, P = 1): keys are
// relative to the block's minimum koff, so the expansion marks relative keys (monotonic in the
// slot, as the max-scan needs) and the stores add koff and flip.
// CB = 8 (round 5): u8 bins -- 64 KiB of counters, 512 threads, two
// workgroups per CU -- halve the fixed per-bucket cost (every bin zeroed and read twice: ~9 us
// per bucket and CU with u16 bins, i.e. 0.29 of the 0.58 ms per 2^28 keys of the P = 4 shape's
// 32 768-key buckets).  A byte that wraps (>= 256 copies of one key) shows as a total below the
// bucket's size: the bucket goes to fb_list (fb_ctr entries, the {h, len} entry as given) with
// its bins cleared, and the u16 kernel redoes it (a list whose count it reads on the device).
// The buckets are the entries of cl's lists walked as one index space (CxLists).
template <typename T, bool EST = false, int CB = 16>
__global__ __launch_bounds__(CB == 8 ? 512 : 1024) void k_count_expand(
    const T *__restrict__ recv, const unsigned long long *__restrict__ pos,
    const unsigned long long *__restrict__ roff, int P,
    const unsigned long long *__restrict__ bstart, CxLists cl, uint32_t *__restrict__ out,
    uint32_t koff = 0, unsigned long long *__restrict__ fb_list = nullptr,
    uint32_t *__restrict__ fb_ctr = nullptr) {
    static_assert(CB == 8 || CB == 16, "u8 or u16 bins");
    constexpr uint32_t NT = CB == 8 ? 512 : 1024, NW = NT / 64;
    constexpr uint32_t WORDS = 65536 * CB / 32;  // 16 384 (u8) / 32 768 (u16) words of bins
    constexpr uint32_t BPW = 32 / CB;            // bins per word
    constexpr uint32_t CW = 256 / BPW;           // words per chunk: 4 bins per lane (8 per lane
                                                 // with u8 bins measured slower: r05_recv_u8_bins)
    constexpr uint32_t CH = WORDS / NW / CW;     // chunks per wave (32 / 16)
    static_assert(WORDS / NW == kCxWaveWords, "cx_expand_wave's range per wave");
    constexpr uint32_t PF = 8;  // prefetched 16-B vectors per thread
    // the lists' lengths (read on the device for a launch queued before the host knew them;
    // the u8 kernel's wrapped buckets: usually none)
    uint32_t nn[kCxLists], nlist = 0;
#pragma unroll
    for (int q = 0; q < kCxLists; ++q) {
        nn[q] = 0;
        if (q < cl.nl) {
            nn[q] = cl.ndev[q] ? ld_run(cl.ndev[q]) : cl.n[q];
            if (q == cl.skip && ld_run(reinterpret_cast<const unsigned long long *>(cl.skip_max)) > kHxMax)
                nn[q] = 0;
        }
        nlist += nn[q];
    }
    if (blockIdx.x >= nlist) return;
    auto entry = [&](uint32_t i) -> const unsigned long long * {  // entry i of the joined lists
#pragma unroll
        for (int q = 0; q < kCxLists; ++q) {
            if (i < nn[q]) return reinterpret_cast<const unsigned long long *>(cl.list[q]) + 2 * i;
            i -= nn[q];
        }
        return nullptr;
    };
    __shared__ uint32_t s_h[WORDS];
    // per wave: 256 window slots + 64 dummy words (a lane's marks outside the window)
    // per wave: 256 window slots + 64 dummy words (a lane's marks outside the window)
    __shared__ uint4 s_mark[NW * 80];
    __shared__ uint32_t s_base[2 * NW];  // waves' output offsets, totals
    __shared__ uint32_t s_wsum[NW];
    __shared__ CxTable<T> s_t[2];
    __shared__ uint32_t s_wb[kCxWrapMax];
    __shared__ int32_t s_wd[kCxWrapMax];
    __shared__ uint32_t s_nw;
    const uint32_t tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    uint32_t cur = 0;
    auto fill = [&](CxTable<T> &t, uint32_t i) {
        if (EST) cx_fill_table_est(t, recv, entry(i));
        else cx_fill_table(t, recv, pos, roff, P, bstart, entry(i));
    };
    if (tid < 64) fill(s_t[0], blockIdx.x);
    __syncthreads();
    {
        uint4 *z = reinterpret_cast<uint4 *>(s_h);
#pragma unroll
        for (uint32_t q = 0; q < WORDS / 4 / NT; ++q) z[q * NT + tid] = make_uint4(0, 0, 0, 0);
    }
    __syncthreads();
    uint4 x[PF];
    {
        const uint32_t nv = s_t[0].cumv[P];
#pragma unroll
        for (uint32_t u = 0; u < PF; ++u)
            if (u * NT + tid < nv) x[u] = ld_run(cx_vec(recv, s_t[0], P, u * NT + tid));
    }
#pragma unroll 1
    for (uint32_t i = blockIdx.x; i < nlist; i += gridDim.x) {
        const uint32_t nxt = cur ^ 1u;
        CxTable<T> &t = s_t[cur];
        // (the bins are zero: before the first bucket, and the expansion zeroes every word
        // after its last read); wave 0 reads the next bucket's pieces, in flight meanwhile
        if (tid < 64) fill(s_t[nxt], i + gridDim.x);
        if (tid == 0) s_nw = 0;
        const uint32_t h = (uint32_t)__builtin_amdgcn_readfirstlane((int)t.h);
        const uint32_t len = (uint32_t)__builtin_amdgcn_readfirstlane((int)t.keys);
        const uint64_t tdst = ((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(t.dst >> 32)) << 32) |
                              (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)t.dst);
        // count with non-returning atomics; a u16 half that wrapped (>= 65 536 copies of one
        // value) shows as a total below len, and only then is the bucket counted again with the
        // wraps tracked (returning atomics)
        uint32_t nw = 0;
        const uint32_t w0 = w * (WORDS / NW);
        auto counts = [&](uint32_t j, uint32_t (&c)[4]) {  // lane's 4 bins of chunk j
            cx_counts<CB>(s_h, w0 + CW * j, lane, nw, s_wb, s_wd, c);
        };
        auto wave_totals = [&]() -> uint32_t {  // the waves' totals into s_wsum; the bucket's
            uint32_t tw = 0;
#pragma unroll 4
            for (uint32_t j = 0; j < CH; ++j) {
                uint32_t c[4];
                counts(j, c);
                tw += c[0] + c[1] + c[2] + c[3];
            }
            const uint32_t y = wave_incl_add(tw);
            if (lane == 63) s_wsum[w] = y;
            __syncthreads();
            uint32_t tot = 0;
#pragma unroll
            for (uint32_t ww = 0; ww < NW; ++ww) tot += s_wsum[ww];
            return tot;
        };
        cx_count_bucket<false, T, PF, NT, CB>(recv, t, P, x, s_h, &s_nw, s_wb, s_wd);
        __syncthreads();
        bool skip = false;  // (CB = 8: a byte wrapped, the bucket went to fb_list)
        if (wave_totals() != len) {
            uint4 *z = reinterpret_cast<uint4 *>(s_h);
#pragma unroll
            for (uint32_t q = 0; q < WORDS / 4 / NT; ++q) z[q * NT + tid] = make_uint4(0, 0, 0, 0);
            if constexpr (CB == 8) {
                if (tid == 0) {
                    const uint32_t e = atomicAdd(fb_ctr, 1u);
                    const unsigned long long *en = entry(i);
                    fb_list[2 * e] = ld_run(en);
                    fb_list[2 * e + 1] = ld_run(en + 1);
                }
                skip = true;
                if (tid < NW) s_wsum[tid] = 0;  // no keys to expand (s_base below)
                __syncthreads();
            } else {  // a half wrapped: count again, tracking the wraps
                __syncthreads();
                cx_count_bucket<true, T, PF>(recv, t, P, x, s_h, &s_nw, s_wb, s_wd);
                __syncthreads();
                nw = min(s_nw, kCxWrapMax);  // uniform
                (void)wave_totals();
            }
        }
        (void)skip;
        // the waves' output offsets (block scan of 16)
        if (tid < NW) {
            uint32_t e = 0;
            for (uint32_t ww = 0; ww < tid; ++ww) e += s_wsum[ww];
            s_base[tid] = e;
            s_base[NW + tid] = s_wsum[tid];
        }
        __syncthreads();
        // the next bucket's first vectors: in flight during the expansion below
        {
            const uint32_t nv = s_t[nxt].keys ? s_t[nxt].cumv[P] : 0u;
#pragma unroll
            for (uint32_t u = 0; u < PF; ++u)
                if (u * NT + tid < nv) x[u] = ld_run(cx_vec(recv, s_t[nxt], P, u * NT + tid));
        }
        // expansion: the wave's keys are ONE run of out (cx_expand_wave)
        const uint32_t nkw = (uint32_t)__builtin_amdgcn_readfirstlane((int)s_base[NW + w]);
        if (nkw) {
            const uint64_t dst0 = tdst + (uint32_t)__builtin_amdgcn_readfirstlane((int)s_base[w]);
            cx_expand_wave<CB, EST>(s_h, w0, s_mark + 80 * w, out + dst0, nkw,
                                    EST ? h << 16 : (h << 16) ^ kFlip, koff, nw, s_wb, s_wd);
        }
        __syncthreads();  // the bins, the marks and table cur are reused
        cur = nxt;
    }
}

// list 0 of the receive side, {h | bstart[h] << 16, len} -> {bstart[h], len} (segments of out
// for the MSD levels).
__global__ __launch_bounds__(256) void k_list_to_segments(unsigned long long *__restrict__ list,
                                                          uint32_t n,
                                                          const unsigned long long *__restrict__ bstart) {
    const uint32_t i = blockIdx.x * 256 + threadIdx.x;
    if (i < n) list[2 * i] = list[2 * i] >> 16;  // (the entry carries bstart[h] above bit 16)
    (void)bstart;
}

// Oversized receive buckets: gather their pieces into out[bstart[h] ..) as ordered u32 (they
// continue through the MSD levels 1 and 0).  One block per bucket; others exit.
template <typename T>
__global__ __launch_bounds__(256) void k_gather_copy(const T *__restrict__ recv,
                                                     const unsigned long long *__restrict__ pos,
                                                     const unsigned long long *__restrict__ roff,
                                                     int P,
                                                     const unsigned long long *__restrict__ bstart,
                                                     uint32_t *__restrict__ out,
                                                     unsigned long long n_out,
                                                     unsigned long long min_len, uint32_t xo) {
    // (buckets of more than min_len keys; every key stored XOR xo: 0 ordered u32, kFlip int32)
    // block b copies output positions [b * CH, (b + 1) * CH): every bucket past kLocalMax
    // overlapping them, piece by piece.  (Round 6: one block per BUCKET took 67 ms per call on a
    // Zipf block's giant buckets -- 82 % of a P = 8 Zipf sample sort, profiles/r06_zipf_p8.txt.)
    constexpr unsigned long long CH = 65536;
    const unsigned long long c0 = (unsigned long long)blockIdx.x * CH;
    if (c0 >= n_out) return;
    const unsigned long long c1 = c0 + CH < n_out ? c0 + CH : n_out;
    uint32_t lo = 0, hi = kBuckets16;  // the last bucket starting at or before c0
    while (hi - lo > 1) {
        const uint32_t mid = (lo + hi) >> 1;
        if (bstart[mid] <= c0) lo = mid; else hi = mid;
    }
    for (uint32_t h = lo; h < kBuckets16; ++h) {
        const unsigned long long b0 = bstart[h], b1 = bstart[h + 1];
        if (b0 >= c1) break;
        if (b1 - b0 <= min_len) continue;
        unsigned long long cum = b0;  // piece p's first output position
        for (int p = 0; p < P; ++p) {
            const unsigned long long a = pos[(uint64_t)p * (kBuckets16 + 1) + h];
            const unsigned long long len = pos[(uint64_t)p * (kBuckets16 + 1) + h + 1] - a;
            const unsigned long long s0 = cum > c0 ? cum : c0;
            const unsigned long long e0 = cum + len < c1 ? cum + len : c1;
            if (s0 < e0) {
                // indexed by output position: the offset formed as an integer (mod 2^64)
                const T *src = run_ptr(recv, roff[p] + a - cum);
                unsigned long long i = s0 + threadIdx.x;
                for (; i + 3 * 256 < e0; i += 4 * 256) {  // four loads in flight per lane
                    T v[4];
#pragma unroll
                    for (int u = 0; u < 4; ++u) v[u] = ld_run(src + (i + u * 256));
#pragma unroll
                    for (int u = 0; u < 4; ++u) out[i + u * 256] = recv_key(v[u], h) ^ xo;
                }
                for (; i < e0; i += 256) out[i] = recv_key(ld_run(src + i), h) ^ xo;
            }
            cum += len;
        }
    }
}

// Packed exchange of the distributed radix (sender): the low 16 bits of every key (the top 16
// are implied by the bucket each piece belongs to, sent as counts).
__global__ __launch_bounds__(256) void k_pack16(const int32_t *__restrict__ a, uint64_t n,
                                                uint16_t *__restrict__ out) {
    const uint64_t stride = (uint64_t)gridDim.x * 256;
    for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += stride)
        out[i] = (uint16_t)(uint32_t)a[i];
}

// Packed sender: out[i] = key of bucket h from its low 16 bits (int32), i < n.
__global__ __launch_bounds__(256) void k_unpack16(const uint16_t *__restrict__ in, uint64_t n,
                                                  uint32_t h, int32_t *__restrict__ out) {
    const uint64_t stride = (uint64_t)gridDim.x * 256;
    for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += stride)
        out[i] = (int32_t)(((h << 16) | in[i]) ^ kFlip);
}

// Packed sender, bucket bounds from the MSD plan instead of the keys: block s (level-3 bucket
// s, bases / totals of level 3) finds its level-2 segment (list0 entry starting at bases[s];
// every non-empty level-3 bucket is one) and copies the 256 child starts; an empty bucket's
// children all start at bases[s].  gb[65536] = n.
__global__ __launch_bounds__(kRadix) void k_gb_from_plan(
    const unsigned long long *__restrict__ bases, const unsigned long long *__restrict__ totals,
    const unsigned long long *__restrict__ segs, uint32_t nseg,
    const unsigned long long *__restrict__ cstart, uint64_t n,
    unsigned long long *__restrict__ gb) {
    __shared__ int s_j;
    const uint32_t sb = blockIdx.x, d = threadIdx.x;
    if (d == 0) s_j = -1;
    __syncthreads();
    const uint64_t b = bases[sb];
    const bool empty = totals[sb] == 0;
    if (!empty)
        for (uint32_t j = d; j < nseg; j += kRadix)
            if (segs[2 * j] == b && segs[2 * j + 1] != 0) s_j = (int)j;
    __syncthreads();
    const int j = s_j;
    gb[(uint64_t)sb * kRadix + d] = (empty || j < 0) ? b : cstart[(uint64_t)j * kRadix + d];
    if (sb == 0 && d == 0) gb[kBuckets16] = n;
}

// K13 on the packed send buffer: out[i] = #keys (ordered u32) < xs[i], from the bucket bounds
// for whole buckets and a binary search of the low 16 bits inside bucket xs[i] >> 16 (which
// the caller has sorted whenever xs[i] is not a bucket start).
__global__ __launch_bounds__(256) void k_count_below16(const uint16_t *__restrict__ a,
                                                       const unsigned long long *__restrict__ gb,
                                                       const unsigned long long *__restrict__ xs,
                                                       int m, unsigned long long *__restrict__ out) {
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i >= m) return;
    const uint64_t x = xs[i];
    const uint64_t h = x >> 16;
    if (h >= kBuckets16) { out[i] = gb[kBuckets16]; return; }
    const uint32_t lo16 = (uint32_t)(x & 0xFFFFu);
    uint64_t lo = gb[h], hi = gb[h + 1];
    if (lo16 == 0) { out[i] = lo; return; }
    while (lo < hi) {
        const uint64_t mid = (lo + hi) >> 1;
        if ((uint32_t)a[mid] < lo16) lo = mid + 1; else hi = mid;
    }
    out[i] = lo;
}

// Sender: for destination block q (rng[5q..] = {a, b, h_lo, nh, out_off}), meta[out_off + i] =
// keys of this rank's cut [a, b) in bucket h_lo + i (gb = bucket bounds of the grouped block).
__global__ __launch_bounds__(256) void k_meta_counts(const unsigned long long *__restrict__ gb,
                                                     const unsigned long long *__restrict__ rng,
                                                     uint32_t *__restrict__ meta) {
    const unsigned long long *r = rng + 5 * blockIdx.y;
    const uint64_t a = r[0], b = r[1], h0 = r[2], nh = r[3], off = r[4];
    for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < nh;
         i += (uint64_t)gridDim.x * 256) {
        const uint64_t x = gb[h0 + i], y = gb[h0 + i + 1];
        const uint64_t lo = x > a ? x : a, hi = y < b ? y : b;
        meta[off + i] = (uint32_t)(hi > lo ? hi - lo : 0);
    }
}

// Row-wise exclusive scans over the 2^16 buckets (one row per source, or the bucket sizes):
// 64 blocks per row each reduce 1024 consecutive values (coalesced), then each block scans
// its 1024 values on top of the reduced prefix of the blocks before it; out[row][65536] =
// the row total.  Value sources: per-source bucket counts of the packed exchange, or sizes.
struct MetaCounts {  // source p's count of bucket h (0 outside [h_lo, h_lo + nh))
    const uint32_t *meta;
    const unsigned long long *moff;
    uint32_t h_lo, nh;
    __device__ unsigned long long operator()(uint32_t p, uint32_t h) const {
        const unsigned long long mo = moff[p];
        return (mo != ~0ull && h >= h_lo && h - h_lo < nh) ? meta[mo + (h - h_lo)] : 0ull;
    }
};
struct MetaCountsSum {  // rows 0 .. P-1: MetaCounts; row P: the bucket's total over the sources
    MetaCounts m;
    uint32_t P;
    __device__ unsigned long long operator()(uint32_t row, uint32_t h) const {
        if (row < P) return m(row, h);
        unsigned long long t = 0;
        for (uint32_t p = 0; p < P; ++p) t += m(p, h);
        return t;
    }
};
struct RowValues {  // v[h] (one row)
    const unsigned long long *v;
    __device__ unsigned long long operator()(uint32_t, uint32_t h) const { return v[h]; }
};
constexpr uint32_t kScanBlocks = kBuckets16 / 1024;  // 64

// zero[0 .. nzero) := 0 by block (0, 0) (the receive side's work-list counters, which the
// classification after the scan adds into: no memset of their own on the stream)
template <typename Gen>
__global__ __launch_bounds__(1024) void k_rowscan_reduce(Gen gen,
                                                         unsigned long long *__restrict__ part,
                                                         unsigned long long *zero = nullptr,
                                                         uint32_t nzero = 0) {
    __shared__ unsigned long long s_w[16];
    const uint32_t row = blockIdx.y, b = blockIdx.x, tid = threadIdx.x, lane = tid & 63,
                   w = tid >> 6;
    if (zero && (row | b) == 0 && tid < nzero) zero[tid] = 0;
    unsigned long long x = gen(row, b * 1024 + tid);
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) x += __shfl_xor(x, o);
    if (lane == 0) s_w[w] = x;
    __syncthreads();
    if (tid == 0) {
        unsigned long long t = 0;
        for (int i = 0; i < 16; ++i) t += s_w[i];
        part[row * kScanBlocks + b] = t;
    }
}

// K15s: the receive plan's row scans in ONE pass -- north_star's single-pass decoupled-lookback
// exclusive scan, where it fits (round 6: the 2^16-bucket rows of the receive plan; the local
// sort's passes lost to it in v0).  Every block of 1024 values publishes its
// aggregate, then its inclusive prefix, in a status word; its wave 0 reads the status words of
// all its predecessors in the row at once (one per lane: 64 blocks per row) and sums aggregates
// back to the nearest inclusive prefix.  A block takes its place in the grid from an atomic
// ticket as it starts, so every predecessor it waits on has started (no reliance on the order
// of dispatch); the block holding the last ticket resets the ticket for the next call.
// Status word: state (bits 62-63: 1 aggregate, 2 inclusive prefix) | epoch (bits 40-61: the
// call, so a word left by an earlier call never counts) | value (bits 0-39).
constexpr unsigned long long kLbValue = (1ull << 40) - 1, kLbEpoch = 0x3FFFFFull << 40;
template <typename Gen>
__global__ __launch_bounds__(1024) void k_rowscan_lookback(Gen gen,
                                                           unsigned long long *__restrict__ status,
                                                           unsigned int *__restrict__ ticket,
                                                           uint32_t epoch,
                                                           unsigned long long *__restrict__ out,
                                                           uint64_t row_stride,
                                                           unsigned long long *out_last,
                                                           unsigned long long *zero,
                                                           uint32_t nzero) {
    __shared__ unsigned long long s_w[16];
    __shared__ unsigned long long s_pre;
    __shared__ uint32_t s_vb;
    const uint32_t tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const uint32_t nblk = gridDim.x * gridDim.y;
    if (tid == 0) s_vb = atomicAdd(ticket, 1u);
    __syncthreads();
    // (the ticket is zero on entry -- the runtime zeroes it with its buffer, the last block of
    // every launch resets it; "% nblk" keeps even a stray value a permutation of the blocks)
    const uint32_t vb = s_vb % nblk;
    const uint32_t row = vb / kScanBlocks, b = vb % kScanBlocks;
    if (zero && vb == 0 && tid < nzero) zero[tid] = 0;
    const unsigned long long c = gen(row, b * 1024 + tid);
    unsigned long long x = c;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const unsigned long long t = __shfl_up(x, o);
        if ((int)lane >= o) x += t;
    }
    if (lane == 63) s_w[w] = x;
    __syncthreads();
    if (w == 0) {
        unsigned long long tot = lane < 16 ? s_w[lane] : 0ull;
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) tot += __shfl_xor(tot, o);
        const unsigned long long ep = ((unsigned long long)epoch << 40) & kLbEpoch;
        unsigned long long *st = status + (uint64_t)row * kScanBlocks;
        unsigned long long excl = 0;
        if (b == 0) {
            if (lane == 0)
                __hip_atomic_store(&st[0], (2ull << 62) | ep | tot, __ATOMIC_RELEASE,
                                   __HIP_MEMORY_SCOPE_AGENT);
        } else {
            if (lane == 0)
                __hip_atomic_store(&st[b], (1ull << 62) | ep | tot, __ATOMIC_RELEASE,
                                   __HIP_MEMORY_SCOPE_AGENT);
            const int p = (int)b - 1 - (int)lane;  // lane j looks at predecessor b - 1 - j
            while (true) {
                unsigned long long v = 0;
                if (p >= 0) v = __hip_atomic_load(&st[p], __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT);
                const bool cur = p >= 0 && (v & kLbEpoch) == ep && (v >> 62) != 0;
                const uint64_t im = __ballot(cur && (v >> 62) == 2);
                const uint64_t cm = __ballot(cur);
                if (im) {  // the nearest inclusive prefix, and every aggregate before it in
                    const uint32_t f = (uint32_t)__builtin_ctzll(im);
                    const uint64_t need = f == 63 ? ~0ull : (2ull << f) - 1;
                    if ((cm & need) == need) {
                        unsigned long long sv = lane <= f ? (v & kLbValue) : 0ull;
#pragma unroll
                        for (int o = 32; o > 0; o >>= 1) sv += __shfl_xor(sv, o);
                        excl = sv;
                        break;
                    }
                }
                __builtin_amdgcn_s_sleep(1);
            }
            if (lane == 0)
                __hip_atomic_store(&st[b], (2ull << 62) | ep | (excl + tot), __ATOMIC_RELEASE,
                                   __HIP_MEMORY_SCOPE_AGENT);
        }
        if (lane == 0) s_pre = excl;
    }
    __syncthreads();
    unsigned long long run = s_pre + x - c;
    for (uint32_t ww = 0; ww < w; ++ww) run += s_w[ww];
    unsigned long long *o = out_last && row == gridDim.y - 1 ? out_last : out + row * row_stride;
    o[b * 1024 + tid] = run;
    if (b == kScanBlocks - 1 && tid == 1023) o[kBuckets16] = run + c;
    // every other block has taken its ticket: the last one resets it for the next launch
    if (tid == 0 && s_vb == nblk - 1)
        __hip_atomic_store(ticket, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

template <typename Gen>
__global__ __launch_bounds__(1024) void k_rowscan_apply(Gen gen,
                                                        const unsigned long long *__restrict__ part,
                                                        unsigned long long *__restrict__ out,
                                                        uint64_t row_stride,
                                                        unsigned long long *out_last) {
    __shared__ unsigned long long s_w[16];
    __shared__ unsigned long long s_pre;
    const uint32_t row = blockIdx.y, b = blockIdx.x, tid = threadIdx.x, lane = tid & 63,
                   w = tid >> 6;
    if (tid < 64) {  // prefix of the earlier blocks of this row (b < 64 partials)
        unsigned long long v = tid < b ? part[row * kScanBlocks + tid] : 0ull;
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
        if (tid == 0) s_pre = v;
    }
    const unsigned long long c = gen(row, b * 1024 + tid);
    unsigned long long x = c;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const unsigned long long t = __shfl_up(x, o);
        if ((int)lane >= o) x += t;
    }
    if (lane == 63) s_w[w] = x;
    __syncthreads();
    unsigned long long run = s_pre + x - c;
    for (uint32_t ww = 0; ww < w; ++ww) run += s_w[ww];
    // (out_last: the last row goes there instead)
    unsigned long long *o = out_last && row == gridDim.y - 1 ? out_last : out + row * row_stride;
    o[b * 1024 + tid] = run;
    if (b == kScanBlocks - 1 && tid == 1023) o[kBuckets16] = run + c;
}

// Self-check of the LDS lane-order property wave_rank<true> relies on: every wave of a block
// ranks 16 rounds of digits drawn from `digits` (nbins-valued) with ds_add_rtn and counts the
// ranks that are not the wave's previous rank of that digit + 1.  bad[0] must stay 0.
__global__ __launch_bounds__(512) void k_lds_order_check(const uint32_t *__restrict__ digits,
                                                          uint32_t nbins,
                                                          unsigned long long *bad) {
    __shared__ uint32_t cnt[8 * kRadix];
    __shared__ uint32_t last[8 * kRadix];
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    for (int i = tid; i < 8 * kRadix; i += 512) { cnt[i] = 0; last[i] = 0xFFFFFFFFu; }
    __syncthreads();
    const uint64_t base = ((uint64_t)blockIdx.x * 8 + w) * 64 * 16;
    uint32_t d[16], r[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) d[i] = digits[base + i * 64 + lane] % nbins;
#pragma unroll
    for (int i = 0; i < 16; ++i) r[i] = atomicAdd(&cnt[w * kRadix + d[i]], 1u);
    // lane order within a round: a lane's rank exceeds the rank of every lower lane with the
    // same digit; across rounds: exceeds every rank of an earlier round
    uint32_t nbad = 0;
#pragma unroll
    for (int i = 0; i < 16; ++i) {
        for (int l = 0; l < 64; ++l) {
            const uint32_t dl = __shfl(d[i], l), rl = __shfl(r[i], l);
            if (l < lane && dl == d[i] && rl >= r[i]) ++nbad;
        }
        uint32_t *lw = last + w * kRadix;
        // every lane of the round, in lane order, checks against the previous round's maximum
        if (i > 0 && lw[d[i]] != 0xFFFFFFFFu && r[i] <= lw[d[i]]) ++nbad;
        __syncthreads();
        atomicMax(&lw[d[i]], r[i]);
        __syncthreads();
    }
    if (nbad) atomicAdd(bad, (unsigned long long)nbad);
}

// =======================================================================================
// Sampled plan (the default local MSD sort for large blocks).  The two-level
// plan reads every key once only to size the level-3 buckets and level-2 children (K1h, 4 B
// per key of the 28).  Here a 1/64 sample sizes them instead: every region gets its estimate
// plus 6 sigma of sampling error, so the partitions write into gapped regions (level 3 into X,
// level 2 into Y) whose true fill is only known afterwards, and K11 sorts each child from Y
// into its exact place in the output.  A level-2 child's keys share their top 16 bits (its
// level-3 bucket and level-2 digit, below the constant prefix of a shifted plan), so Y holds
// only the low 16 bits of every key (u16) and K11e puts the child's top half back: 4 + 4 (K3r)
// + 4 + 2 (K3a) + 2 + 4 (K11e) = 20 B/key.  A run that would overflow its region is
// diverted to a scratch tile and flagged (the runtime then re-sorts on the exact plan), so the
// estimate decides speed, never the result.
//   K1e k_est_sample: sample histograms (8 consecutive keys at a hashed offset of every
//       512-key block: short segments keep the estimate of position-correlated input, e.g.
//       concatenated sorted runs, close to that of independent samples), 65536 u8 child
//       counters + 8 x 256 shard counters per workgroup
//   K12e k_est_plan: region capacities, bases and cursors; eligibility
//   K3r / K3a (EST): the reservation partitions with region limits
//   K12f k_est_tiles: K3a tile descriptors over the level-3 pieces (bucket x shard)
//   K12g k_est_classify: exact child sizes from the cursors, output offsets, K11 lists
//   K11e k_local_sort_e: K11 over {src in Y | top 16 bits, dst in out | len} entries
// The eflag word: bit 2 = ineligible (a child estimate above kLocalMax, a u8 counter wrap,
// every sample in one level-3 bucket, or a region total past its buffer): every later kernel
// returns at once and the runtime takes the exact plan.  ovf: a region overflowed.
// =======================================================================================
constexpr uint32_t kEstBlockKeys = kEstBlockKeysHost, kEstSegKeys = 8;
constexpr uint32_t kEstWG = kEstWGs;  // K1e workgroups (= partial histograms)
constexpr uint32_t kEstPartWords = kBuckets16 / 4, kEstPart3 = kShards * kRadix;

__device__ __forceinline__ uint32_t est_seg_off(uint32_t j) {  // sample offset in block j
    return (uint32_t)(mix64((uint64_t)j * kGolden + 0x5EEDull) >> 58) * kEstSegKeys;  // 0 .. 504
}

// K1e: thread tid samples key tid % 8 of segment tid / 8; workgroup b takes the 512-key
// blocks j = b * 128 + seg, + kEstWG * 128, ... (so every child's samples spread over all
// workgroups), sixteen loads in flight per thread.  part8[b][.] = the 65536 u8 child counters
// (packed 4 per word), part3[(d * kEstWG + b) * 8 + x] = samples of level-3 bucket d in shard x (tile
// pair j / 32, shard pair % 8, as K3r deals them), msamp[b] = samples | wrap << 31,
// msamp[kEstWG + b] = the key bits that differ from in[0] among its samples, msamp[2 / 3 *
// kEstWG + b] = their min / max.  koff: keys are taken as ordered u32 minus koff (the
// runtime's offset retry; 0 otherwise).  sb (0 .. 16):
// the plan's digits start sb bits lower (the top sb bits are one constant prefix: the runtime
// retries a block whose samples share leading bits that way; K3r verifies the prefix).
// Block 0 also initializes eflag[0..8] (eflag, ovf, K12g's and K12e's finished-block counts,
// K12e's count of sampled children, the samples' varying bits, min, max, largest child).
template <bool FIN>
__global__ __launch_bounds__(1024) void k_est_sample(const uint32_t *__restrict__ in, uint64_t n,
                                                     uint32_t *__restrict__ part8,
                                                     uint32_t *__restrict__ part3,
                                                     uint32_t *__restrict__ msamp,
                                                     uint32_t *__restrict__ eflag, int sb,
                                                     uint32_t koff) {
    __shared__ uint32_t s_h[kEstPartWords];
    __shared__ uint32_t s_3[kEstPart3];
    __shared__ uint32_t s_m, s_vary, s_lo, s_hi;
    const uint32_t tid = threadIdx.x;
    for (uint32_t i = tid; i < kEstPartWords; i += 1024) s_h[i] = 0;
    for (uint32_t i = tid; i < kEstPart3; i += 1024) s_3[i] = 0;
    if (tid == 0) { s_m = 0; s_vary = 0; s_lo = ~0u; s_hi = 0; }
    if (blockIdx.x == 0 && tid < 9) eflag[tid] = tid == 6 ? ~0u : 0u;
    // bits that vary across the samples (against key 0), and the samples' range
    const uint32_t ref = (FIN ? in[0] ^ kFlip : in[0]) - koff;
    __syncthreads();
    const uint32_t nblk = (uint32_t)((n + kEstBlockKeys - 1) / kEstBlockKeys);
    constexpr uint32_t SEGS = 1024 / kEstSegKeys;  // segments per workgroup round
    static_assert(kEstBlockKeys / kEstSegKeys == 64, "64 segment offsets per block");
    const uint32_t seg = tid / kEstSegKeys, kk = tid % kEstSegKeys, step = gridDim.x * SEGS;
    constexpr int U = 16;
    uint32_t cnt = 0, wrap = 0, vary = 0, lo = ~0u, hi = 0;
    for (uint32_t j0 = blockIdx.x * SEGS + seg; j0 < nblk; j0 += U * step) {
        uint32_t key[U], jj[U];
        bool ok[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            jj[u] = j0 + (uint32_t)u * step;
            const uint64_t pos = (uint64_t)jj[u] * kEstBlockKeys + est_seg_off(jj[u]) + kk;
            ok[u] = jj[u] < nblk && pos < n;
            key[u] = ok[u] ? in[pos] : 0u;
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            if (!ok[u]) continue;
            const uint32_t k = (FIN ? key[u] ^ kFlip : key[u]) - koff;
            vary |= k ^ ref;
            lo = min(lo, k);
            hi = max(hi, k);
            const uint32_t b = (k >> (16 - sb)) & 0xffffu, sh = (b & 3u) << 3;
            constexpr uint32_t kPairBlocks = 2 * kSweepTile / kEstBlockKeys;
            const uint32_t i3 = ((jj[u] / kPairBlocks) % kShards) * kRadix + ((k >> (24 - sb)) & 255u);
            // a wave whose samples all hit one counter word (8- / 16-bit keys, one frequent
            // value: same-address LDS adds serialize) adds them with one atomic from its first
            // lane; a byte wrapped when its old value plus its lanes passed 255
            const uint64_t ex = __builtin_amdgcn_read_exec();
            const bool first = lane_rank(ex) == 0;
            const uint32_t w0 = __builtin_amdgcn_readfirstlane(b >> 2);
            if (__ballot((b >> 2) == w0) == ex) {
                uint32_t inc = 0;
#pragma unroll
                for (uint32_t q = 0; q < 4; ++q)
                    inc |= (uint32_t)__popcll(__ballot((b & 3u) == q)) << (8 * q);
                uint32_t old = 0;
                if (first) old = atomicAdd(&s_h[w0], inc);
#pragma unroll
                for (uint32_t q = 0; q < 4; ++q)
                    wrap |= ((old >> (8 * q)) & 255u) + ((inc >> (8 * q)) & 255u) > 255u;
            } else {
                const uint32_t old = atomicAdd(&s_h[b >> 2], 1u << sh);
                wrap |= ((old >> sh) & 255u) == 255u;
            }
            const uint32_t i30 = __builtin_amdgcn_readfirstlane(i3);
            if (__ballot(i3 == i30) == ex) {
                if (first) atomicAdd(&s_3[i30], (uint32_t)__popcll(ex));
            } else {
                atomicAdd(&s_3[i3], 1u);
            }
            ++cnt;
        }
    }
    // wave reductions first: 64 lanes on one LDS word serialize
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        cnt += (uint32_t)__shfl_xor((int)cnt, o);
        wrap |= (uint32_t)__shfl_xor((int)wrap, o);
        vary |= (uint32_t)__shfl_xor((int)vary, o);
        lo = min(lo, (uint32_t)__shfl_xor((int)lo, o));
        hi = max(hi, (uint32_t)__shfl_xor((int)hi, o));
    }
    if ((tid & 63) == 0) {
        // (the wrap bit by OR: two waves adding it would cancel -- at n = 2^22 only 64
        // workgroups sample, 1024 keys each, and a 60 % child wraps its u8 counter twice)
        atomicAdd(&s_m, cnt);
        if (wrap) atomicOr(&s_m, 1u << 31);
        if (vary) atomicOr(&s_vary, vary);
        if (cnt) { atomicMin(&s_lo, lo); atomicMax(&s_hi, hi); }
    }
    __syncthreads();
    uint32_t *dst = part8 + (uint64_t)blockIdx.x * kEstPartWords;
    for (uint32_t i = tid; i < kEstPartWords; i += 1024) dst[i] = s_h[i];
    // part3 bucket-major, [d][b][x]: K12e's block d then reads its 2048 words contiguously (a
    // workgroup-major layout made that a 4-B load per 64-B line: 34 MB fetched for 19 MB)
    for (uint32_t i = tid; i < kEstPart3; i += 1024) {
        const uint32_t d = i >> 3, x = i & (kShards - 1);
        part3[((uint64_t)d * kEstWG + blockIdx.x) * kShards + x] = s_3[x * kRadix + d];
    }
    if (tid == 0) {
        msamp[blockIdx.x] = s_m;
        msamp[kEstWG + blockIdx.x] = s_vary;
        msamp[2 * kEstWG + blockIdx.x] = s_lo;
        msamp[3 * kEstWG + blockIdx.x] = s_hi;
    }
}

// A region's capacity from its sample count: the estimate + the larger of 6 sigma of the
// sampling error and two sample blocks (on position-correlated input -- sorted runs -- a
// region's keys are contiguous and its only error is the two blocks its ends cut) + 64 keys.
// slack scales the margin (GSORT_EST_SLACK, a test hook: 0 forces overflows).
__device__ __forceinline__ uint64_t est_cap(uint32_t cnt, double scale, double slack) {
    const double c = (double)cnt;
    const double sig = fmax(6.0 * sqrt(c + 1.0) * scale, 2.0 * kEstBlockKeys);
    return (uint64_t)ceil(c * scale + slack * (sig + 64.0));
}

// K12e: block s (level-3 bucket), thread e (level-2 child).  capc = the child's capacity,
// cap3[x*256+s] = shard x's capacity in bucket s; the child cursors cur2[s*256+e] (u32, offset
// in bucket s's Y region) with their limits lim2 and start copies init2; the shard cursors
// cur3[x*256+s] (offset in bucket s's X region), lim3, init3; r2[s] / r3[s] = bucket s's
// region sizes.  The last block to finish scans r3 / r2 into the region bases bases3 / bases2,
// zeroes the nzero work-list counters at zero and sets the last eligibility bit; block 0 of
// K3r then hands the eligibility word and the number of children with samples to the host
// (publish_elig).
// Ineligible (eflag bit 2): a child estimate + 4 sigma past kHxMax (K18c could not take it in
// one pass; capacities are clamped to kHxMax), a u8 wrap in K1e, every sample in one level-3 bucket (level 3 would copy; the exact
// plan skips that level), or X / Y outgrowing their buffers (capx / capy keys).
__global__ __launch_bounds__(kRadix) void k_est_plan(
    const uint32_t *__restrict__ part8, const uint32_t *__restrict__ part3,
    const uint32_t *__restrict__ msamp, uint32_t nwg, uint64_t n, double slack, uint64_t capx,
    uint64_t capy, uint32_t *__restrict__ capc, uint32_t *__restrict__ cap3,
    unsigned long long *__restrict__ r2, unsigned long long *__restrict__ r3,
    unsigned long long *__restrict__ bases3, unsigned long long *__restrict__ bases2,
    uint32_t *__restrict__ cur2, uint32_t *__restrict__ lim2, uint32_t *__restrict__ init2,
    uint32_t *__restrict__ cur3, uint32_t *__restrict__ lim3, uint32_t *__restrict__ init3,
    unsigned long long *__restrict__ zero, uint32_t nzero, uint32_t *__restrict__ eflag) {
    constexpr uint32_t G = kRadix / 64;  // thread groups, each over every G-th partial
    __shared__ uint32_t s_m, s_bad, s_last, s_ne, s_maxc;
    __shared__ uint32_t s_c[G][kRadix], s_3[kRadix / kShards][kShards];
    __shared__ unsigned long long s_w[kRadix / 64], s_c3[kShards];
    const uint32_t s = blockIdx.x, e = threadIdx.x, g = e >> 6, l = e & 63;
    if (e == 0) { s_m = 0; s_bad = 0; s_ne = 0; s_maxc = 0; }
    __syncthreads();
    static_assert(kEstWG <= kRadix && kEstWG % (kRadix / 8) == 0, "K12e geometry");
    // every load issued before any is used: the partial words, the shard counts, then the
    // per-workgroup sample totals (their adds used to wait for their own load first, and block 0's
    // summaries with their global atomics ran ahead of its partial loads -- both in front of the
    // kernel's one HBM round trip)
    // bucket s's 64 packed words of every partial: lane l reads word l of the partials
    // b = g, g + G, ..; four children per word
    uint32_t c4[4] = {0, 0, 0, 0};
    const uint32_t *pw = part8 + s * (kRadix / 4) + l;
    constexpr uint32_t NB = kEstWG / G;  // all of a thread's partial words in flight at once
    uint32_t pv[NB];
#pragma unroll
    for (uint32_t b = 0; b < NB; ++b) pv[b] = pw[(uint64_t)(g + b * G) * kEstPartWords];
    // shard counts of bucket s: thread (b0 = e >> 3, x = e & 7) over partials b0, b0 + 32, ..
    const uint32_t x3 = e & 7u, b0 = e >> 3;
    constexpr uint32_t NB3 = kEstWG / (kRadix / 8);
    uint32_t pv3[NB3];
#pragma unroll
    for (uint32_t b = 0; b < NB3; ++b)
        pv3[b] = part3[((uint64_t)s * kEstWG + b0 + b * (kRadix / 8)) * kShards + x3];
    const uint32_t mv = e < kEstWG ? msamp[e] : 0u;
#pragma unroll
    for (uint32_t b = 0; b < NB; ++b)
#pragma unroll
        for (int q = 0; q < 4; ++q) c4[q] += (pv[b] >> (8 * q)) & 255u;
#pragma unroll
    for (int q = 0; q < 4; ++q) s_c[g][4 * l + q] = c4[q];
    {
        uint32_t c3 = 0;
#pragma unroll
        for (uint32_t b = 0; b < NB3; ++b) c3 += pv3[b];
        s_3[b0][x3] = c3;
    }
    {  // the samples' total (one atomic a wave) and any wrapped counter
        const uint32_t tot = wave_incl_add(mv & 0x7fffffffu);
        const bool wrapped = __ballot((mv >> 31) != 0u) != 0;
        if (l == 63) {
            atomicAdd(&s_m, tot);
            if (wrapped) s_bad = 1;
        }
    }
    if (s == 0) {  // block 0: the samples' varying bits, min, max and any wrap, one atomic a wave
        uint32_t vy = 0, lo = ~0u, hi = 0, wr = 0;
        for (uint32_t b = e; b < kEstWG; b += kRadix) {
            vy |= msamp[kEstWG + b];
            lo = min(lo, msamp[2 * kEstWG + b]);
            hi = max(hi, msamp[3 * kEstWG + b]);
            wr |= msamp[b] >> 31;
        }
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) {
            vy |= (uint32_t)__shfl_xor((int)vy, o);
            lo = min(lo, (uint32_t)__shfl_xor((int)lo, o));
            hi = max(hi, (uint32_t)__shfl_xor((int)hi, o));
            wr |= (uint32_t)__shfl_xor((int)wr, o);
        }
        if ((e & 63) == 0) {
            if (vy) atomicOr(eflag + 5, vy);
            atomicMin(eflag + 6, lo);
            atomicMax(eflag + 7, hi);
            if (wr) atomicMax(eflag + 8, ~0u);  // wrapped: the child counts say nothing
        }
    }
    __syncthreads();
    uint32_t cnt = 0;
#pragma unroll
    for (uint32_t q = 0; q < G; ++q) cnt += s_c[q][e];
    const uint32_t m = s_m;
    const double scale = m ? (double)n / (double)m : 0.0;
    const uint64_t cap = est_cap(cnt, scale, slack);
    // A child is finished by K11e (<= kLocalMax keys) or, past that, by K18c's one-read
    // counting sort (kLocalMax < len <= kHxMax, K12g's list 0): a peaked block (Gaussian keys
    // after the offset retry) has children of ~27K keys near its mode, right at kLocalMax.
    // Eligible while the estimate + 4 sigma fits kHxMax; regions are the 6-sigma capacity
    // clamped to kHxMax (a child that outgrows it overflows: the exact plan sorts again).
    if ((double)cnt * scale + 4.0 * sqrt((double)cnt + 1.0) * scale + 64.0 > (double)kHxMax)
        s_bad = 1;
    uint32_t wmax = cnt;  // the largest child's samples (the runtime's retry), per block
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) wmax = max(wmax, (uint32_t)__shfl_xor((int)wmax, o));
    if ((e & 63) == 0) atomicMax(&s_maxc, wmax);
    const uint64_t sampled = __ballot(cnt > 0);  // (outside the branch: all lanes vote)
    if ((e & 63) == 0) atomicAdd(&s_ne, (uint32_t)__popcll(sampled));
    const uint32_t cc = (uint32_t)min(cap, (uint64_t)kHxMax);
    const uint32_t i = s * kRadix + e;
    capc[i] = cc;
    unsigned long long tot;
    const uint32_t off = (uint32_t)block_excl_scan32(cc, s_w, &tot);  // (cc <= kHxMax: sums < 2^28)
    cur2[i] = off;
    init2[i] = off;
    lim2[i] = off + cc;
    if (e < kShards) {
        uint32_t c3 = 0;
        for (uint32_t r = 0; r < kRadix / kShards; ++r) c3 += s_3[r][e];
        const uint64_t cp = est_cap(c3, scale, slack);
        cap3[e * kRadix + s] = (uint32_t)min(cp, (uint64_t)0xffffffffu);
        s_c3[e] = ((unsigned long long)c3 << 32) | min(cp, (uint64_t)0xffffffffu);
    }
    __syncthreads();
    if (e == 0) {
        unsigned long long r = 0, samp = 0;
        for (uint32_t x = 0; x < kShards; ++x) {
            const uint32_t j = x * kRadix + s, cx = (uint32_t)(s_c3[x] & 0xffffffffull);
            cur3[j] = (uint32_t)r;
            init3[j] = (uint32_t)r;
            lim3[j] = (uint32_t)(r + cx);
            r += cx;
            samp += s_c3[x] >> 32;
        }
        r2[s] = tot;
        r3[s] = r;
        if (m && samp == m) s_bad = 1;
        if (s_bad) atomicOr(eflag, 4u);
        atomicAdd(eflag + 4, s_ne);
        if (s_maxc) atomicMax(eflag + 8, s_maxc);
        __threadfence();
        s_last = atomicAdd(eflag + 3, 1u) == gridDim.x - 1;
    }
    __syncthreads();
    if (!s_last) return;
    __threadfence();
    unsigned long long tx, ty;
    const unsigned long long v3 = __hip_atomic_load(r3 + e, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const unsigned long long v2 = __hip_atomic_load(r2 + e, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    bases3[e] = block_excl_scan(v3, s_w, &tx);
    bases2[e] = block_excl_scan(v2, s_w, &ty);
    if (e < nzero) zero[e] = 0;
    if (e == 0 && (tx > capx || ty > capy)) atomicOr(eflag, 4u);
}


// K12f: K3a's tile descriptors.  Level-3 bucket s is the concatenation of its 8 pieces (shard
// x: keys [bases3[s] + init3[x*256+s], + their count, clamped to the region: an overflowed
// piece's excess went to the scratch tile)); its tiles cover that concatenation in kSweepTile
// steps, so a bucket has one partial tile, not one per piece (2048 half-full tiles cost K3a ~3 %).
// A tile inside one piece gets {first key, length, s}; one that crosses a piece boundary gets
// {virtual start, length, s | kStraddle} and K3a maps every key through the bucket's piece
// table pieces[s*8 + x] = {first key, virtual start, virtual end}.  Every block rebuilds the
// 256-bucket tile prefix in LDS and describes its 256 tiles; tp[256] = the tile total.
__global__ __launch_bounds__(256) void k_est_tiles(const uint32_t *__restrict__ cur3,
                                                   const uint32_t *__restrict__ init3,
                                                   const uint32_t *__restrict__ lim3,
                                                   const unsigned long long *__restrict__ bases3,
                                                   uint32_t max_tiles, const uint32_t *eflag,
                                                   uint32_t *__restrict__ tp,
                                                   TileDesc *__restrict__ desc,
                                                   TileDesc *__restrict__ pieces) {
    __shared__ uint32_t s_tp[kRadix + 1];
    __shared__ uint32_t s_w[4];
    if ((*eflag & 4u) || eflag[1]) return;  // ineligible, or level 3 overflowed
    const uint32_t tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    uint32_t vs[kShards + 1];  // bucket tid's piece starts in its concatenation
    vs[0] = 0;
#pragma unroll
    for (uint32_t x = 0; x < kShards; ++x) {
        const uint32_t j = x * kRadix + tid;
        vs[x + 1] = vs[x] + (min(cur3[j], lim3[j]) - init3[j]);
    }
    if (blockIdx.x == 0) {
#pragma unroll
        for (uint32_t x = 0; x < kShards; ++x)
            pieces[tid * kShards + x] = {bases3[tid] + init3[x * kRadix + tid], vs[x], vs[x + 1]};
    }
    const uint32_t nt = (vs[kShards] + kSweepTile - 1) / kSweepTile;
    const uint32_t v = wave_incl_add(nt);  // (DPP: no LDS round trip per step)
    if (lane == 63) s_w[w] = v;
    __syncthreads();
    uint32_t run = v - nt;
    for (uint32_t ww = 0; ww < w; ++ww) run += s_w[ww];
    s_tp[tid] = run;
    if (tid == 255) s_tp[kRadix] = run + nt;
    __syncthreads();
    const uint32_t total = s_tp[kRadix];
    if (blockIdx.x == 0 && tid == 0) tp[kRadix] = total;
    const uint32_t t = blockIdx.x * 256 + tid;
    if (t >= total || t >= max_tiles) return;
    uint32_t lo = 0, hi = kRadix;  // s_tp[lo] <= t < s_tp[hi]
    while (hi - lo > 1) {
        const uint32_t mid = (lo + hi) >> 1;
        if (s_tp[mid] <= t) lo = mid;
        else hi = mid;
    }
    const uint32_t sb = lo;
    uint32_t vb[kShards + 1];
    vb[0] = 0;
#pragma unroll
    for (uint32_t x = 0; x < kShards; ++x) {
        const uint32_t j = x * kRadix + sb;
        vb[x + 1] = vb[x] + (min(cur3[j], lim3[j]) - init3[j]);
    }
    const uint32_t v0 = (t - s_tp[sb]) * kSweepTile, len = min(vb[kShards] - v0, (uint32_t)kSweepTile);
    uint32_t x = 0;
#pragma unroll
    for (uint32_t q = 1; q < kShards; ++q) x += v0 >= vb[q];
    if (v0 + len <= vb[x + 1])
        desc[t] = {bases3[sb] + init3[x * kRadix + sb] + (v0 - vb[x]), len, sb};
    else
        desc[t] = {v0, len, sb | kStraddle};
}


// K12g: block s, thread e.  Exact sizes: child (s, e) holds cur2 - init2 keys, bucket s' holds
// sum_x (cur3 - init3) keys, so the child's output offset is the scan of the bucket totals
// before s plus the scan of its siblings before e.  Non-empty children go to the K11e class
// lists as {src = bases2[s] + init2, dst | len << 40}.  A child past its limit raises ovf and
// is not listed (K3a has flagged it already).  The list counters and the status words reach
// the host through publish_lists, run by block 0 of the K11e launch queued behind K12g.
// The entry's src carries the child's top 16 bits above bit 40 (Y holds only the low 16 bits):
// the ordered-u32 key (minus koff) of child (s, e) is pfx . s . e . rest, the digits sb bits
// below the constant prefix pfx of the shifted plan (K3r's check, from in[0]).
__global__ __launch_bounds__(kRadix) void k_est_classify(
    const uint32_t *__restrict__ cur2, const uint32_t *__restrict__ init2,
    const uint32_t *__restrict__ lim2, const uint32_t *__restrict__ cur3,
    const uint32_t *__restrict__ init3, const unsigned long long *__restrict__ bases2,
    WorkLists wl, uint32_t *__restrict__ eflag, const uint32_t *__restrict__ in, int sb,
    uint32_t koff) {
    constexpr int NL = kLocalClasses + 1;
    __shared__ unsigned long long s_w[kRadix / 64];
    __shared__ unsigned long long s_fb;
    __shared__ unsigned int s_n[NL];
    __shared__ unsigned long long s_keys[NL], s_max[NL], s_base[NL];
    const uint32_t s = blockIdx.x, e = threadIdx.x;
    unsigned long long *ctr = reinterpret_cast<unsigned long long *>(wl.ctr);
    // (the cursors loaded before the status word is looked at: every load in flight at once;
    // an ineligible plan's stale cursors are read, never used)
    const uint32_t i = s * kRadix + e;
    const uint32_t c0 = init2[i], c2 = cur2[i], l2 = lim2[i];
    uint32_t c3[kShards], i3[kShards];
#pragma unroll
    for (uint32_t x = 0; x < kShards; ++x) { c3[x] = cur3[x * kRadix + e]; i3[x] = init3[x * kRadix + e]; }
    if (!(*eflag & 4u)) {
        if (e < NL) { s_n[e] = 0; s_keys[e] = 0; s_max[e] = 0; }
        uint32_t te = 0;  // (bucket e's keys: at most the block's, < 2^32)
#pragma unroll
        for (uint32_t x = 0; x < kShards; ++x) te += c3[x] - i3[x];
        unsigned long long all;
        const unsigned long long fb = block_excl_scan32(te, s_w, &all);
        if (e == s) s_fb = fb;
        const uint32_t len = c2 - c0;
        const bool over = c2 > l2;
        if (over) atomicOr(eflag + 1, 1u);
        unsigned long long tot;
        const unsigned long long ex = block_excl_scan32(len, s_w, &tot);  // (syncs: s_fb visible)
        const unsigned long long dst = s_fb + ex;
        int which = -1;  // K11e class, or 0: past kLocalMax, K18c
        if (len > 0 && !over) {
            which = 0;
            for (int k = 1; k < NL && (k < kEstCx || sb >= 8); ++k)  // (kEstCx, gsort_kernels.h)
                if (len <= kLocalCap[k]) { which = k; break; }
        }
        unsigned int idx = 0;
        if (which >= 0) {
            idx = atomicAdd(&s_n[which], 1u);
            atomicAdd(&s_keys[which], (unsigned long long)len);
            atomicMax(&s_max[which], (unsigned long long)len);
        }
        __syncthreads();
        if (e < NL && s_n[e]) {
            s_base[e] = atomicAdd(&ctr[3 * e], (unsigned long long)s_n[e]);
            atomicAdd(&ctr[3 * e + 1], s_keys[e]);
            atomicMax(&ctr[3 * e + 2], s_max[e]);
        }
        __syncthreads();
        if (which >= 0) {
            unsigned long long *list = reinterpret_cast<unsigned long long *>(wl.list[which]);
            const unsigned long long j = s_base[which] + idx;
            const uint32_t pfx = sb ? ((in[0] ^ kFlip) - koff) >> (32 - sb) : 0u;
            const unsigned long long full = ((unsigned long long)pfx << (32 - sb)) |
                                            ((unsigned long long)s << (24 - sb)) |
                                            ((unsigned long long)e << (16 - sb));
            const unsigned long long top = (full >> 16) & 0xffffull;
            list[2 * j] = (bases2[s] + c0) | (top << 40);
            list[2 * j + 1] = dst | ((unsigned long long)len << 40);
        }
    }
}

// The K12g results for the host: the 15 work-list counters and the status words {eflag, ovf}
// into the mailbox, then seq (threads 0 .. 15 of one block; K12g has completed).
__device__ __forceinline__ void publish_lists(unsigned long long *mail,
                                              const unsigned long long *ctr,
                                              const uint32_t *eflag, unsigned long long seq) {
    constexpr uint32_t NC = 3 * (kLocalClasses + 1);
    const uint32_t e = threadIdx.x;
    if (e < NC) mail[kMailCtr + e] = ctr[e];
    if (e == NC) mail[kMailStatus] = *reinterpret_cast<const unsigned long long *>(eflag);
    __syncthreads();
    if (e == 0) mail_release(mail + kMailSeq, seq);
}

// K12p for the sampled plan when no K11e launch follows K12g directly.
__global__ __launch_bounds__(64) void k_publish_lists(unsigned long long *mail,
                                                      const unsigned long long *ctr,
                                                      const uint32_t *eflag,
                                                      unsigned long long seq) {
    publish_lists(mail, ctr, eflag, seq);
}

// K11e: K11 over a class list of the sampled plan: entry blockIdx.x = {src, dst | len << 40} is
// loaded from in + src, sorted on its low ndigits digits and stored flipped at out + dst.
// (A persistent form that read the entry count on the device was tried: inlined into its loop
// the sort took 177 VGPRs, under launch bounds it spilled; both ran at half speed.)
// Entry first + blockIdx.x, if below the class's entry count ctr[0]: the runtime launches the
// class it expects to hold most children right behind K12g with a grid of the sampled children
// (no host round trip in between), and the rest once it has read the counts.  With mail set,
// block 0 first hands K12g's counters and status to the host (publish_lists), off the kernels'
// critical path.
// The child's keys come from Y as their low 16 bits; the entry's src word carries the top 16.
template <int BLOCK, int ITEMS, bool ATOMIC, bool COPY = false, int ND = 0>
__global__ __launch_bounds__(BLOCK) void k_local_sort_e(const uint16_t *__restrict__ in,
                                                        uint32_t *__restrict__ out,
                                                        const unsigned long long *__restrict__ list,
                                                        const unsigned long long *__restrict__ ctr,
                                                        uint32_t first, int ndigits,
                                                        unsigned long long *mail,
                                                        const unsigned long long *ctr_all,
                                                        const uint32_t *eflag,
                                                        unsigned long long seq, uint32_t koff) {
    constexpr int WAVES = BLOCK / 64;
    constexpr int TILE = BLOCK * ITEMS;
    __shared__ uint32_t s_a[lds_slots(TILE)];
    __shared__ uint32_t s_wc[WAVES * kRadix];
    if (mail && blockIdx.x == 0) publish_lists(mail, ctr_all, eflag, seq);  // K12g is done
    const uint32_t i = first + blockIdx.x;
    if (i >= (uint32_t)*ctr) return;
    const uint64_t sw = list[2 * i];
    const uint64_t e = list[2 * i + 1];
    const uint32_t len = (uint32_t)(e >> 40), top = (uint32_t)(sw >> 40) << 16;
    if (threadIdx.x < kRadix) s_wc[threadIdx.x] = 0;
    uint32_t k[ITEMS];
    {
        const __amdgpu_buffer_rsrc_t rs = bucket_rsrc(in + (sw & ((1ull << 40) - 1)), len * 2u);
#pragma unroll
        for (int j = 0; j < ITEMS; ++j)
            k[j] = __builtin_amdgcn_raw_buffer_load_b16(rs, (j * BLOCK + (int)threadIdx.x) * 2, 0, 0);
#pragma unroll
        for (int j = 0; j < ITEMS; ++j) k[j] |= top;
    }
    uint32_t *dst = out + (e & ((1ull << 40) - 1));
    if (COPY) {  // every key of the child is one value (digits below a constant prefix)
        const __amdgpu_buffer_rsrc_t rs = bucket_rsrc(dst, len * 4u);
#pragma unroll
        for (int j = 0; j < ITEMS; ++j)
            __builtin_amdgcn_raw_buffer_store_b32((k[j] + koff) ^ kFlip, rs, (j * BLOCK + (int)threadIdx.x) * 4, 0, 0);
        return;
    }
    __syncthreads();
    // (ND: the digit count as a constant -- one straight-line pass pair, as K11g has)
    sort_bucket<BLOCK, ITEMS, ATOMIC>(k, len, ND ? ND : ndigits, dst, s_a, s_wc, koff);
}

// K11e's 16 896-key class on the packed body (sort_bucket16: two u16 keys per register, u16
// LDS slots -- three workgroups per CU instead of two, as K11g class 3); ndigits 1 or 2.
template <int BLOCK, int ITEMS, bool ATOMIC, int ND>
__global__ __launch_bounds__(BLOCK) void k_local_sort_e16(const uint16_t *__restrict__ in,
                                                          uint32_t *__restrict__ out,
                                                          const unsigned long long *__restrict__ list,
                                                          const unsigned long long *__restrict__ ctr,
                                                          uint32_t first, int ndigits,
                                                          unsigned long long *mail,
                                                          const unsigned long long *ctr_all,
                                                          const uint32_t *eflag,
                                                          unsigned long long seq, uint32_t koff) {
    constexpr int WAVES = BLOCK / 64;
    constexpr int TILE = BLOCK * ITEMS;
    constexpr int NP = (ITEMS + 1) / 2;
    __shared__ __attribute__((aligned(16))) uint16_t s_a[(lds_slots(TILE) + 1) & ~1];  // (s_wsum: u32 words in it)
    __shared__ uint32_t s_wc[WAVES * kRadix];
    if (mail && blockIdx.x == 0) publish_lists(mail, ctr_all, eflag, seq);  // K12g is done
    const uint32_t i = first + blockIdx.x;
    if (i >= (uint32_t)*ctr) return;
    const uint64_t sw = list[2 * i];
    const uint64_t e = list[2 * i + 1];
    const uint32_t len = (uint32_t)(e >> 40), top = (uint32_t)(sw >> 40) << 16;
    if (threadIdx.x < kRadix) s_wc[threadIdx.x] = 0;
    uint32_t kp[NP];
    {
        const uint16_t *src = in + (sw & ((1ull << 40) - 1));
        const uint32_t last = len ? len - 1 : 0u;
        uint16_t v[ITEMS];
#pragma unroll
        for (int j = 0; j < ITEMS; ++j) v[j] = src[min((uint32_t)(j * BLOCK) + threadIdx.x, last)];
#pragma unroll
        for (int q = 0; q < NP; ++q)
            kp[q] = (uint32_t)v[2 * q] | (2 * q + 1 < ITEMS ? (uint32_t)v[2 * q + 1] << 16 : 0u);
    }
    __syncthreads();
    (void)ndigits;
    sort_bucket16<BLOCK, ITEMS, ATOMIC>(kp, len, top, out + (e & ((1ull << 40) - 1)), s_a, s_wc,
                                        ND, koff);
}

// class geometries (block x items): class 3 as 1024 x 16 measured slower than 512 x 32 (local
// 30-bit keys K11e 0.80 -> 0.90 ms, receive 16 384-key buckets 0.73 -> 0.87 ms per 2^28 keys,
// round 4); class 2 as 256 x 36 needs 133 VGPRs (12 waves per CU).  Class 3 holds 512 x 33 =
// 16 896 keys (round 4): the P = 2 weak-scaling receive buckets (16 384 +- 128 keys) then all
// fit it instead of half of them going to K18c's 65 536 counters; 2 workgroups still fit a CU
// (76 KiB of LDS each)
constexpr int kC3Block = 512, kC3Items = 33;
constexpr int kC2Block = 512, kC2Items = 18;  // (1024 x 9: 1.36 -> 1.73 ms per 2^28-key sort, r05_ab_k11e_1024x9_rejected)

constexpr int cls_of(int block, int items) {
    return block * items == 16896 ? 3 : block * items == 9216 ? 2 : block * items == 4608 ? 1 : 4;
}

unsigned grid_for(uint64_t n, unsigned block, unsigned cap) {
    uint64_t g = (n + block - 1) / block;
    if (g < 1) g = 1;
    return (unsigned)(g < cap ? g : cap);
}

}  // namespace

// Every kernel of the library launches through launch_k.  With a launch timer set on the
// calling thread (the runtime's gsort_stats timing), the dispatch itself carries a fresh stop
// event (hipExtLaunchKernel), so timing a sort adds no marker packets between its kernels: a
// hipEventRecord between two kernels left ~5-8 us of idle, 4 % of a 2^28-key sort, and an
// attached start event ~5 us (tools/experiments/launch_gap.hip).
namespace {
thread_local LaunchTimer *tl_timer = nullptr;
}  // namespace

void set_launch_timer(LaunchTimer *t) { tl_timer = t; }

#ifdef GSORT_STAMPS
extern "C" __attribute__((visibility("default"))) int gsort_diag_stamps(void *d_buf) {
    return (int)hipMemcpyToSymbol(HIP_SYMBOL(g_stamps), &d_buf, sizeof(d_buf));
}
#endif

template <typename... KA, typename... A>
inline void launch_k(void (*k)(KA...), dim3 g, dim3 b, uint32_t shm, hipStream_t s, A... a) {
    hipEvent_t e1 = nullptr;
    if (LaunchTimer *t = tl_timer) {
        e1 = t->make(t->u);
        if (e1) t->last_stop = e1;
    }
    hipExtLaunchKernelGGL(k, g, b, shm, s, nullptr, e1, 0u, static_cast<KA>(a)...);
}

hipError_t launch_generate(int dist, uint64_t seed, uint64_t start, uint64_t n, int32_t *out,
                           hipStream_t s) {
    if (n == 0) return hipSuccess;
    launch_k(k_generate, grid_for(n, 256, 4096), 256, 0, s, dist, seed, start, n, out);
    return hipGetLastError();
}

hipError_t launch_tile_counts(const uint32_t *in, uint64_t n, int shift, bool flip,
                              uint32_t *tcounts, uint64_t *hist4, hipStream_t s) {
    if (n == 0) return hipSuccess;
    constexpr int B = 256;
    const uint32_t ntiles = (uint32_t)sweep_tiles(n);
    const unsigned g = ntiles < 2048 ? ntiles : 2048;
    const uint32_t fl = flip ? kFlip : 0u;
    auto *h = reinterpret_cast<unsigned long long *>(hist4);
    const bool vec = (reinterpret_cast<uintptr_t>(in) & 15) == 0;
    if (hist4) {
        if (shift != 0) return hipErrorInvalidValue;  // ALL4 counts tiles by digit 0
        if (vec) launch_k(k_tile_counts<B, true, true>, g, B, 0, s, in, n, 0, fl, tcounts, h, ntiles);
        else launch_k(k_tile_counts<B, true, false>, g, B, 0, s, in, n, 0, fl, tcounts, h, ntiles);
    } else {
        if (vec) launch_k(k_tile_counts<B, false, true>, g, B, 0, s, in, n, shift, fl, tcounts, h, ntiles);
        else launch_k(k_tile_counts<B, false, false>, g, B, 0, s, in, n, shift, fl, tcounts, h, ntiles);
    }
    return hipGetLastError();
}

hipError_t launch_scan_tiles(uint32_t *tcounts, uint64_t n, uint64_t *gsum, uint64_t *totals,
                             uint64_t *bases, hipStream_t s) {
    if (n == 0) return hipSuccess;
    const uint32_t ntiles = (uint32_t)sweep_tiles(n);
    const uint32_t ng = (uint32_t)scan_groups(n);
    auto *gs = reinterpret_cast<unsigned long long *>(gsum);
    auto *tot = reinterpret_cast<unsigned long long *>(totals);
    launch_k(k_scan_tiles, ng, kRadix, 0, s, tcounts, ntiles, gs);
    launch_k(k_scan_groups, kRadix, 1024, 0, s, gs, ng, tot);
    launch_k(k_scan_digits, 1, kRadix, 0, s, tot, reinterpret_cast<unsigned long long *>(bases));
    return hipGetLastError();
}

hipError_t launch_scatter(const uint32_t *in, uint32_t *out, uint64_t n, int shift,
                          const uint32_t *toff, const uint64_t *gpfx, const uint64_t *bases,
                          bool flip_in, bool flip_out, hipStream_t s, const uint32_t *vin,
                          uint32_t *vout) {
    if (n == 0) return hipSuccess;
    const unsigned g = (unsigned)sweep_tiles(n);
    auto *gp = reinterpret_cast<const unsigned long long *>(gpfx);
    auto *bs = reinterpret_cast<const unsigned long long *>(bases);
    constexpr int B = kSweepBlock, I = kSweepItems;
    if (vin) {  // the reference-compat key-value pass (keys are never flipped there)
        if (flip_in || flip_out || !vout) return hipErrorInvalidValue;
        launch_k(k_scatter<B, I, false, false, true>, g, B, 0, s, in, out, n, shift, toff, gp, bs,
                                                            vin, vout);
    } else if (flip_in && flip_out)
        launch_k(k_scatter<B, I, true, true>, g, B, 0, s, in, out, n, shift, toff, gp, bs, nullptr,
                 nullptr);
    else if (flip_in)
        launch_k(k_scatter<B, I, true, false>, g, B, 0, s, in, out, n, shift, toff, gp, bs, nullptr,
                 nullptr);
    else if (flip_out)
        launch_k(k_scatter<B, I, false, true>, g, B, 0, s, in, out, n, shift, toff, gp, bs, nullptr,
                 nullptr);
    else
        launch_k(k_scatter<B, I, false, false>, g, B, 0, s, in, out, n, shift, toff, gp, bs, nullptr,
                 nullptr);
    return hipGetLastError();
}

hipError_t launch_place(const uint32_t *recv, uint32_t *out, const uint64_t *segs, int nseg,
                        uint64_t n_out, uint64_t *hist, int next_shift, bool flip_out,
                        hipStream_t s) {
    if (n_out == 0 || nseg == 0) return hipSuccess;
    constexpr int B = 256, I = 16;
    const unsigned g = (unsigned)((n_out + B * I - 1) / (B * I));
    launch_k(k_place<B, I>, g, B, 0, s, recv, out, reinterpret_cast<const unsigned long long *>(segs),
                                  nseg, n_out, reinterpret_cast<unsigned long long *>(hist),
                                  next_shift, flip_out ? kFlip : 0u);
    return hipGetLastError();
}

hipError_t launch_fingerprint(const int32_t *keys, uint64_t n, unsigned long long *acc,
                              hipStream_t s) {
    if (n == 0) return hipSuccess;
    launch_k(k_fingerprint, grid_for(n, 256, 2048), 256, 0, s, keys, n, acc);
    return hipGetLastError();
}

hipError_t launch_count_below(const int32_t *sorted, uint64_t n, const uint64_t *xs, int m,
                              uint64_t *out, hipStream_t s) {
    if (m <= 0) return hipSuccess;
    launch_k(k_count_below, (m + 255) / 256, 256, 0, s, sorted, n,
                                                  reinterpret_cast<const unsigned long long *>(xs),
                                                  m, reinterpret_cast<unsigned long long *>(out));
    return hipGetLastError();
}

hipError_t launch_regular_sample(const int32_t *sorted, uint64_t interval, int k, int32_t *out,
                                 hipStream_t s) {
    launch_k(k_regular_sample, 1, 64 * ((k + 63) / 64), 0, s, sorted, interval, k, out);
    return hipGetLastError();
}

hipError_t launch_select_splitters(const int32_t *samples, int m, int k, int nsplit,
                                   int32_t *splitters, hipStream_t s) {
    if (m > 1024 || nsplit <= 0) return nsplit <= 0 ? hipSuccess : hipErrorInvalidValue;
    launch_k(k_select_splitters, 1, 1024, 0, s, samples, m, k, nsplit, splitters);
    return hipGetLastError();
}

hipError_t launch_bucket_bounds(const int32_t *sorted, uint64_t n, const int32_t *splitters,
                                int nsplit, uint64_t *bounds, hipStream_t s, bool strict) {
    if (nsplit <= 0) return hipSuccess;
    launch_k(k_bucket_bounds, nsplit, 64, 0, s, sorted, n, splitters,
                                          reinterpret_cast<unsigned long long *>(bounds),
                                          strict ? 1 : 0);
    return hipGetLastError();
}

hipError_t launch_tile_counts1(const uint32_t *in, uint64_t n, int shift, bool flip,
                               uint32_t *tcounts, hipStream_t s) {
    if (n == 0) return hipSuccess;
    const unsigned g = (unsigned)sweep_tiles(n);
    if (flip)
        launch_k(k_seg_counts<512, false, true>, g, 512, 0, s, in, n, nullptr, nullptr, nullptr, nullptr,
                                                         0, shift, tcounts);
    else
        launch_k(k_seg_counts<512, false, false>, g, 512, 0, s, in, n, nullptr, nullptr, nullptr,
                                                          nullptr, 0, shift, tcounts);
    return hipGetLastError();
}

hipError_t launch_partition(const uint32_t *in, uint32_t *out, uint64_t n, int shift,
                            const uint32_t *toff, const uint64_t *gpfx, const uint64_t *bases,
                            bool flip_in, hipStream_t s) {
    if (n == 0) return hipSuccess;
    const unsigned g = (unsigned)sweep_tiles(n);
    auto *gp = reinterpret_cast<const unsigned long long *>(gpfx);
    auto *bs = reinterpret_cast<const unsigned long long *>(bases);
    constexpr int B = kPartBlock, I = kSweepTile / kPartBlock;
    if (flip_in) launch_k(k_partition<B, I, true>, g, B, 0, s, in, out, n, shift, toff, gp, bs);
    else launch_k(k_partition<B, I, false>, g, B, 0, s, in, out, n, shift, toff, gp, bs);
    return hipGetLastError();
}

hipError_t launch_classify_buckets(const uint64_t *bases, const uint64_t *totals,
                                   const WorkLists &wl, hipStream_t s) {
    using ull = unsigned long long;
    launch_k(k_classify_buckets, 1, kRadix, 0, s, reinterpret_cast<const ull *>(bases),
                                            reinterpret_cast<const ull *>(totals), wl);
    return hipGetLastError();
}

hipError_t launch_seg_count(const SegPass &sp, hipStream_t s) {
    using ull = unsigned long long;
    if (sp.nseg == 0) return hipSuccess;
    const ull *segs = reinterpret_cast<const ull *>(sp.segs);
    ull *gsum = reinterpret_cast<ull *>(sp.gsum);
    launch_k(k_seg_plan, 1, 1024, 0, s, segs, sp.nseg, sp.tpfx, sp.gpfx);
    launch_k(k_seg_map, sp.nseg, 256, 0, s, sp.tpfx, sp.gpfx, sp.segmap, sp.groupmap);
    if (sp.flip_in)
        launch_k(k_seg_counts<512, true, true>, sp.max_tiles, 512, 0, s,
            sp.in, 0, segs, sp.tpfx, sp.gpfx, sp.segmap, sp.nseg, sp.shift, sp.tcounts);
    else
        launch_k(k_seg_counts<512, true, false>, sp.max_tiles, 512, 0, s,
            sp.in, 0, segs, sp.tpfx, sp.gpfx, sp.segmap, sp.nseg, sp.shift, sp.tcounts);
    launch_k(k_seg_scan_tiles, sp.max_groups, kRadix, 0, s, sp.tcounts, sp.tpfx, sp.gpfx, sp.groupmap,
                                                      sp.nseg, gsum);
    launch_k(k_seg_scan_groups, sp.nseg, kRadix, 0, s, gsum, segs, sp.gpfx,
                                                 reinterpret_cast<ull *>(sp.cstart), sp.lists);
    return hipGetLastError();
}

hipError_t launch_seg_partition(const SegPass &sp, hipStream_t s) {
    using ull = unsigned long long;
    if (sp.nseg == 0) return hipSuccess;
    const ull *segs = reinterpret_cast<const ull *>(sp.segs);
    ull *gsum = reinterpret_cast<ull *>(sp.gsum);
    constexpr int B = kPartBlock, I = kSweepTile / kPartBlock;
    if (sp.flip_in) {  // level 1 straight from the int32 input (levels 3 and 2 trivial)
        if (sp.out16 || sp.flip_out) return hipErrorInvalidValue;
        launch_k(k_seg_partition<B, I, false, uint32_t, true>, sp.max_tiles, B, 0, s,
            sp.in, sp.out, sp.shift, sp.tcounts, gsum, reinterpret_cast<const ull *>(sp.cstart),
            segs, sp.tpfx, sp.gpfx, sp.segmap, sp.nseg);
    } else if (sp.out16)
        launch_k(k_seg_partition<B, I, false, uint16_t>, sp.max_tiles, B, 0, s,
            sp.in, sp.out16, sp.shift, sp.tcounts, gsum, reinterpret_cast<const ull *>(sp.cstart),
            segs, sp.tpfx, sp.gpfx, sp.segmap, sp.nseg);
    else if (sp.flip_out)
        launch_k(k_seg_partition<B, I, true>, sp.max_tiles, B, 0, s,
            sp.in, sp.out, sp.shift, sp.tcounts, gsum, reinterpret_cast<const ull *>(sp.cstart),
            segs, sp.tpfx, sp.gpfx, sp.segmap, sp.nseg);
    else
        launch_k(k_seg_partition<B, I, false>, sp.max_tiles, B, 0, s,
            sp.in, sp.out, sp.shift, sp.tcounts, gsum, reinterpret_cast<const ull *>(sp.cstart),
            segs, sp.tpfx, sp.gpfx, sp.segmap, sp.nseg);
    return hipGetLastError();
}

hipError_t launch_hist16(const uint32_t *in, uint64_t n, bool flip, uint32_t *part, uint64_t *fix,
                         uint32_t *nblk, hipStream_t s) {
    if (n == 0) return hipErrorInvalidValue;
    const uint64_t pairs = (sweep_tiles(n) + 1) / 2;
    // a multiple of kShards (shard of tile pair p == p % 8 == the counting workgroup % 8)
    const uint64_t g = std::min<uint64_t>((pairs + kShards - 1) / kShards * kShards, kH16Blocks);
    static_assert(kH16Blocks % kShards == 0, "K1h grid");
    *nblk = (uint32_t)g;
    auto *fx = reinterpret_cast<unsigned long long *>(fix);
    if (flip) launch_k(k_hist16<1024, true>, (unsigned)g, 1024, 0, s, in, n, part, fx);
    else launch_k(k_hist16<1024, false>, (unsigned)g, 1024, 0, s, in, n, part, fx);
    return hipGetLastError();
}

hipError_t launch_plan16(const uint32_t *part, uint32_t nblk, uint64_t *fix, uint64_t n,
                         bool force, uint64_t *ccount, uint64_t *t3, uint64_t *tot,
                         uint64_t *bases, uint64_t *totals, uint64_t *cstart, uint32_t *cur,
                         uint32_t *cur3, uint32_t *tpfx, const WorkLists &wl2,
                         const WorkLists &wl3, uint64_t *zero, uint32_t nzero, uint32_t *flags,
                         hipStream_t s) {
    using ull = unsigned long long;
    if (nblk % kShards || nzero > kRadix) return hipErrorInvalidValue;
    launch_k(k_plan16_count, kRadix, kRadix, 0, s, part, nblk, reinterpret_cast<ull *>(fix),
             reinterpret_cast<ull *>(ccount), reinterpret_cast<ull *>(t3),
             reinterpret_cast<ull *>(tot), reinterpret_cast<ull *>(zero), zero ? nzero : 0u);
    launch_k(k_plan16_place, kRadix, kRadix, 0, s,
        reinterpret_cast<const ull *>(ccount), reinterpret_cast<const ull *>(t3),
        reinterpret_cast<const ull *>(tot), n, force ? 1 : 0, reinterpret_cast<ull *>(bases),
        reinterpret_cast<ull *>(totals), reinterpret_cast<ull *>(cstart), cur, cur3, tpfx, wl2,
        wl3, flags);
    return hipGetLastError();
}

hipError_t launch_partition3r(const uint32_t *in, uint32_t *out, uint64_t n, uint32_t *cur3,
                              const uint64_t *bases, const uint32_t *flags, hipStream_t s) {
    using ull = unsigned long long;
    if (n == 0) return hipSuccess;
    constexpr int B = kPartBlock, I = kSweepTile / kPartBlock;
    const uint64_t pairs = (sweep_tiles(n) + 1) / 2;
    launch_k(k_partition_res<B, I, true, true>, (unsigned)pairs, B, 0, s,
        in, out, n, nullptr, nullptr, reinterpret_cast<const ull *>(bases), cur3, flags,
        (const uint32_t *)nullptr, (const uint32_t *)nullptr, (uint32_t *)nullptr,
        (uint32_t *)nullptr, (const TileDesc *)nullptr, (unsigned long long *)nullptr, 0ull, 0, 0u);
    return hipGetLastError();
}

hipError_t launch_partition2r(const uint32_t *in, uint32_t *out, uint16_t *out16, uint64_t n,
                              const uint32_t *tpfx, void *tdesc, const uint64_t *bases,
                              const uint64_t *totals, uint32_t *cur, const uint32_t *flags,
                              const uint32_t *raw, hipStream_t s) {
    using ull = unsigned long long;
    if (n == 0) return hipSuccess;
    constexpr int B = kPartBlock, I = kSweepTile / kPartBlock;
    const ull *bs = reinterpret_cast<const ull *>(bases);
    const ull *tt = reinterpret_cast<const ull *>(totals);
    // the level-2 tiles number at most sweep_tiles(n) + 256 (one partial tile per bucket)
    const uint32_t max_tiles = (uint32_t)(sweep_tiles(n) + kRadix);
    TileDesc *desc = static_cast<TileDesc *>(tdesc);
    launch_k(k_tile_desc, (max_tiles + 255) / 256, 256, 0, s, tpfx, bs, tt, max_tiles, desc);
    const unsigned g2 = (max_tiles + 1) / 2;
    if (out16)
        launch_k(k_partition_res<B, I, false, false, uint16_t>, g2, B, 0, s, in, out16, n, tpfx,
                 desc, bs, cur, flags, raw, (const uint32_t *)nullptr, (uint32_t *)nullptr,
                 (uint16_t *)nullptr, (const TileDesc *)nullptr, (unsigned long long *)nullptr,
                 0ull, 0, 0u);
    else
        launch_k(k_partition_res<B, I, false, false>, g2, B, 0, s, in, out, n, tpfx, desc, bs,
                 cur, flags, raw, (const uint32_t *)nullptr, (uint32_t *)nullptr,
                 (uint32_t *)nullptr, (const TileDesc *)nullptr, (unsigned long long *)nullptr, 0ull, 0, 0u);
    return hipGetLastError();
}

hipError_t launch_unpack16(const uint16_t *in, uint64_t n, uint32_t h, int32_t *out,
                           hipStream_t s) {
    if (n == 0) return hipSuccess;
    launch_k(k_unpack16, grid_for(n, 256, 4096), 256, 0, s, in, n, h, out);
    return hipGetLastError();
}

hipError_t launch_gb_from_plan(const uint64_t *bases, const uint64_t *totals,
                               const uint64_t *segs, uint32_t nseg, const uint64_t *cstart,
                               uint64_t n, uint64_t *gb, hipStream_t s) {
    using ull = unsigned long long;
    launch_k(k_gb_from_plan, kRadix, kRadix, 0, s,
        reinterpret_cast<const ull *>(bases), reinterpret_cast<const ull *>(totals),
        reinterpret_cast<const ull *>(segs), nseg, reinterpret_cast<const ull *>(cstart), n,
        reinterpret_cast<ull *>(gb));
    return hipGetLastError();
}

hipError_t launch_count_below16(const uint16_t *a, const uint64_t *gb, const uint64_t *xs,
                                int m, uint64_t *out, hipStream_t s) {
    using ull = unsigned long long;
    if (m <= 0) return hipSuccess;
    launch_k(k_count_below16, (m + 255) / 256, 256, 0, s, a, reinterpret_cast<const ull *>(gb),
                                                    reinterpret_cast<const ull *>(xs), m,
                                                    reinterpret_cast<ull *>(out));
    return hipGetLastError();
}

// K13s (radix select, a round decided on the device): boundary q = block, digit d = thread.
// all = the P all-gathered rows of nb x M counts, all[p][q][d] = rank p's keys below
// prefix[q] + (d << shift); the round's digit is the largest d < 256 whose global count stays
// <= g[q] (the counts grow with d), prefix[q] gains it, and the next round's M thresholds
// prefix[q] + (d << (shift - 8)) go to xs.  Boundaries at the end (g[q] >= N) keep their prefix.
__global__ __launch_bounds__(256) void k_select_digit(const unsigned long long *__restrict__ all,
                                                      int W,
                                                      const unsigned long long *__restrict__ g,
                                                      unsigned long long N, int P, int nb, int M,
                                                      int shift, unsigned long long *prefix,
                                                      unsigned long long *__restrict__ xs) {
    __shared__ uint32_t s_ok;
    const int q = blockIdx.x, d = threadIdx.x;
    unsigned long long below = 0;  // (rank p's row: W words, boundary q's M counts at q * M)
    for (int p = 0; p < P; ++p) below += all[(size_t)p * W + (size_t)q * M + d];
    const unsigned long long gq = g[q], p0 = prefix[q];
    if (d == 0) s_ok = 0;
    __syncthreads();
    const uint64_t okm = __ballot(below <= gq);
    if ((d & 63) == 0) atomicAdd(&s_ok, (uint32_t)__popcll(okm));
    __syncthreads();
    const uint32_t best = s_ok ? s_ok - 1 : 0;
    const unsigned long long pf = gq >= N ? p0 : p0 + ((unsigned long long)best << shift);
    if (d == 0) prefix[q] = pf;
    if (shift >= 8)  // (the last round leaves the boundary keys; no next thresholds)
        for (int j = d; j < M; j += 256) xs[(size_t)q * M + j] = pf + ((unsigned long long)j << (shift - 8));
}

// K13g: after the second select round every boundary's 16-bit group h_q = prefix[q] >> 16 is
// known on the device; block q sorts its group in place in the packed send buffer (u16 low
// halves, gb = the 16-bit bucket bounds) so that rounds 3 and 4 can binary-search it and the
// cut splits it by value -- with no host round trip.  Boundaries sharing a group
// (consecutive q: the boundary keys grow with q) leave it to the first of them; a boundary at
// the block's end (g[q] >= N) has none.  A group past this kernel's 32 768 keys is left as it
// is and flagged in big[q] (every block writes its flag, 0 or 1; the rounds' all-gathered count
// rows carry the flags to every rank, and the runtime then sorts such groups on the host path
// and repeats rounds 3 and 4).
template <bool ATOMIC>
__global__ __launch_bounds__(1024) void k_boundary_sort16(uint16_t *__restrict__ pack,
                                                          const unsigned long long *__restrict__ gb,
                                                          const unsigned long long *__restrict__ prefix,
                                                          const unsigned long long *__restrict__ g,
                                                          unsigned long long N,
                                                          unsigned long long *__restrict__ big) {
    constexpr int BLOCK = 1024, ITEMS = 32, TILE = BLOCK * ITEMS;
    __shared__ uint32_t s_a[lds_slots(TILE)];
    __shared__ uint32_t s_wc[(BLOCK / 64) * kRadix];
    const int q = blockIdx.x;
    const unsigned long long h = prefix[q] >> 16;
    const bool mine = g[q] < N && h < kBuckets16 &&
                      !(q > 0 && g[q - 1] < N && (prefix[q - 1] >> 16) == h);
    const unsigned long long a = mine ? gb[h] : 0ull, b = mine ? gb[h + 1] : 0ull;
    const bool too_big = b > a && b - a > (unsigned long long)TILE;
    if (threadIdx.x == 0) big[q] = too_big ? 1ull : 0ull;
    if (b <= a || too_big) return;
    const uint32_t len = (uint32_t)(b - a), top = (uint32_t)h << 16;
    if (threadIdx.x < kRadix) s_wc[threadIdx.x] = 0;
    uint32_t k[ITEMS];
    const __amdgpu_buffer_rsrc_t rs = bucket_rsrc(pack + a, len * 2u);
#pragma unroll
    for (int j = 0; j < ITEMS; ++j)
        k[j] = top | __builtin_amdgcn_raw_buffer_load_b16(rs, (j * BLOCK + (int)threadIdx.x) * 2, 0, 0);
    __syncthreads();
    sort_bucket<BLOCK, ITEMS, ATOMIC, true>(k, len, 2, reinterpret_cast<uint32_t *>(pack + a), s_a,
                                            s_wc);
}

hipError_t launch_boundary_sort16(uint16_t *pack, const uint64_t *gb, const uint64_t *prefix,
                                  const uint64_t *g, uint64_t N, int nb, bool atomic_rank,
                                  uint64_t *big, hipStream_t s) {
    using ull = unsigned long long;
    if (nb <= 0) return hipSuccess;
    if (atomic_rank)
        launch_k(k_boundary_sort16<true>, nb, 1024, 0, s, pack, reinterpret_cast<const ull *>(gb),
                 reinterpret_cast<const ull *>(prefix), reinterpret_cast<const ull *>(g), (ull)N,
                 reinterpret_cast<ull *>(big));
    else
        launch_k(k_boundary_sort16<false>, nb, 1024, 0, s, pack, reinterpret_cast<const ull *>(gb),
                 reinterpret_cast<const ull *>(prefix), reinterpret_cast<const ull *>(g), (ull)N,
                 reinterpret_cast<ull *>(big));
    return hipGetLastError();
}

// ---- sample sort on the grouped (packed) block: the reference's regular samples and bucket
// bounds without sorting the block (mpi_sample_sort.c:85-105, :148-155) ---------
// K4g: sample i sits at position x = i * interval of the sorted block (mpi_sample_sort.c:95);
// in the grouped block that is the (x - gb[h])-th smallest key of group h, gb[h] <= x <
// gb[h + 1].  pref[i] = h << 16 and g[i] = 0 make K13g sort exactly those groups in place
// (ascending i gives ascending h, so K13g's shared-group skip applies).
__global__ __launch_bounds__(128) void k_sample_groups(const unsigned long long *__restrict__ gb,
                                                       unsigned long long interval, int k,
                                                       unsigned long long *__restrict__ pref,
                                                       unsigned long long *__restrict__ g) {
    const int i = threadIdx.x;
    if (i >= k) return;
    const unsigned long long x = (unsigned long long)i * interval;
    uint32_t lo = 0, hi = kBuckets16;  // the last h with gb[h] <= x lies in [lo, hi); gb[0] = 0
    while (hi - lo > 1) {
        const uint32_t mid = (lo + hi) >> 1;
        if (gb[mid] <= x) lo = mid; else hi = mid;
    }
    pref[i] = (unsigned long long)lo << 16;
    g[i] = 0;
}

// K4r: the samples from their sorted groups, int32 (mpi_sample_sort.c:101-103).
__global__ __launch_bounds__(128) void k_read_samples16(const uint16_t *__restrict__ pack,
                                                        const unsigned long long *__restrict__ pref,
                                                        unsigned long long interval, int k,
                                                        int32_t *__restrict__ out) {
    const int i = threadIdx.x;
    if (i >= k) return;
    const uint32_t key = (uint32_t)pref[i] | (uint32_t)pack[(unsigned long long)i * interval];
    out[i] = (int32_t)(key ^ 0x80000000u);
}

// K6g: splitter j's group for K13g (pref[j] = its top 16 bits << 16, g[j] = 0) and the
// thresholds of count_below16: xs[j] = ord(s_j) + 1 (keys <= s_j: the reference's bucket rule,
// mpi_sample_sort.c:150), xs[S + j] = ord(s_j) (keys < s_j: the duplicate-aware cut).
__global__ __launch_bounds__(64) void k_splitter_groups(const int32_t *__restrict__ spl, int S,
                                                        unsigned long long *__restrict__ pref,
                                                        unsigned long long *__restrict__ g,
                                                        unsigned long long *__restrict__ xs) {
    for (int j = threadIdx.x; j < S; j += 64) {
        const unsigned long long o = (uint32_t)spl[j] ^ 0x80000000u;
        pref[j] = o >> 16 << 16;
        g[j] = 0;
        xs[j] = o + 1;  // (2^32 for the largest key: count_below16 answers n)
        xs[S + j] = o;
    }
}

hipError_t launch_sample_groups(const uint64_t *gb, uint64_t interval, int k, uint64_t *pref,
                                uint64_t *g, hipStream_t s) {
    using ull = unsigned long long;
    if (k <= 0) return hipSuccess;
    if (k > 128) return hipErrorInvalidValue;
    launch_k(k_sample_groups, 1, 128, 0, s, reinterpret_cast<const ull *>(gb), (ull)interval, k,
             reinterpret_cast<ull *>(pref), reinterpret_cast<ull *>(g));
    return hipGetLastError();
}

hipError_t launch_read_samples16(const uint16_t *pack, const uint64_t *pref, uint64_t interval,
                                 int k, int32_t *out, hipStream_t s) {
    using ull = unsigned long long;
    if (k <= 0) return hipSuccess;
    if (k > 128) return hipErrorInvalidValue;
    launch_k(k_read_samples16, 1, 128, 0, s, pack, reinterpret_cast<const ull *>(pref),
             (ull)interval, k, out);
    return hipGetLastError();
}

hipError_t launch_splitter_groups(const int32_t *spl, int S, uint64_t *pref, uint64_t *g,
                                  uint64_t *xs, hipStream_t s) {
    using ull = unsigned long long;
    if (S <= 0) return hipSuccess;
    launch_k(k_splitter_groups, 1, 64, 0, s, spl, S, reinterpret_cast<ull *>(pref),
             reinterpret_cast<ull *>(g), reinterpret_cast<ull *>(xs));
    return hipGetLastError();
}

hipError_t launch_select_digit(const uint64_t *all, int W, const uint64_t *g, uint64_t N, int P,
                               int nb, int M, int shift, uint64_t *prefix, uint64_t *xs,
                               hipStream_t s) {
    using ull = unsigned long long;
    if (nb <= 0) return hipSuccess;
    if (shift < 0 || shift > 24 || shift % 8 || M < 256 || W < nb * M) return hipErrorInvalidValue;
    launch_k(k_select_digit, nb, 256, 0, s, reinterpret_cast<const ull *>(all), W,
             reinterpret_cast<const ull *>(g), (ull)N, P, nb, M, shift,
             reinterpret_cast<ull *>(prefix), reinterpret_cast<ull *>(xs));
    return hipGetLastError();
}

hipError_t launch_local_sort(const uint32_t *in, uint32_t *out, const uint64_t *list,
                             uint32_t nlist, int cls, int ndigits, bool flip_in,
                             bool atomic_rank, hipStream_t s) {
    if (nlist == 0) return hipSuccess;
    if (ndigits < 1 || ndigits > 4 || cls < 1 || cls > kLocalClasses) return hipErrorInvalidValue;
    auto *l = reinterpret_cast<const unsigned long long *>(list);
#define GSORT_K11(B, I)                                                                        \
    do {                                                                                       \
        static_assert((uint64_t)B * I == kLocalCap[cls_of(B, I)], "class geometry");          \
        if (atomic_rank) {                                                                     \
            if (flip_in) launch_k(k_local_sort<B, I, true, true>, nlist, B, 0, s, in, out, l, ndigits); \
            else launch_k(k_local_sort<B, I, false, true>, nlist, B, 0, s, in, out, l, ndigits);        \
        } else {                                                                               \
            if (flip_in) launch_k(k_local_sort<B, I, true, false>, nlist, B, 0, s, in, out, l, ndigits); \
            else launch_k(k_local_sort<B, I, false, false>, nlist, B, 0, s, in, out, l, ndigits);       \
        }                                                                                      \
    } while (0)
    switch (cls) {
        case 1: GSORT_K11(256, 18); break;
        case 2: GSORT_K11(kC2Block, kC2Items); break;
        case 3: GSORT_K11(kC3Block, kC3Items); break;
        default: GSORT_K11(1024, 32); break;
    }
#undef GSORT_K11
    return hipGetLastError();
}

hipError_t launch_run_bounds(const int32_t *recv, const uint64_t *roff, const uint64_t *rlen,
                             int P, uint64_t *pos, hipStream_t s) {
    using ull = unsigned long long;
    if (P < 1 || P > 64) return hipErrorInvalidValue;
    const uint64_t m = (uint64_t)P * (kBuckets16 + 1);
    launch_k(k_run_bounds, (unsigned)((m + 255) / 256), 256, 0, s,
        recv, reinterpret_cast<const ull *>(roff), reinterpret_cast<const ull *>(rlen), P,
        reinterpret_cast<ull *>(pos));
    return hipGetLastError();
}

hipError_t launch_pos_from_meta(const uint32_t *meta, const uint64_t *moff, uint32_t h_lo,
                                uint32_t nh, int P, uint64_t *pos, uint64_t *scratch,
                                hipStream_t s) {
    using ull = unsigned long long;
    if (P < 1 || P > 64) return hipErrorInvalidValue;
    const MetaCounts gen{meta, reinterpret_cast<const ull *>(moff), h_lo, nh};
    ull *part = reinterpret_cast<ull *>(scratch);
    launch_k(k_rowscan_reduce<decltype(gen)>, dim3(kScanBlocks, P), 1024, 0, s, gen, part,
             (ull *)nullptr, 0u);
    launch_k(k_rowscan_apply<decltype(gen)>, dim3(kScanBlocks, P), 1024, 0, s, gen, part, reinterpret_cast<ull *>(pos),
                                                          kBuckets16 + 1, (ull *)nullptr);
    return hipGetLastError();
}

hipError_t launch_recv_plan_from_meta(const uint32_t *meta, const uint64_t *moff, uint32_t h_lo,
                                     uint32_t nh, int P, uint64_t *pos, uint64_t *bstart,
                                     uint64_t *scratch, hipStream_t s, uint64_t *zero,
                                     uint32_t nzero, uint32_t epoch) {
    using ull = unsigned long long;
    if (P < 1 || P > 64 || nzero > 1024) return hipErrorInvalidValue;
    const MetaCountsSum gen{MetaCounts{meta, reinterpret_cast<const ull *>(moff), h_lo, nh},
                            (uint32_t)P};
    ull *status = reinterpret_cast<ull *>(scratch);
    unsigned int *ticket = reinterpret_cast<unsigned int *>(scratch + kRecvScanStatusWords);
    launch_k(k_rowscan_lookback<decltype(gen)>, dim3(kScanBlocks, P + 1), 1024, 0, s, gen, status,
             ticket, epoch, reinterpret_cast<ull *>(pos), (uint64_t)kBuckets16 + 1,
             reinterpret_cast<ull *>(bstart), reinterpret_cast<ull *>(zero), nzero);
    return hipGetLastError();
}

hipError_t launch_recv_bounds(const uint64_t *pos, int P, uint64_t *bsize, uint64_t *bstart,
                              uint64_t *scratch, hipStream_t s) {
    using ull = unsigned long long;
    launch_k(k_bucket_sizes, kBuckets16 / 256, 256, 0, s, reinterpret_cast<const ull *>(pos), P,
                                                     reinterpret_cast<ull *>(bsize));
    const RowValues gen{reinterpret_cast<const ull *>(bsize)};
    ull *part = reinterpret_cast<ull *>(scratch);
    launch_k(k_rowscan_reduce<decltype(gen)>, dim3(kScanBlocks, 1), 1024, 0, s, gen, part,
             (ull *)nullptr, 0u);
    launch_k(k_rowscan_apply<decltype(gen)>, dim3(kScanBlocks, 1), 1024, 0, s, gen, part, reinterpret_cast<ull *>(bstart),
                                                          kBuckets16 + 1, (ull *)nullptr);
    return hipGetLastError();
}

hipError_t launch_classify_range(const uint64_t *bsize, const uint64_t *bstart,
                                 const WorkLists &wl, uint32_t h0, uint32_t h1, hipStream_t s) {
    using ull = unsigned long long;
    launch_k(k_classify_gather, kBuckets16 / kRadix, kRadix, 0, s,
        reinterpret_cast<const ull *>(bsize), reinterpret_cast<const ull *>(bstart), wl, h0, h1);
    return hipGetLastError();
}

hipError_t launch_recv_classify(const uint64_t *pos, int P, uint64_t *bsize, uint64_t *bstart,
                                const WorkLists &wl, uint64_t *scratch, hipStream_t s) {
    const hipError_t e = launch_recv_bounds(pos, P, bsize, bstart, scratch, s);
    if (e != hipSuccess) return e;
    return launch_classify_range(bsize, bstart, wl, 0, kBuckets16, s);
}

hipError_t launch_gather_sort(const void *recv, bool packed16, const uint64_t *pos,
                              const uint64_t *roff, int P, const uint64_t *bstart,
                              const uint64_t *list, uint32_t nlist, int cls, bool atomic_rank,
                              uint32_t *out, hipStream_t s, const uint32_t *ndev,
                              uint32_t first) {
    using ull = unsigned long long;
    if (nlist == 0) return hipSuccess;
    if (cls < 1 || cls > kLocalClasses || P < 1 || P > 64) return hipErrorInvalidValue;
    auto *ps = reinterpret_cast<const ull *>(pos);
    auto *ro = reinterpret_cast<const ull *>(roff);
    auto *bs = reinterpret_cast<const ull *>(bstart);
    auto *l = reinterpret_cast<const ull *>(list);
    auto *r32 = reinterpret_cast<const int32_t *>(recv);
    auto *r16 = reinterpret_cast<const uint16_t *>(recv);
#define GSORT_K11G(B, I, AT)                                                                   \
    do {                                                                                       \
        if (packed16) launch_k(k_gather_sort<B, I, AT, uint16_t>, nlist, B, 0, s, r16, ps, ro, P, bs, l, out, ndev, first); \
        else launch_k(k_gather_sort<B, I, AT, int32_t>, nlist, B, 0, s, r32, ps, ro, P, bs, l, out, ndev, first);          \
    } while (0)
    switch (cls) {
        case 1: if (atomic_rank) GSORT_K11G(256, 18, true); else GSORT_K11G(256, 18, false); break;
        case 2: if (atomic_rank) GSORT_K11G(kC2Block, kC2Items, true); else GSORT_K11G(kC2Block, kC2Items, false); break;
        case 3:  // packed buckets: the two-to-a-register body (three workgroups per CU)
            if (packed16) {
                if (atomic_rank) launch_k(k_gather_sort16<kC3Block, kC3Items, true>, nlist, kC3Block, 0, s, r16, ps, ro, P, l, out, ndev, first);
                else launch_k(k_gather_sort16<kC3Block, kC3Items, false>, nlist, kC3Block, 0, s, r16, ps, ro, P, l, out, ndev, first);
            } else if (atomic_rank) GSORT_K11G(kC3Block, kC3Items, true); else GSORT_K11G(kC3Block, kC3Items, false);
            break;
        default: if (atomic_rank) GSORT_K11G(1024, 32, true); else GSORT_K11G(1024, 32, false); break;
    }
#undef GSORT_K11G
    return hipGetLastError();
}

hipError_t launch_gather_copy(const void *recv, bool packed16, const uint64_t *pos,
                              const uint64_t *roff, int P, const uint64_t *bstart, uint64_t n_out,
                              uint32_t *out, hipStream_t s, uint64_t min_len, bool as_int32) {
    using ull = unsigned long long;
    if (n_out == 0) return hipSuccess;
    auto *ps = reinterpret_cast<const ull *>(pos);
    auto *ro = reinterpret_cast<const ull *>(roff);
    auto *bs = reinterpret_cast<const ull *>(bstart);
    const unsigned grid = (unsigned)((n_out + 65535) / 65536);
    if (packed16)
        launch_k(k_gather_copy<uint16_t>, grid, 256, 0, s, reinterpret_cast<const uint16_t *>(recv), ps, ro,
                                                 P, bs, out, (ull)n_out, (ull)min_len,
                                                 as_int32 ? kFlip : 0u);
    else
        launch_k(k_gather_copy<int32_t>, grid, 256, 0, s, reinterpret_cast<const int32_t *>(recv), ps, ro,
                                                 P, bs, out, (ull)n_out, (ull)min_len,
                                                 as_int32 ? kFlip : 0u);
    return hipGetLastError();
}

hipError_t launch_hist_expand(const void *recv, bool packed16, const uint64_t *pos,
                              const uint64_t *roff, int P, const uint64_t *bstart,
                              const uint64_t *list, uint32_t nlist, uint32_t *out,
                              hipStream_t s) {
    using ull = unsigned long long;
    if (nlist == 0) return hipSuccess;
    if (P < 1 || P > 64) return hipErrorInvalidValue;
    auto *ps = reinterpret_cast<const ull *>(pos);
    auto *ro = reinterpret_cast<const ull *>(roff);
    auto *bs = reinterpret_cast<const ull *>(bstart);
    auto *l = reinterpret_cast<const ull *>(list);
    if (packed16)
        launch_k(k_hist_expand<uint16_t>, nlist, 1024, 0, s, reinterpret_cast<const uint16_t *>(recv), ps, ro, P,
                                             bs, l, out);
    else
        launch_k(k_hist_expand<int32_t>, nlist, 1024, 0, s, reinterpret_cast<const int32_t *>(recv), ps, ro, P,
                                             bs, l, out);
    return hipGetLastError();
}

hipError_t launch_count_expand_lists(const void *recv, bool packed16, const uint64_t *pos,
                                     const uint64_t *roff, int P, const uint64_t *bstart,
                                     const CxLists &cl, int ncu, uint32_t *out, hipStream_t s,
                                     uint64_t *fb_list, uint32_t *fb_ctr) {
    using ull = unsigned long long;
    const uint32_t nb = cl.bound();
    if (nb == 0) return hipSuccess;
    if (P < 1 || P > 64 || ncu < 1 || cl.nl < 1 || cl.nl > kCxLists ||
        (cl.skip >= 0 && (cl.skip >= cl.nl || !cl.skip_max)))
        return hipErrorInvalidValue;
    auto *ps = reinterpret_cast<const ull *>(pos);
    auto *ro = reinterpret_cast<const ull *>(roff);
    auto *bs = reinterpret_cast<const ull *>(bstart);
    ull *fl = reinterpret_cast<ull *>(fb_list);
    if (fb_list) {  // u8 bins, two workgroups per CU; wrapped buckets appended to fb_list
        const uint32_t grid = std::min<uint32_t>(nb, 2u * (uint32_t)ncu);
        if (packed16)
            launch_k(k_count_expand<uint16_t, false, 8>, grid, 512, 0, s,
                     reinterpret_cast<const uint16_t *>(recv), ps, ro, P, bs, cl, out, 0u, fl, fb_ctr);
        else
            launch_k(k_count_expand<int32_t, false, 8>, grid, 512, 0, s,
                     reinterpret_cast<const int32_t *>(recv), ps, ro, P, bs, cl, out, 0u, fl, fb_ctr);
        return hipGetLastError();
    }
    // u16 bins, one workgroup per CU
    const uint32_t grid = std::min<uint32_t>(nb, (uint32_t)ncu);
    if (packed16)
        launch_k(k_count_expand<uint16_t>, grid, 1024, 0, s, reinterpret_cast<const uint16_t *>(recv), ps, ro, P,
                 bs, cl, out, 0u, (ull *)nullptr, (uint32_t *)nullptr);
    else
        launch_k(k_count_expand<int32_t>, grid, 1024, 0, s, reinterpret_cast<const int32_t *>(recv), ps, ro, P,
                 bs, cl, out, 0u, (ull *)nullptr, (uint32_t *)nullptr);
    return hipGetLastError();
}

hipError_t launch_count_expand(const void *recv, bool packed16, const uint64_t *pos,
                               const uint64_t *roff, int P, const uint64_t *bstart,
                               const uint64_t *list, uint32_t nlist, int ncu, uint32_t *out,
                               hipStream_t s, uint64_t *fb_list, uint32_t *fb_ctr,
                               const uint32_t *nlist_dev) {
    CxLists cl;
    cl.add(list, nlist, nlist_dev);
    return launch_count_expand_lists(recv, packed16, pos, roff, P, bstart, cl, ncu, out, s,
                                     fb_list, fb_ctr);
}

hipError_t launch_list_to_segments(uint64_t *list, uint32_t n, const uint64_t *bstart,
                                   hipStream_t s) {
    if (n == 0) return hipSuccess;
    launch_k(k_list_to_segments, (n + 255) / 256, 256, 0, s,
        reinterpret_cast<unsigned long long *>(list), n,
        reinterpret_cast<const unsigned long long *>(bstart));
    return hipGetLastError();
}

hipError_t launch_pack16(const int32_t *a, uint64_t n, uint16_t *out, hipStream_t s) {
    if (n == 0) return hipSuccess;
    launch_k(k_pack16, grid_for(n, 256, 8192), 256, 0, s, a, n, out);
    return hipGetLastError();
}

hipError_t launch_meta_counts(const uint64_t *gb, const uint64_t *rng, int nrng, uint32_t *meta,
                              hipStream_t s) {
    if (nrng <= 0) return hipSuccess;
    launch_k(k_meta_counts, dim3(kBuckets16 / 256, nrng), 256, 0, s,
        reinterpret_cast<const unsigned long long *>(gb),
        reinterpret_cast<const unsigned long long *>(rng), meta);
    return hipGetLastError();
}

hipError_t launch_lds_order_check(const uint32_t *digits, uint32_t nblocks, uint32_t nbins,
                                  uint64_t *bad, hipStream_t s) {
    launch_k(k_lds_order_check, nblocks, 512, 0, s, digits, nbins,
                                              reinterpret_cast<unsigned long long *>(bad));
    return hipGetLastError();
}

hipError_t launch_stream_copy(const void *in, void *out, uint64_t bytes, hipStream_t s) {
    if (bytes == 0) return hipSuccess;
    if (bytes % 16 || (reinterpret_cast<uintptr_t>(in) | reinterpret_cast<uintptr_t>(out)) % 16)
        return hipErrorInvalidValue;
    const uint64_t n16 = bytes / 16, grid = (n16 + 1023) / 1024;
    if (grid > 0x7fffffffull) return hipErrorInvalidValue;
    launch_k(k_stream_copy, (unsigned)grid, 256, 0, s, static_cast<const u32x4 *>(in),
                                                 static_cast<u32x4 *>(out), n16);
    return hipGetLastError();
}

hipError_t launch_minmax(const int32_t *a, uint64_t n, int *mm, hipStream_t s) {
    if (n == 0) return hipSuccess;
    launch_k(k_minmax, grid_for(n, 256, 2048), 256, 0, s, a, n, mm);
    return hipGetLastError();
}

hipError_t launch_compat_keys(const int32_t *a, uint64_t n, int P, int loop, const int *mod,
                              const double *scale, uint32_t *key, uint64_t *bad, hipStream_t s) {
    if (n == 0) return hipSuccess;
    if (P < 2 || loop < 1 || loop > kCompatMaxDigits) return hipErrorInvalidValue;
    CompatDigits cd{};
    cd.P = P;
    cd.loop = loop;
    unsigned long long w = 1;
    for (int d = 0; d < loop; ++d) {
        cd.mod[d] = mod[d];
        cd.scale[d] = scale[d];
        cd.weight[d] = w;
        w = w > (1ull << 40) ? (1ull << 40) : w * (unsigned long long)P;  // digits there are 0
    }
    launch_k(k_compat_keys, grid_for(n, 256, 2048), 256, 0, s,
        a, n, cd, key, reinterpret_cast<unsigned long long *>(bad));
    return hipGetLastError();
}

hipError_t launch_publish(const uint64_t *src, uint32_t n, uint64_t *dst, uint64_t *flag,
                          uint64_t seq, hipStream_t s) {
    using ull = unsigned long long;
    launch_k(k_publish, 1, 64, 0, s, reinterpret_cast<const ull *>(src), n,
             reinterpret_cast<ull *>(dst), reinterpret_cast<ull *>(flag), (ull)seq);
    return hipGetLastError();
}

// ---- sampled plan (K1e, K12e, K3r/K3a EST, K12f, K12g, K11e) ----------------------------
hipError_t launch_est_front(const EstPlan &p, hipStream_t s) {
    using ull = unsigned long long;
    if (p.n == 0 || p.n > kEstMaxKeys) return hipErrorInvalidValue;
    if (p.sb < 0 || p.sb > 16) return hipErrorInvalidValue;
    if (p.flip_in) launch_k(k_est_sample<true>, kEstWG, 1024, 0, s, p.in, p.n, p.part8, p.part3, p.msamp, p.eflag, p.sb, p.koff);
    else launch_k(k_est_sample<false>, kEstWG, 1024, 0, s, p.in, p.n, p.part8, p.part3, p.msamp, p.eflag, p.sb, p.koff);
    launch_k(k_est_plan, kRadix, kRadix, 0, s, p.part8, p.part3, p.msamp, kEstWG, p.n, p.slack,
             p.capx, p.capy, p.capc, p.cap3, reinterpret_cast<ull *>(p.r2),
             reinterpret_cast<ull *>(p.r3), reinterpret_cast<ull *>(p.bases3),
             reinterpret_cast<ull *>(p.bases2), p.cur2, p.lim2, p.init2, p.cur3, p.lim3, p.init3,
             reinterpret_cast<ull *>(p.wl.ctr), (uint32_t)(3 * (kLocalClasses + 1)), p.eflag);
    return hipGetLastError();
}

// the sampled plan's K3r / K3a: a tile pair per 1024-thread workgroup (one tile per 512-thread
// workgroup measured slower overall: profiles/r04_ab_k3_pipe_and_tiles.txt)
constexpr int kEstTiles = 2;
constexpr int kEstPartBlock = kPartBlock;
constexpr int kEstTilesL2 = 2;  // K3a: a pair per 1024 threads (one tile per 512: r04_ab_k3a_one_tile_rejected)

hipError_t launch_est_level3(const EstPlan &p, hipStream_t s) {
    using ull = unsigned long long;
    constexpr int B = kEstPartBlock, I = kSweepTile / B;
    const uint64_t pairs = (sweep_tiles(p.n) + kEstTiles - 1) / kEstTiles;
    if (!p.flip_in) return hipErrorInvalidValue;  // K3r loads the int32 input
    launch_k(k_partition_res<B, I, true, true, uint32_t, true, kEstTiles>, (unsigned)pairs, B, 0, s,
             p.in, p.x, p.n, (const uint32_t *)nullptr, (const TileDesc *)nullptr,
             reinterpret_cast<const ull *>(p.bases3), p.cur3, (const uint32_t *)p.eflag,
             (const uint32_t *)nullptr, (const uint32_t *)p.lim3, p.eflag + 1, p.dump,
             (const TileDesc *)nullptr, reinterpret_cast<ull *>(p.mail), (ull)p.seq_elig, p.sb,
             p.koff);
    return hipGetLastError();
}

hipError_t launch_est_level2(const EstPlan &p, hipStream_t s) {
    using ull = unsigned long long;
    constexpr int T2 = kEstTilesL2, B = kPartBlock * T2 / 2, I = kSweepTile / B;
    const uint32_t max_tiles = (uint32_t)est_max_tiles(p.n);
    TileDesc *desc = static_cast<TileDesc *>(p.tdesc);
    TileDesc *pieces = desc + max_tiles;
    launch_k(k_est_tiles, (max_tiles + 255) / 256, 256, 0, s, (const uint32_t *)p.cur3,
             (const uint32_t *)p.init3, (const uint32_t *)p.lim3,
             reinterpret_cast<const ull *>(p.bases3), max_tiles, (const uint32_t *)p.eflag, p.tp,
             desc, pieces);
    launch_k(k_partition_res<B, I, false, false, uint16_t, true, T2>,
             (max_tiles + T2 - 1) / T2, B, 0, s,
             (const uint32_t *)p.x, p.y, p.n, (const uint32_t *)p.tp, (const TileDesc *)desc,
             reinterpret_cast<const ull *>(p.bases2), p.cur2, (const uint32_t *)p.eflag,
             (const uint32_t *)nullptr, (const uint32_t *)p.lim2, p.eflag + 1,
             reinterpret_cast<uint16_t *>(p.dump),
             (const TileDesc *)pieces, (ull *)nullptr, (ull)0, p.sb, 0u);
    return hipGetLastError();
}

hipError_t launch_est_classify(const EstPlan &p, hipStream_t s) {
    using ull = unsigned long long;
    launch_k(k_est_classify, kRadix, kRadix, 0, s, (const uint32_t *)p.cur2,
             (const uint32_t *)p.init2, (const uint32_t *)p.lim2, (const uint32_t *)p.cur3,
             (const uint32_t *)p.init3, reinterpret_cast<const ull *>(p.bases2), p.wl, p.eflag,
             p.in, p.sb, p.koff);
    return hipGetLastError();
}

hipError_t launch_est_oversized(const EstPlan &p, uint32_t nlist, int ncu, hipStream_t s) {
    using ull = unsigned long long;
    if (nlist == 0) return hipSuccess;
    const unsigned grid = (unsigned)std::min<uint32_t>(nlist, (uint32_t)std::max(ncu, 1));
    CxLists cl;
    cl.add(p.wl.list[0], nlist);
    launch_k(k_count_expand<uint16_t, true>, grid, 1024, 0, s, (const uint16_t *)p.y,
             (const ull *)nullptr, (const ull *)nullptr, 1, (const ull *)nullptr, cl, p.out,
             p.koff, (ull *)nullptr, (uint32_t *)nullptr);
    return hipGetLastError();
}

hipError_t launch_est_publish(const EstPlan &p, hipStream_t s) {
    using ull = unsigned long long;
    launch_k(k_publish_lists, 1, 64, 0, s, reinterpret_cast<ull *>(p.mail),
             reinterpret_cast<const ull *>(p.wl.ctr), (const uint32_t *)p.eflag, (ull)p.seq_done);
    return hipGetLastError();
}

hipError_t launch_local_sort_e(const EstPlan &p, int cls, uint32_t first, uint32_t nlist,
                               bool publish, hipStream_t s) {
    using ull = unsigned long long;
    if (nlist == 0) return hipSuccess;
    if (cls < 1 || cls > kLocalClasses) return hipErrorInvalidValue;
    const ull *l = reinterpret_cast<const ull *>(p.wl.list[cls]);
    const ull *call = reinterpret_cast<const ull *>(p.wl.ctr), *ctr = call + 3 * cls;
    const uint16_t *y = p.y;
    const uint32_t *ef = p.eflag;
    const uint32_t ko = p.koff;
    const int nd = (16 - p.sb + 7) / 8;  // digits for the bits below the plan's two levels
                                         // (sb = 16: a child is one value, K11e copies it)
    ull *mail = publish ? reinterpret_cast<ull *>(p.mail) : nullptr;
    const ull seq = (ull)p.seq_done;
#define GSORT_K11E(B, I)                                                                       \
    do {                                                                                       \
        if (nd == 0)                                                                           \
            launch_k(k_local_sort_e<B, I, true, true>, nlist, B, 0, s, y, p.out, l, ctr, first, \
                     nd, mail, call, ef, seq, ko);                                             \
        else if (p.atomic_rank && nd == 2)                                                     \
            launch_k(k_local_sort_e<B, I, true, false, 2>, nlist, B, 0, s, y, p.out, l, ctr,   \
                     first, nd, mail, call, ef, seq, ko);                                      \
        else if (p.atomic_rank)                                                                \
            launch_k(k_local_sort_e<B, I, true>, nlist, B, 0, s, y, p.out, l, ctr, first, nd,  \
                     mail, call, ef, seq, ko);                                                 \
        else                                                                                   \
            launch_k(k_local_sort_e<B, I, false>, nlist, B, 0, s, y, p.out, l, ctr, first, nd, \
                     mail, call, ef, seq, ko);                                                 \
    } while (0)
    switch (cls) {
        case 1: GSORT_K11E(256, 18); break;
        case 2: GSORT_K11E(kC2Block, kC2Items); break;
        case 3:  // the packed body (a one-value child: the copy kernel)
            if (nd == 0) GSORT_K11E(kC3Block, kC3Items);
            else if (nd == 1)
                launch_k(k_local_sort_e16<kC3Block, kC3Items, true, 1>, nlist, kC3Block, 0, s, y,
                         p.out, l, ctr, first, nd, mail, call, ef, seq, ko);
            else if (p.atomic_rank)
                launch_k(k_local_sort_e16<kC3Block, kC3Items, true, 2>, nlist, kC3Block, 0, s, y,
                         p.out, l, ctr, first, nd, mail, call, ef, seq, ko);
            else
                launch_k(k_local_sort_e16<kC3Block, kC3Items, false, 2>, nlist, kC3Block, 0, s, y,
                         p.out, l, ctr, first, nd, mail, call, ef, seq, ko);
            break;
        default: GSORT_K11E(1024, 32); break;  // (shifted plans only: kEstCx)
    }
#undef GSORT_K11E
    return hipGetLastError();
}

// ---------------------------------------------------------------------------------------
// One dominant 16-bit child ("giant child").  When at least half of a block's
// keys share their top 16 bits c (Zipf keys: ~99.6 % are below 2^16; 8- or 16-bit keys; one
// frequent value), every MSD level moves nearly every key again (the exact plan walks all four
// levels with buckets of up to the whole block; the sampled plan's children outgrow K11).  Keys
// carry no payload, so child c is sorted by COUNTING its low 16 bits: K1g reads the block once
// -- child c's keys into a 65536-bin histogram per workgroup (K1h's packed u16 pairs and wrap
// repair), every other ("cold") key compacted into its XCD shard's region of a scratch buffer
// -- K12m sums the partials, K12s scans them into output starts (after the cold keys below c),
// K12w maps every 8192-key output chunk to its first bin, and K18g writes child c's keys
// straight from the counts.  The cold keys are sorted by the regular local sort.  4 B/key read
// + 4 B/key write for the child, instead of 8 B/key per MSD level.
// ---------------------------------------------------------------------------------------
namespace {

// Workgroup barrier that waits only for this wave's LDS operations: a __syncthreads() also
// drains the global loads in flight (s_waitcnt vmcnt(0)), which would cost K1g its prefetch of
// the next tile at every per-tile reservation.
__device__ __forceinline__ void lds_barrier() {
    __asm__ volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
}

// K1m: does one top-16-bit child hold at least half of min(n, 16384) sampled keys (1024 evenly
// spaced groups of 16 consecutive keys)?  A
// Boyer-Moore majority vote finds the only child that can (per thread over its 16 samples, then
// pairwise across lanes, waves: a majority survives any pairing), and one counting pass checks
// it: res[0] = the candidate (ordered u32 >> 16), res[1] = its samples, res[2] = the samples.
// (Round 4: the 65 536-bin LDS histogram it replaces serialized its adds on skewed samples and
// read its bins with 32-way bank conflicts -- 49 us, now a few.)
constexpr uint32_t kModeSamples = 16384;
__device__ __forceinline__ void bm_merge(uint32_t &c, uint32_t &k, uint32_t c2, uint32_t k2) {
    if (c == c2) { k += k2; }
    else if (k >= k2) { k -= k2; }
    else { c = c2; k = k2 - k; }
}
__global__ __launch_bounds__(1024) void k_est_mode(const uint32_t *__restrict__ in, uint64_t n,
                                                   uint64_t stride,
                                                   unsigned long long *__restrict__ res) {
    constexpr uint32_t PER = kModeSamples / 1024;
    __shared__ uint32_t s_c[16], s_k[16];
    __shared__ uint32_t s_cand;
    __shared__ unsigned long long s_cnt[16];
    const uint32_t tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const uint32_t S = n < kModeSamples ? (uint32_t)n : kModeSamples;
    uint32_t d[PER];
#pragma unroll
    for (uint32_t j = 0; j < PER; ++j) {
        const uint32_t i = j * 1024 + tid;
        // groups of 16 consecutive keys, group g at g * stride (16 strided single keys per
        // thread missed the TLB on every load: 35 us for 16 384 keys over 1 GiB)
        const uint64_t at = (uint64_t)(i >> 4) * stride + (i & 15u);
        d[j] = i < S ? (in[at] ^ kFlip) >> 16 : 0x10000u;
    }
    uint32_t c = 0x10000u, k = 0;  // candidate (0x10000: none), its surplus
#pragma unroll
    for (uint32_t j = 0; j < PER; ++j)
        if (d[j] != 0x10000u) bm_merge(c, k, d[j], 1u);
#pragma unroll
    for (int o = 32; o; o >>= 1) {
        const uint32_t c2 = (uint32_t)__shfl_xor((int)c, o), k2 = (uint32_t)__shfl_xor((int)k, o);
        bm_merge(c, k, c2, k2);
    }
    if (lane == 0) { s_c[w] = c; s_k[w] = k; }
    __syncthreads();
    if (tid == 0) {
        uint32_t cc = s_c[0], kk = s_k[0];
        for (int i = 1; i < 16; ++i) bm_merge(cc, kk, s_c[i], s_k[i]);
        s_cand = cc;
    }
    __syncthreads();
    const uint32_t cand = s_cand;
    uint32_t m = 0;
#pragma unroll
    for (uint32_t j = 0; j < PER; ++j) m += d[j] == cand ? 1u : 0u;
    unsigned long long mm = m;
#pragma unroll
    for (int o = 32; o; o >>= 1) mm += (unsigned long long)__shfl_xor(mm, o);
    if (lane == 0) s_cnt[w] = mm;
    __syncthreads();
    if (tid == 0) {
        unsigned long long t = 0;
        for (int i = 0; i < 16; ++i) t += s_cnt[i];
        res[0] = cand & 0xffffu;
        res[1] = cand == 0x10000u ? 0ull : t;
        res[2] = S;
    }
}

// K1g: K1h's loop (tile pairs b, b + G, .. with the next tile prefetched) over the block; keys of
// child c go into the workgroup's packed histogram of their LOW 16 bits (part, fix as K1h);
// every other key is written (as the input int32) into the workgroup's own segment
// cold + b * wg_cap, each wave reserving its run there with one LDS atomic -- no barrier and no
// device atomic per tile (round 4: the per-tile shard reservation behind two workgroup
// barriers made K1g ~2x K1h's time); ctr[1 + b] = the segment's cold keys, ctr[0] += the cold
// keys below child c (ctr zeroed by the caller).
template <int BLOCK, bool FIN>
__global__ __launch_bounds__(BLOCK) void k_giant_hist(const uint32_t *__restrict__ in, uint64_t n,
                                                      uint32_t child, uint32_t *__restrict__ part,
                                                      unsigned long long *__restrict__ fix,
                                                      uint32_t *__restrict__ cold,
                                                      unsigned long long wg_cap,
                                                      unsigned long long *__restrict__ ctr) {
    constexpr int ITEMS = kSweepTile / BLOCK;
    constexpr uint32_t kWords = kBuckets16 / 2;
    __shared__ uint32_t s_h[kWords + kAggSpare];
    __shared__ uint32_t s_cnt[2];
    uint32_t *spare = s_h + kWords;
    const uint32_t tid = threadIdx.x, lane = tid & 63;
    for (uint32_t i = tid; i < kWords; i += BLOCK) s_h[i] = 0;
    if (tid < 2) s_cnt[tid] = 0;
    const uint32_t ntiles = (uint32_t)((n + kSweepTile - 1) / kSweepTile);
    const uint32_t last_len = (uint32_t)(n - (uint64_t)(ntiles - 1) * kSweepTile);
    auto tile_len = [&](uint32_t t) -> uint32_t {
        return t == ntiles - 1 ? last_len : (uint32_t)kSweepTile;
    };
    auto tile_of = [&](uint32_t i) -> uint32_t {
        return 2 * (blockIdx.x + (i >> 1) * gridDim.x) + (i & 1);
    };
    const uint32_t shard = blockIdx.x % kShards;
    unsigned long long *fx = fix + (uint64_t)shard * kBuckets16;
    uint32_t *cs = cold + (uint64_t)blockIdx.x * wg_cap;
    uint32_t below = 0;  // lane 0: the wave's cold keys below child c
    uint32_t t = tile_of(0);
    uint32_t k[ITEMS];
    if (t < ntiles) {
        const uint32_t len = tile_len(t);
        load_tile<BLOCK, ITEMS, FIN>(in + (uint64_t)t * kSweepTile + tid,
                                     len == (uint32_t)kSweepTile, len, k);
    }
    __syncthreads();  // zeroing done
    for (uint32_t i = 1; t < ntiles; ++i) {
        const uint32_t len = tile_len(t);
        const uint32_t tn = tile_of(i);
        uint32_t kn[ITEMS];
        if (tn < ntiles) {
            const uint32_t lenn = tile_len(tn);
            load_tile<BLOCK, ITEMS, FIN>(in + (uint64_t)tn * kSweepTile + tid,
                                         lenn == (uint32_t)kSweepTile, lenn, kn);
        }
        bool g[ITEMS];
        uint32_t old[ITEMS];
#pragma unroll
        for (int j = 0; j < ITEMS; ++j)
            g[j] = (uint32_t)(j * BLOCK) + tid < len && (k[j] >> 16) == child;
        // a skewed wave (a frequent low half: Zipf keys put ~38 % of the child on one value, whose
        // plain LDS adds serialize ~24-way): of the words of the first two distinct child keys of
        // item 0, the one more lanes share is aggregated in every item when at least 8 share it
        // (~1 % of the keys on one value in uniform children: plain adds)
        const uint32_t wd = (k[0] & 0xffffu) >> 1;
        const uint64_t gm = __ballot(g[0]);
        uint32_t w0 = ~0u, best = 0;
        if (gm) {
            const uint32_t wa = (uint32_t)__builtin_amdgcn_readlane((int)wd, (int)__builtin_ctzll(gm));
            const uint64_t ma = __ballot(g[0] && wd == wa), rest = gm & ~ma;
            w0 = wa;
            best = (uint32_t)__popcll(ma);
            if (rest) {
                const uint32_t wb = (uint32_t)__builtin_amdgcn_readlane((int)wd, (int)__builtin_ctzll(rest));
                const uint32_t nb = (uint32_t)__popcll(__ballot(g[0] && wd == wb));
                if (nb > best) { w0 = wb; best = nb; }
            }
        }
        const bool skew = best >= 8;
        bool wrap = false;
#pragma unroll
        for (int j = 0; j < ITEMS; ++j) {  // (all lanes issue: a key off the child adds 0 --
            // an `if` per item left the compiler waiting on each atomic in turn)
            const uint32_t b = k[j] & 0xffffu;
            old[j] = skew ? agg_add_pair_at(s_h, b, w0, spare, g[j])
                          : atomicAdd(&s_h[b >> 1], g[j] ? 1u << ((b & 1u) << 4) : 0u);
        }
#pragma unroll
        for (int j = 0; j < ITEMS; ++j)
            wrap |= g[j] && ((old[j] >> ((k[j] & 1u) << 4)) & 0xffffu) == 0xffffu;
        if (__builtin_expect(wrap, 0)) {
#pragma unroll
            for (int j = 0; j < ITEMS; ++j)
                if (g[j] && ((old[j] >> ((k[j] & 1u) << 4)) & 0xffffu) == 0xffffu)
                    h16_wrap(fx, k[j] & 0xffffu, old[j]);
        }
        // cold keys: per-wave counts, the wave's run reserved in the workgroup's segment
        uint64_t m[ITEMS];
        uint32_t wc = 0, wl = 0;
#pragma unroll
        for (int j = 0; j < ITEMS; ++j) {
            const bool cj = (uint32_t)(j * BLOCK) + tid < len && !g[j];
            m[j] = __ballot(cj);
            wc += (uint32_t)__popcll(m[j]);
            wl += (uint32_t)__popcll(__ballot(cj && (k[j] >> 16) < child));
        }
        below += wl;
        if (wc) {  // (wave-uniform)
            uint32_t woff = 0;
            if (lane == 0) woff = atomicAdd(&s_cnt[0], wc);
            const unsigned long long base = (uint32_t)__shfl((int)woff, 0);
            uint32_t run = 0;
#pragma unroll
            for (int j = 0; j < ITEMS; ++j) {
                if ((m[j] >> lane) & 1ull) cs[base + run + lane_rank(m[j])] = k[j] ^ (FIN ? kFlip : 0u);
                run += (uint32_t)__popcll(m[j]);
            }
        }
#pragma unroll
        for (int j = 0; j < ITEMS; ++j) k[j] = kn[j];
        t = tn;
    }
    if (lane == 0 && below) atomicAdd(&s_cnt[1], below);
    __syncthreads();
    uint32_t *dst = part + (uint64_t)blockIdx.x * kWords;
    for (uint32_t i = tid; i < kWords; i += BLOCK) dst[i] = s_h[i];
    if (tid == 0) {
        ctr[1 + blockIdx.x] = s_cnt[0];
        if (s_cnt[1]) atomicAdd(&ctr[0], (unsigned long long)s_cnt[1]);
    }
}

// K1g's cold segments gathered: segment b (ctr[1 + b] keys at cold + b * wg_cap) to
// out[sum of ctr[1 .. b]), one workgroup per segment.
__global__ __launch_bounds__(1024) void k_giant_gather(const uint32_t *__restrict__ cold,
                                                       unsigned long long wg_cap,
                                                       const unsigned long long *__restrict__ ctr,
                                                       uint32_t *__restrict__ out) {
    __shared__ unsigned long long s_off;
    const uint32_t b = blockIdx.x, tid = threadIdx.x;
    if (tid < 64) {
        unsigned long long x = 0;
        for (uint32_t q = tid; q < b; q += 64) x += ctr[1 + q];
#pragma unroll
        for (int o = 32; o; o >>= 1) x += (unsigned long long)__shfl_xor(x, o);
        if (tid == 0) s_off = x;
    }
    __syncthreads();
    const unsigned long long cnt = ctr[1 + b];
    const uint32_t *src = cold + (uint64_t)b * wg_cap;
    uint32_t *dst = out + s_off;
    for (unsigned long long i = tid; i < cnt; i += 1024) dst[i] = src[i];
}

// K12m: counts[b] = child c's keys with low 16 bits b: the b-half of word b/2 over the nblk
// partials + the wrap repairs of all shards (which it zeroes for the next K1h / K1g).  One thread
// per packed word.
__global__ __launch_bounds__(256) void k_giant_count(const uint32_t *__restrict__ part,
                                                     uint32_t nblk,
                                                     unsigned long long *__restrict__ fix,
                                                     unsigned long long *__restrict__ counts) {
    constexpr uint32_t kWords = kBuckets16 / 2;
    const uint32_t w = blockIdx.x * 256 + threadIdx.x;
    unsigned long long lo = 0, hi = 0;
#pragma unroll 8
    for (uint32_t b = 0; b < nblk; ++b) {
        const uint32_t v = part[(uint64_t)b * kWords + w];
        lo += v & 0xffffu;
        hi += v >> 16;
    }
#pragma unroll
    for (uint32_t x = 0; x < kShards; ++x) {
        unsigned long long *f = fix + (uint64_t)x * kBuckets16 + 2 * w;
        lo += f[0];
        hi += f[1];
        f[0] = 0;
        f[1] = 0;
    }
    counts[2 * w] = lo;
    counts[2 * w + 1] = hi;
}

// K12s: starts[b] = ctr[0] (the cold keys below the child) + the exclusive scan of counts,
// starts[65536] = the end; two passes of 64 workgroups over coalesced 1024-bin blocks (one
// 1024-thread workgroup walking 64 bins per thread took 49 us): K12s-a sums each block into
// part[64], K12s-b offsets its block by the sums before it.
__global__ __launch_bounds__(1024) void k_giant_scan_a(const unsigned long long *__restrict__ counts,
                                                       unsigned long long *__restrict__ part) {
    __shared__ unsigned long long s_w[16];
    const uint32_t tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    unsigned long long x = counts[blockIdx.x * 1024 + tid];
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) x += (unsigned long long)__shfl_xor(x, o);
    if (lane == 0) s_w[w] = x;
    __syncthreads();
    if (tid == 0) {
        unsigned long long t = 0;
        for (int i = 0; i < 16; ++i) t += s_w[i];
        part[blockIdx.x] = t;
    }
}
__global__ __launch_bounds__(1024) void k_giant_scan_b(const unsigned long long *__restrict__ counts,
                                                       const unsigned long long *__restrict__ part,
                                                       const unsigned long long *__restrict__ ctr,
                                                       unsigned long long *__restrict__ starts) {
    __shared__ unsigned long long s_w[16];
    __shared__ unsigned long long s_pre;
    const uint32_t b = blockIdx.x, tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    if (tid < 64) {
        unsigned long long v = tid < b ? part[tid] : 0ull;
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) v += (unsigned long long)__shfl_xor(v, o);
        if (tid == 0) s_pre = v + ctr[0];
    }
    const unsigned long long c = counts[b * 1024 + tid];
    unsigned long long x = c;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const unsigned long long t = __shfl_up(x, o);
        if ((int)lane >= o) x += t;
    }
    if (lane == 63) s_w[w] = x;
    __syncthreads();
    unsigned long long run = s_pre + x - c;
    for (uint32_t ww = 0; ww < w; ++ww) run += s_w[ww];
    starts[b * 1024 + tid] = run;
    if (b == gridDim.x - 1 && tid == 1023) starts[kBuckets16] = run + c;
}

// K12w: chunk_bin[w] = the bin holding output position starts[0] + w * kExpandChunk (the last
// bin b with starts[b] <= that position), one thread per chunk.
// K18g geometry (round 4, profiles/r04_ab_k18g_geometry.txt): 4096-key chunks per 512-thread
// workgroup (four in flight per CU instead of two 8192 x 1024: each chunk is a chain of
// dependent loads -- starts, chunk_bin, the bins -- before its stores); the stores of chunks
// spanning several bins nontemporal (16-bit keys K18g 0.294 -> 0.21 ms), a chunk inside one bin
// (a frequent value: 8-bit keys, Zipf) stored plainly (nontemporal there measured slower)
constexpr uint32_t kExpandChunk = 4096, kExpandThreads = 512;
__global__ __launch_bounds__(256) void k_giant_chunks(const unsigned long long *__restrict__ starts,
                                                      uint32_t nchunks, uint32_t *__restrict__ chunk_bin) {
    const uint32_t w = blockIdx.x * 256 + threadIdx.x;
    if (w >= nchunks) return;
    const unsigned long long q = starts[0] + (unsigned long long)w * kExpandChunk;
    uint32_t lo = 0, hi = kBuckets16;  // starts[lo] <= q < starts[hi]
    while (hi - lo > 1) {
        const uint32_t mid = (lo + hi) >> 1;
        if (starts[mid] <= q) lo = mid;
        else hi = mid;
    }
    chunk_bin[w] = lo;
}

// K18g: chunk w = output positions [q0, q0 + 8192) of child c: every non-empty bin b starting
// in it marks its first position with b + 1 (the chunk's first bin marks position 0), an
// inclusive max-scan gives every position its bin, and the keys (c << 16 | bin) go out as int32
// in coalesced stores.
__global__ __launch_bounds__(kExpandThreads) void k_giant_expand(const unsigned long long *__restrict__ starts,
                                                       const uint32_t *__restrict__ chunk_bin,
                                                       uint32_t nchunks, uint32_t child,
                                                       uint32_t *__restrict__ out) {
    constexpr uint32_t C = kExpandChunk, NT = kExpandThreads, PER = C / NT;
    __shared__ uint32_t s_m[C];
    __shared__ uint32_t s_w[NT / 64];
    const uint32_t tid = threadIdx.x, lane = tid & 63, w = tid >> 6, ch = blockIdx.x;
    const unsigned long long end = starts[kBuckets16];
    const unsigned long long q0 = starts[0] + (unsigned long long)ch * C;
    const uint32_t len = (uint32_t)min((unsigned long long)C, end - q0);
#pragma unroll
    for (uint32_t i = 0; i < PER; ++i) s_m[i * NT + tid] = 0;
    const uint32_t b0 = chunk_bin[ch];
    const uint32_t b1 = ch + 1 < nchunks ? chunk_bin[ch + 1] : kBuckets16 - 1;
    if (starts[b0 + 1] >= q0 + len) {  // one bin covers the chunk (a frequent value)
        const uint32_t key = ((child << 16) | b0) ^ kFlip;
        uint32_t *o = out + q0;
#pragma unroll
        for (uint32_t i = 0; i < PER; ++i)
            if (i * NT + tid < len) o[i * NT + tid] = key;
        return;
    }
    __syncthreads();
    for (uint32_t b = b0 + tid; b <= b1; b += NT) {
        const unsigned long long st = starts[b], en = starts[b + 1];
        if (en > st && (b == b0 || st < q0 + len))
            atomicMax(&s_m[st > q0 ? (uint32_t)(st - q0) : 0u], b + 1);
    }
    __syncthreads();
    uint32_t v[PER], mx = 0;
#pragma unroll
    for (uint32_t i = 0; i < PER; ++i) { v[i] = max(mx, s_m[tid * PER + i]); mx = v[i]; }
    uint32_t x = mx;  // inclusive max over the threads of the wave
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t t = __shfl_up(x, o);
        if ((int)lane >= o) x = max(x, t);
    }
    if (lane == 63) s_w[w] = x;
    uint32_t pre = __shfl_up(x, 1);
    if (lane == 0) pre = 0;
    __syncthreads();
    for (uint32_t ww = 0; ww < w; ++ww) pre = max(pre, s_w[ww]);
#pragma unroll
    for (uint32_t i = 0; i < PER; ++i) s_m[tid * PER + i] = max(v[i], pre);
    __syncthreads();
    uint32_t *o = out + q0;
#pragma unroll
    for (uint32_t i = 0; i < PER; ++i) {
        const uint32_t j = i * NT + tid;
        if (j < len) __builtin_nontemporal_store(((child << 16) | (s_m[j] - 1u)) ^ kFlip, o + j);
    }
}

}  // namespace

hipError_t launch_est_mode(const uint32_t *in, uint64_t n, uint64_t *res, hipStream_t s) {
    if (n == 0) return hipErrorInvalidValue;
    // sample i at (i / 16) * stride + i % 16: 1024 groups of 16 keys spread over the block
    const uint64_t stride = n < kModeSamples ? 16 : n / (kModeSamples / 16);
    launch_k(k_est_mode, 1, 1024, 0, s, in, n, stride, reinterpret_cast<unsigned long long *>(res));
    return hipGetLastError();
}

hipError_t launch_giant_hist(const uint32_t *in, uint64_t n, uint32_t child, uint32_t *part,
                             uint64_t *fix, uint32_t *cold, uint64_t *ctr, hipStream_t s) {
    if (n == 0) return hipErrorInvalidValue;
    uint32_t g = 0;
    const uint64_t wg_cap = giant_wg_cap(n, &g);
    using ull = unsigned long long;
    launch_k(k_giant_hist<1024, true>, g, 1024, 0, s, in, n, child, part,
             reinterpret_cast<ull *>(fix), cold, (ull)wg_cap, reinterpret_cast<ull *>(ctr));
    return hipGetLastError();
}

hipError_t launch_giant_gather(const uint32_t *cold, uint64_t n, const uint64_t *ctr,
                               uint32_t *out, hipStream_t s) {
    uint32_t g = 0;
    const uint64_t wg_cap = giant_wg_cap(n, &g);
    using ull = unsigned long long;
    launch_k(k_giant_gather, g, 1024, 0, s, cold, (ull)wg_cap, reinterpret_cast<const ull *>(ctr),
             out);
    return hipGetLastError();
}

hipError_t launch_giant_plan(const uint32_t *part, uint32_t nblk, uint64_t *fix,
                             const uint64_t *ctr, uint64_t *counts, uint64_t *starts,
                             hipStream_t s) {
    using ull = unsigned long long;
    launch_k(k_giant_count, kBuckets16 / 2 / 256, 256, 0, s, part, nblk,
             reinterpret_cast<ull *>(fix), reinterpret_cast<ull *>(counts));
    static_assert(kBuckets16 == 64 * 1024, "K12s: 64 blocks of 1024 bins");
    ull *bsum = reinterpret_cast<ull *>(starts + kBuckets16 + 1);  // 64 u64 of scratch
    launch_k(k_giant_scan_a, 64, 1024, 0, s, reinterpret_cast<const ull *>(counts), bsum);
    launch_k(k_giant_scan_b, 64, 1024, 0, s, reinterpret_cast<const ull *>(counts),
             reinterpret_cast<const ull *>(bsum), reinterpret_cast<const ull *>(ctr),
             reinterpret_cast<ull *>(starts));
    return hipGetLastError();
}

hipError_t launch_giant_expand(const uint64_t *starts, uint64_t n_child, uint32_t child,
                               uint32_t *chunk_bin, uint32_t *out, hipStream_t s) {
    if (n_child == 0) return hipSuccess;
    const uint64_t nch = (n_child + kExpandChunk - 1) / kExpandChunk;
    using ull = unsigned long long;
    launch_k(k_giant_chunks, (unsigned)((nch + 255) / 256), 256, 0, s,
             reinterpret_cast<const ull *>(starts), (uint32_t)nch, chunk_bin);
    launch_k(k_giant_expand, (unsigned)nch, kExpandThreads, 0, s, reinterpret_cast<const ull *>(starts),
             chunk_bin, (uint32_t)nch, child, out);
    return hipGetLastError();
}

hipError_t launch_copy(const uint32_t *in, uint32_t *out, uint64_t n, hipStream_t s) {
    if (n == 0) return hipSuccess;
    launch_k(k_copy, grid_for(n, 256, 8192), 256, 0, s, in, out, n);
    return hipGetLastError();
}

}  // namespace gsort
