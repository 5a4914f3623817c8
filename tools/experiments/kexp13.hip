// kexp13.hip -- what bounds K1h (k_hist16: the 16-bit histogram read pass)?  (experiment, not
// the product).  Same grid as the product (256 x 1024 threads, 128 KiB LDS histogram, tile
// pairs p = b, b + G, ..), over 2^28 uniform 31-bit keys:
//   product     k_hist16 from gsort_kernels.hip
//   LOADS 0/1   dword loads strided by the block (product) / two 16-B loads per thread
//   ATOM 0/1/2  no atomics (xor into a sink) / returning u16-pair atomics / non-returning
//   DEPTH 1/2   tiles in flight while the current one is counted
//   SYNTH       keys from a hash of the index instead of loads (atomic rate alone)
// Every atomic variant's partials are checked against the product's.
//   hipcc --offload-arch=gfx950 -O3 -I mpi-test_amd/csrc tools/experiments/kexp13.hip -o kexp13
#include <stdio.h>
#include <stdlib.h>

#include <algorithm>
#include <vector>

#include "../../mpi-test_amd/csrc/gsort_kernels.hip"

using namespace gsort;

#define CK(x)                                                                            \
    do {                                                                                 \
        hipError_t e = (x);                                                              \
        if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); exit(1); } \
    } while (0)

typedef unsigned int v4u __attribute__((ext_vector_type(4)));

namespace {
constexpr int BLOCK = 1024, ITEMS = kSweepTile / BLOCK;  // 8 keys per thread per tile

// 1 GiB copy with plain (write-back, cache-allocating) stores, as K11 stores its output
__global__ __launch_bounds__(256) void k_plain_copy(const v4u *__restrict__ in, v4u *__restrict__ out,
                                                    uint64_t n16) {
    const uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    if (i < n16) out[i] = in[i];
}

__device__ __forceinline__ uint32_t hash_key(uint32_t i) {
    uint32_t z = i * 0x9E3779B9u;
    z ^= z >> 15; z *= 0x85EBCA6Bu; z ^= z >> 13;
    return (z >> 1) ^ 0x80000000u;
}

template <int LOADS, bool SYNTH>
__device__ __forceinline__ void ld(const uint32_t *__restrict__ in, uint32_t t, uint32_t (&k)[ITEMS]) {
    const uint32_t tid = threadIdx.x;
    if (SYNTH) {
#pragma unroll
        for (int i = 0; i < ITEMS; ++i) k[i] = hash_key(t * kSweepTile + i * BLOCK + tid);
        return;
    }
    const uint32_t *src = in + (uint64_t)t * kSweepTile;
    if (LOADS == 0) {
#pragma unroll
        for (int i = 0; i < ITEMS; ++i) k[i] = src[i * BLOCK + tid] ^ kFlip;
    } else {
        const v4u *s4 = reinterpret_cast<const v4u *>(src);
#pragma unroll
        for (int h = 0; h < ITEMS / 4; ++h) {
            const v4u v = s4[h * BLOCK + tid];
            k[4 * h + 0] = v.x ^ kFlip; k[4 * h + 1] = v.y ^ kFlip;
            k[4 * h + 2] = v.z ^ kFlip; k[4 * h + 3] = v.w ^ kFlip;
        }
    }
}

template <int LOADS, int ATOM, int DEPTH, bool SYNTH>
__global__ __launch_bounds__(BLOCK) void k1h(const uint32_t *__restrict__ in, uint32_t ntiles,
                                             uint32_t *__restrict__ part, uint32_t *sink) {
    constexpr uint32_t kWords = kBuckets16 / 2;
    __shared__ uint32_t s_h[kWords];
    const uint32_t tid = threadIdx.x;
    for (uint32_t i = tid; i < kWords; i += BLOCK) s_h[i] = 0;
    auto tile_of = [&](uint32_t i) -> uint32_t { return 2 * (blockIdx.x + (i >> 1) * gridDim.x) + (i & 1); };
    uint32_t k[DEPTH][ITEMS];
#pragma unroll
    for (int d = 0; d < DEPTH; ++d) {
        const uint32_t t = tile_of(d);
        if (t < ntiles) ld<LOADS, SYNTH>(in, t, k[d]);
    }
    __syncthreads();
    uint32_t acc = 0, wrapc = 0;
    for (uint32_t i = 0; tile_of(i) < ntiles; ++i) {
        uint32_t cur[ITEMS];
#pragma unroll
        for (int j = 0; j < ITEMS; ++j) cur[j] = k[0][j];
#pragma unroll
        for (int d = 0; d + 1 < DEPTH; ++d)
#pragma unroll
            for (int j = 0; j < ITEMS; ++j) k[d][j] = k[d + 1][j];
        const uint32_t tn = tile_of(i + DEPTH);
        if (tn < ntiles) ld<LOADS, SYNTH>(in, tn, k[DEPTH - 1]);
        if (ATOM == 0) {
#pragma unroll
            for (int j = 0; j < ITEMS; ++j) acc ^= cur[j];
        } else if (ATOM == 1) {
            uint32_t old[ITEMS];
#pragma unroll
            for (int j = 0; j < ITEMS; ++j) {
                const uint32_t b = cur[j] >> 16;
                old[j] = atomicAdd(&s_h[b >> 1], 1u << ((b & 1u) << 4));
            }
#pragma unroll
            for (int j = 0; j < ITEMS; ++j)
                wrapc += ((old[j] >> (((cur[j] >> 16) & 1u) << 4)) & 0xffffu) == 0xffffu;
        } else {
#pragma unroll
            for (int j = 0; j < ITEMS; ++j) {
                const uint32_t b = cur[j] >> 16;
                __hip_atomic_fetch_add(&s_h[b >> 1], 1u << ((b & 1u) << 4), __ATOMIC_RELAXED,
                                       __HIP_MEMORY_SCOPE_WORKGROUP);
            }
        }
    }
    if (acc == 0x12345678u || wrapc) sink[0] = acc + wrapc;
    __syncthreads();
    uint32_t *dst = part + (uint64_t)blockIdx.x * kWords;
    for (uint32_t i = tid; i < kWords; i += BLOCK) dst[i] = s_h[i];
}
}  // namespace

int main(int argc, char **argv) {
    const uint64_t n = 1ull << 28;
    const uint32_t ntiles = (uint32_t)(n / kSweepTile);
    const int reps = 10;
    uint32_t *in, *part, *part_ref, *sink;
    uint64_t *fix;
    CK(hipMalloc(&in, n * 4));
    CK(hipMalloc(&part, (size_t)kH16Blocks * kH16PartWords * 4));
    CK(hipMalloc(&part_ref, (size_t)kH16Blocks * kH16PartWords * 4));
    CK(hipMalloc(&fix, (size_t)kH16Shards * kBuckets16 * 8));
    CK(hipMalloc(&sink, 64));
    CK(launch_generate(0, 42, 0, n, reinterpret_cast<int32_t *>(in), 0));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    const size_t pbytes = (size_t)kH16Blocks * kH16PartWords * 4;
    std::vector<uint32_t> h_ref(pbytes / 4), h(pbytes / 4);
    auto time = [&](const char *name, auto launch, bool check) {
        std::vector<float> t;
        for (int r = 0; r < reps + 2; ++r) {
            CK(hipMemset(fix, 0, (size_t)kH16Shards * kBuckets16 * 8));
            CK(hipEventRecord(e0, 0));
            launch();
            CK(hipEventRecord(e1, 0));
            CK(hipEventSynchronize(e1));
            float ms;
            CK(hipEventElapsedTime(&ms, e0, e1));
            if (r >= 2) t.push_back(ms);
        }
        std::sort(t.begin(), t.end());
        const char *ok = "";
        if (check) {
            CK(hipMemcpy(h.data(), part, pbytes, hipMemcpyDeviceToHost));
            ok = h == h_ref ? "  partials == product" : "  PARTIALS DIFFER";
        }
        printf("%-34s median %.4f ms  min %.4f  (%.0f GB/s)%s\n", name, t[t.size() / 2], t[0],
               n * 4.0 / (t[t.size() / 2] * 1e-3) / 1e9, ok);
        fflush(stdout);
    };
    uint32_t nblk = 0;
    time("product k_hist16", [&] {
        CK(launch_hist16(in, n, true, part_ref, fix, &nblk, 0));
    }, false);
    CK(hipMemcpy(h_ref.data(), part_ref, pbytes, hipMemcpyDeviceToHost));
    // the product kernel right after a 1 GiB write-heavy pass (as in a sort loop, where K1h
    // follows the previous sort's K11): is K1h slowed by the dirty lines draining?
    {
        uint32_t *junk;
        CK(hipMalloc(&junk, n * 4));
        std::vector<float> t;
        for (int r = 0; r < reps + 2; ++r) {
            CK(launch_stream_copy(in, junk, n * 4, 0));
            CK(hipMemset(fix, 0, (size_t)kH16Shards * kBuckets16 * 8));
            CK(hipEventRecord(e0, 0));
            CK(launch_hist16(in, n, true, part_ref, fix, &nblk, 0));
            CK(hipEventRecord(e1, 0));
            CK(hipEventSynchronize(e1));
            float ms;
            CK(hipEventElapsedTime(&ms, e0, e1));
            if (r >= 2) t.push_back(ms);
        }
        std::sort(t.begin(), t.end());
        printf("%-34s median %.4f ms  min %.4f\n", "product after 1 GiB copy", t[t.size() / 2], t[0]);
        t.clear();
        for (int r = 0; r < reps + 2; ++r) {
            CK(launch_stream_copy(in, junk, n * 4, 0));
            CK(hipDeviceSynchronize());
            CK(hipMemset(fix, 0, (size_t)kH16Shards * kBuckets16 * 8));
            CK(hipEventRecord(e0, 0));
            CK(launch_hist16(in, n, true, part_ref, fix, &nblk, 0));
            CK(hipEventRecord(e1, 0));
            CK(hipEventSynchronize(e1));
            float ms;
            CK(hipEventElapsedTime(&ms, e0, e1));
            if (r >= 2) t.push_back(ms);
        }
        std::sort(t.begin(), t.end());
        printf("%-34s median %.4f ms  min %.4f\n", "product after copy + host sync", t[t.size() / 2], t[0]);
        t.clear();
        for (int r = 0; r < reps + 2; ++r) {
            k_plain_copy<<<(unsigned)(n / 4 / 256), 256>>>((const v4u *)in, (v4u *)junk, n / 4);
            CK(hipDeviceSynchronize());
            CK(hipMemset(fix, 0, (size_t)kH16Shards * kBuckets16 * 8));
            CK(hipEventRecord(e0, 0));
            CK(launch_hist16(in, n, true, part_ref, fix, &nblk, 0));
            CK(hipEventRecord(e1, 0));
            CK(hipEventSynchronize(e1));
            float ms;
            CK(hipEventElapsedTime(&ms, e0, e1));
            if (r >= 2) t.push_back(ms);
        }
        std::sort(t.begin(), t.end());
        printf("%-34s median %.4f ms  min %.4f\n", "product after PLAIN-store copy", t[t.size() / 2], t[0]);
        CK(hipFree(junk));
    }
    const unsigned G = nblk;
#define V(L, A, D, S, chk)                                                                  \
    time("L" #L " A" #A " D" #D " S" #S, [&] { k1h<L, A, D, S><<<G, BLOCK>>>(in, ntiles, part, sink); }, chk)
    V(0, 1, 1, false, true);
    V(0, 0, 1, false, false);
    V(1, 0, 1, false, false);
    V(0, 0, 2, false, false);
    V(1, 0, 2, false, false);
    V(0, 1, 1, true, false);
    V(0, 2, 1, true, false);
    V(1, 1, 1, false, true);
    V(1, 1, 2, false, true);
    V(0, 1, 2, false, true);
    V(1, 2, 1, false, true);
    V(1, 2, 2, false, true);
    return 0;
}
