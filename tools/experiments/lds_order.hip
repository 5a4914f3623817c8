// lds_order.hip -- does ds_add_rtn_u32 hand out return values in lane order when several lanes
// of ONE instruction hit the same LDS address?  (development probe, not the product)
// Every wave runs R rounds of `r = atomicAdd(&cnt[wave][digit], 1)` over per-wave counters and
// stores r; the host checks that, per wave and digit, r increases in (round, lane) order.
#include <stdio.h>
#include <stdlib.h>

#include <vector>

#include <hip/hip_runtime.h>

#define CK(x)                                                                         \
    do {                                                                              \
        hipError_t e = (x);                                                           \
        if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); exit(1); } \
    } while (0)

constexpr int BLOCK = 512, WAVES = 8, R = 16;

__global__ __launch_bounds__(BLOCK) void probe(const uint32_t *digits, uint32_t *ranks,
                                               uint32_t nbins) {
    __shared__ uint32_t cnt[WAVES * 256];
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    for (int i = tid; i < WAVES * 256; i += BLOCK) cnt[i] = 0;
    __syncthreads();
    const uint64_t base = ((uint64_t)blockIdx.x * WAVES + w) * 64 * R;
    uint32_t d[R], r[R];
#pragma unroll
    for (int i = 0; i < R; ++i) d[i] = digits[base + i * 64 + lane] % nbins;
#pragma unroll
    for (int i = 0; i < R; ++i) r[i] = atomicAdd(&cnt[w * 256 + d[i]], 1u);
#pragma unroll
    for (int i = 0; i < R; ++i) ranks[base + i * 64 + lane] = r[i];
}

int main(int argc, char **argv) {
    const int nblocks = argc > 1 ? atoi(argv[1]) : 4096;
    const uint64_t n = (uint64_t)nblocks * BLOCK * R;
    uint32_t *d_dig, *d_rank;
    CK(hipMalloc(&d_dig, n * 4));
    CK(hipMalloc(&d_rank, n * 4));
    std::vector<uint32_t> dig(n), rank(n);
    uint64_t x = 88172645463325252ull;
    for (auto &v : dig) { x ^= x << 13; x ^= x >> 7; x ^= x << 17; v = (uint32_t)x; }
    CK(hipMemcpy(d_dig, dig.data(), n * 4, hipMemcpyHostToDevice));
    uint64_t total_bad = 0, total_checked = 0;
    for (uint32_t nbins : {1u, 2u, 3u, 7u, 16u, 64u, 256u}) {
        for (int rep = 0; rep < 3; ++rep) {
            probe<<<nblocks, BLOCK>>>(d_dig, d_rank, nbins);
            CK(hipDeviceSynchronize());
            CK(hipMemcpy(rank.data(), d_rank, n * 4, hipMemcpyDeviceToHost));
            uint64_t bad = 0;
            for (uint64_t wv = 0; wv < n / (64 * R); ++wv) {
                std::vector<int64_t> last(256, -1);
                for (int i = 0; i < R; ++i)
                    for (int l = 0; l < 64; ++l) {
                        const uint64_t p = wv * 64 * R + i * 64 + l;
                        const uint32_t dd = dig[p] % nbins;
                        if ((int64_t)rank[p] != last[dd] + 1) ++bad;
                        last[dd] = rank[p];
                    }
            }
            total_bad += bad;
            total_checked += n;
            printf("{\"bins\": %u, \"rep\": %d, \"keys\": %llu, \"out_of_lane_order\": %llu}\n",
                   nbins, rep, (unsigned long long)n, (unsigned long long)bad);
        }
    }
    printf("{\"total_checked\": %llu, \"total_bad\": %llu}\n", (unsigned long long)total_checked,
           (unsigned long long)total_bad);
    return 0;
}
