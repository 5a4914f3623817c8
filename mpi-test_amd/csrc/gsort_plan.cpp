// gsort_plan.cpp -- host-side planning of the distributed passes (no GPU code).
//
// The reference moves every key through rank 0 on every radix pass (MPI_Scatter at
// mpi_radix_sort.c:139, MPI_Gatherv at :192) so that rank q always holds positions
// [qB, (q+1)B) of the partially sorted array.  The build keeps that block invariant without
// the round trip: from the all-gathered per-rank digit counts every rank computes the global
// position of each (source rank, digit) run and therefore which contiguous slice of its
// locally digit-sorted block goes to which destination, and where received runs land.
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <vector>

#include "gsort.h"

extern "C" gsort_status gsort_plan_radix_route(int P, const uint64_t *hist, uint64_t B, int me,
                                               uint64_t *send, uint64_t *recv, uint64_t *seg,
                                               size_t *nseg) {
    if (P < 1 || !hist || !send || !recv || !seg || !nseg || me < 0 || me >= P)
        return GSORT_EINVAL;
    // G[d]: global start of digit d; R[r][d]: keys of digit d on ranks < r (stable order:
    // digit, then source rank, then source order -- mpi_radix_sort.c:164-173 + :185-192).
    std::vector<uint64_t> G(256), run(256, 0);
    uint64_t total = 0;
    for (int d = 0; d < 256; ++d) {
        G[d] = total;
        for (int r = 0; r < P; ++r) total += hist[(size_t)r * 256 + d];
    }
    for (int q = 0; q < P; ++q) send[q] = recv[q] = 0;
    const uint64_t lo = (uint64_t)me * B, hi = lo + B;
    size_t rows = 0;
    for (int r = 0; r < P; ++r) {
        uint64_t chunk = 0;
        for (int d = 0; d < 256; ++d) {
            const uint64_t c = hist[(size_t)r * 256 + d];
            const uint64_t a = G[d] + run[d], e = a + c;  // global range of run (r, d)
            run[d] += c;
            if (c == 0) continue;
            if (r == me) {
                // destinations of this run: blocks overlapping [a, e)
                for (uint64_t q = a / B; q < (uint64_t)P && q * B < e; ++q) {
                    const uint64_t x = std::max(a, q * B), y = std::min(e, (q + 1) * B);
                    if (y > x) send[q] += y - x;
                }
            }
            const uint64_t x = std::max(a, lo), y = std::min(e, hi);
            if (y > x) {
                seg[4 * rows + 0] = (uint64_t)r;
                seg[4 * rows + 1] = chunk;
                seg[4 * rows + 2] = x - lo;
                seg[4 * rows + 3] = y - x;
                ++rows;
                chunk += y - x;
                recv[r] += y - x;
            }
        }
    }
    *nseg = rows;
    return GSORT_OK;
}

extern "C" gsort_status gsort_plan_splitters(int P, const int32_t *samples, int32_t *splitters) {
    if (P < 1 || !samples || (P > 1 && !splitters)) return GSORT_EINVAL;
    const int k = 2 * P - 1;
    std::vector<int32_t> s(samples, samples + (size_t)P * k);
    std::sort(s.begin(), s.end());
    for (int i = 0; i < P - 1; ++i) splitters[i] = s[(size_t)(i + 1) * k];
    return GSORT_OK;
}
