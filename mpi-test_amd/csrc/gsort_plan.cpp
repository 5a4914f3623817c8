// gsort_plan.cpp -- host-side planning of the distributed passes (no GPU code).
//
// The reference moves every key through rank 0 on every radix pass (MPI_Scatter at
// mpi_radix_sort.c:139, MPI_Gatherv at :192) so that rank q always holds positions
// [qB, (q+1)B) of the partially sorted array.  The build keeps that block invariant without
// the round trip: from the all-gathered per-rank digit counts every rank computes the global
// position of each (source rank, digit) run and therefore which contiguous slice of its
// locally digit-sorted block goes to which destination, and where received runs land.
#include <math.h>
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

// Exact split of P locally sorted blocks into the global balanced blocks [qB, (q+1)B).
// For each inner boundary q (1..P-1) at global position g_q = min(qB, N), v_q is the g_q-th
// smallest key (found on device by radix select, gsort_runtime.cpp), lt[p][q-1] / le[p][q-1]
// = keys of rank p that are < / <= v_q.  Copies of v_q left of the boundary
// (L_q = g_q - sum_p lt) are taken from the ranks in rank order, so rank p's block is cut at
//   s_p(q) = lt_p(q) + clamp(L_q - sum_{p'<p} eq_{p'}(q), 0, eq_p(q)),   eq = le - lt,
// with s_p(0) = 0, s_p(P) = n_p and s_p(q) = n_p when g_q >= N.  Rank me sends
// [s_me(q), s_me(q+1)) to q and receives s_p(me+1) - s_p(me) keys from each p.
// (Replaces the per-pass digit routing through rank 0, mpi_radix_sort.c:139,150-192: one
// exchange instead of one per base-P digit.)
// balanced (gsort_plan_split_balanced): v_q is the q-th sample splitter instead, so g_q need
// not fall among its copies; the boundary moves to clamp(min(qB, N), LT_q + 1, LE_q) -- as
// close to qB as v_q's copies allow, keeping at least one copy left as the reference's rule
// does (keys <= s go left), so a splitter value held once gives exactly the reference's
// bucket -- and the copies are again taken in rank order.
static gsort_status plan_split(int P, const uint64_t *n_all, const uint64_t *lt,
                               const uint64_t *le, int me, uint64_t *send, uint64_t *recv,
                               bool balanced) {
    if (P < 1 || !n_all || (P > 1 && (!lt || !le)) || !send || !recv || me < 0 || me >= P)
        return GSORT_EINVAL;
    uint64_t N = 0;
    for (int p = 0; p < P; ++p) N += n_all[p];
    const uint64_t B = (N + P - 1) / P;
    // cut[p][q], q = 0..P
    std::vector<uint64_t> cut((size_t)P * (P + 1), 0);
    for (int p = 0; p < P; ++p) cut[(size_t)p * (P + 1) + P] = n_all[p];
    for (int q = 1; q < P; ++q) {
        uint64_t g = std::min<uint64_t>((uint64_t)q * B, N);
        uint64_t lt_all = 0, le_all = 0, eq_before = 0;
        for (int p = 0; p < P; ++p) {
            lt_all += lt[(size_t)p * (P - 1) + (q - 1)];
            le_all += le[(size_t)p * (P - 1) + (q - 1)];
        }
        if (balanced) {
            if (le_all < lt_all || le_all > N) return GSORT_EINVAL;
            g = std::min(std::max(g, lt_all + (le_all > lt_all ? 1 : 0)), le_all);
        }
        if (g >= N) {
            for (int p = 0; p < P; ++p) cut[(size_t)p * (P + 1) + q] = n_all[p];
            continue;
        }
        if (lt_all > g) return GSORT_EINVAL;  // counts inconsistent with v_q
        const uint64_t L = g - lt_all;
        for (int p = 0; p < P; ++p) {
            const uint64_t l = lt[(size_t)p * (P - 1) + (q - 1)];
            const uint64_t e = le[(size_t)p * (P - 1) + (q - 1)];
            if (e < l || e > n_all[p]) return GSORT_EINVAL;
            const uint64_t eq = e - l;
            const uint64_t want = L > eq_before ? L - eq_before : 0;
            cut[(size_t)p * (P + 1) + q] = l + std::min(want, eq);
            eq_before += eq;
        }
    }
    for (int q = 0; q < P; ++q) {
        const uint64_t a = cut[(size_t)me * (P + 1) + q], b = cut[(size_t)me * (P + 1) + q + 1];
        if (b < a) return GSORT_EINVAL;
        send[q] = b - a;
        const uint64_t ra = cut[(size_t)q * (P + 1) + me], rb = cut[(size_t)q * (P + 1) + me + 1];
        if (rb < ra) return GSORT_EINVAL;
        recv[q] = rb - ra;
    }
    return GSORT_OK;
}

extern "C" gsort_status gsort_plan_split(int P, const uint64_t *n_all, const uint64_t *lt,
                                         const uint64_t *le, int me, uint64_t *send,
                                         uint64_t *recv) {
    return plan_split(P, n_all, lt, le, me, send, recv, false);
}

extern "C" gsort_status gsort_plan_split_balanced(int P, const uint64_t *n_all,
                                                  const uint64_t *lt, const uint64_t *le, int me,
                                                  uint64_t *send, uint64_t *recv) {
    return plan_split(P, n_all, lt, le, me, send, recv, true);
}

// The reference radix sort's digit plan for the compat key map (gsort_set_ref_compat):
//   loop     = number_digits(max_element, P) = (int)(log(|max| or 1) / log(P)) + 1
//              (mpi_radix_sort.c:48-52, :91, :100; max_element starts at -1, :77)
//   mod[d]   = (int)pow(P, d + 1)     the modulus of number_digit_at at position d + 1 (:57)
//   scale[d] = pow(P, d)              its divisor
// with glibc's log / pow and x86's double -> int conversion (cvttsd2si: every out-of-range
// value, inf and nan become INT_MIN), so P = 1 gives loop = INT_MIN + 1 (no pass, quirk Q1) and
// P = 3 reproduces the reference's floating-point digit under-count (Q3).
static int x86_dtoi(double x) {
    if (!(x > -2147483649.0 && x < 2147483648.0)) return INT32_MIN;
    return (int)x;
}

extern "C" gsort_status gsort_plan_ref_digits(int P, int32_t max_element, int *loop,
                                              int32_t *mod, double *scale, int cap) {
    if (P < 1 || !loop) return GSORT_EINVAL;
    const int64_t mag = max_element < 0 ? -(int64_t)max_element : max_element;
    if (max_element == INT32_MIN) return GSORT_EINVAL;  // abs(INT_MIN) is undefined there
    const double l = log(mag > 0 ? (double)mag : 1.0) / log((double)P);
    const int lp = x86_dtoi(l);
    *loop = lp == INT32_MIN ? INT32_MIN + 1 : lp + 1;
    if (*loop > cap) return (mod || scale) ? GSORT_EINVAL : GSORT_OK;
    for (int d = 0; d < *loop; ++d) {
        if (mod) mod[d] = x86_dtoi(pow((double)P, (double)(d + 1)));
        if (scale) scale[d] = pow((double)P, (double)d);
    }
    return GSORT_OK;
}
