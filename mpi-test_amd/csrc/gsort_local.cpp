// gsort_local.cpp -- the one-rank sorts of libgsort: the LSD passes, the MSD
// levels, the exact two-level plan, the sampled plan, the counted dominant child, and
// msd_sort / local_sort that pick among them.
// Reference being replaced: the per-key digit loop of mpi_radix_sort.c:144-147 and the local
// qsort of mpi_sample_sort.c:85 / :174.
#include "gsort_ctx.h"

namespace gsort {
namespace rt {

// ---- LSD local sort: K1 (+ all four histograms) then per non-trivial digit K1/K2/K3 -----
// Reference: the per-key digit loop mpi_radix_sort.c:144-147 (there: base P, all passes
// through rank 0) and the local qsort mpi_sample_sort.c:85 / :174.
gsort_status lsd_sort(gsort_ctx *c, const uint32_t *in, uint64_t n, uint32_t *out,
                      uint32_t *tmp, int *passes_run) {
    if (passes_run) *passes_run = 0;
    if (n == 0) return GSORT_OK;
    ST_TRY(ensure_pass_scratch(c, n));
    uint64_t *d_hist = reinterpret_cast<uint64_t *>(c->d_small + OFF_HIST);
    uint64_t *h_hist = reinterpret_cast<uint64_t *>(c->h_small + OFF_HIST);
    HIP_TRY(c, hipMemsetAsync(d_hist, 0, 4 * kRadix * 8, c->stream));
    hipEvent_t t = tic(c);
    HIP_TRY(c, launch_tile_counts(in, n, 0, true, d_tcounts(c), d_hist, c->stream));
    toc(c, PH_COUNT, t);
    HIP_TRY(c, hipMemcpyAsync(h_hist, d_hist, 4 * kRadix * 8, hipMemcpyDeviceToHost, c->stream));
    HIP_TRY(c, hipStreamSynchronize(c->stream));
    int active[4], k = 0;
    for (int p = 0; p < 4; ++p) {
        const uint64_t *h = h_hist + p * kRadix;
        if (*std::max_element(h, h + kRadix) < n) active[k++] = p;  // skip trivial digits
    }
    if (k == 0) {
        HIP_TRY(c, launch_copy(in, out, n, c->stream));
        return GSORT_OK;
    }
    const uint32_t *src = in;
    for (int i = 0; i < k; ++i) {
        uint32_t *dst = ((k - 1 - i) % 2 == 0) ? out : tmp;
        if (!(i == 0 && active[0] == 0)) ST_TRY(count_tiles(c, src, n, active[i], i == 0));
        ST_TRY(scan_and_scatter(c, src, dst, n, active[i], i == 0, i == k - 1));
        src = dst;
    }
    if (passes_run) *passes_run = k;
    return GSORT_OK;
}

// The MSD levels L, L-1, .. 0 (gsort_kernels.hip, "MSD partition sort").  On entry h holds
// the counters of the work lists filled by level L+1: m_next[cur_list] (buckets still larger
// than kLocalMax, ordered u32 in `cur`) and m_local[k] (K11 buckets of `cur`, digits L..0
// left).  Level L partitions cur -> the other buffer (tmp <-> out); level 0 stores int32 into
// out, as does K11.
// flip_first: cur is the int32 input itself (the first level flips on load).
gsort_status msd_levels(gsort_ctx *c, int L, uint32_t *cur, uint32_t *out, uint32_t *tmp,
                        int cur_list, uint64_t *h, gsort_stats *stats, int *levels,
                        int last_level, uint16_t *out16, bool flip_first) {
    auto lst = [](DevBuf &b) { return reinterpret_cast<uint64_t *>(b.p); };
    uint64_t *ctr = reinterpret_cast<uint64_t *>(c->d_small + OFF_CTR);
    auto lists = [&](int next) { return work_lists(c, next); };
    hipEvent_t t;
    for (;; --L) {
        for (int k = 0; k < kLocalClasses; ++k) {  // buckets finished in LDS: digits L..0 remain
            const uint64_t *hk = h + 3 * (k + 1);
            if (!hk[0]) continue;
            t = tic(c);
            HIP_TRY(c, launch_local_sort(cur, out, lst(c->m_local[k]), (uint32_t)hk[0], k + 1,
                                         L + 1, false, c->atomic_rank, c->stream));
            toc(c, PH_BUCKET, t);
            if (stats) { stats->buckets_local += hk[0]; stats->keys_bucket_sort += hk[1]; }
        }
        const uint64_t nseg = h[0], keys = h[1];
        if (nseg == 0 || L < 0) break;
        uint32_t *dst = cur == tmp ? out : tmp;
        const uint64_t max_tiles = sweep_tiles(keys) + nseg;
        const uint64_t max_groups = (max_tiles + kScanGroup - 1) / kScanGroup + nseg;
        ST_TRY(ensure(c, c->m_tpfx, (nseg + 1) * 4));
        ST_TRY(ensure(c, c->m_gpfx, (nseg + 1) * 4));
        ST_TRY(ensure(c, c->m_segmap, max_tiles * 4));
        ST_TRY(ensure(c, c->m_groupmap, max_groups * 4));
        ST_TRY(ensure(c, c->tcounts, max_tiles * kRadix * 4));
        ST_TRY(ensure(c, c->gsum, max_groups * kRadix * 8));
        ST_TRY(ensure(c, c->m_cstart, nseg * kRadix * 8));
        const uint64_t child_cap = std::min<uint64_t>(nseg * kRadix, keys);
        ST_TRY(ensure_list(c, c->m_next[cur_list ^ 1], std::min<uint64_t>(child_cap, keys / kLocalMax + 1)));
        for (int k = 0; k < kLocalClasses; ++k)
            ST_TRY(ensure_list(c, c->m_local[k],
                               std::min<uint64_t>(child_cap, keys / (kLocalCap[k] + 1) + 1)));
        SegPass sp;
        sp.in = cur;
        sp.out = dst;
        sp.flip_in = flip_first;
        flip_first = false;
        sp.segs = lst(c->m_next[cur_list]);
        sp.nseg = (uint32_t)nseg;
        sp.shift = 8 * L;
        sp.flip_out = L == last_level;
        sp.max_tiles = (uint32_t)max_tiles;
        sp.max_groups = (uint32_t)max_groups;
        sp.tpfx = reinterpret_cast<uint32_t *>(c->m_tpfx.p);
        sp.gpfx = reinterpret_cast<uint32_t *>(c->m_gpfx.p);
        sp.segmap = reinterpret_cast<uint32_t *>(c->m_segmap.p);
        sp.groupmap = reinterpret_cast<uint32_t *>(c->m_groupmap.p);
        sp.tcounts = d_tcounts(c);
        sp.gsum = d_gsum(c);
        sp.cstart = reinterpret_cast<uint64_t *>(c->m_cstart.p);
        sp.lists = lists(cur_list ^ 1);
        // digit 0: every child is a run of equal keys; a partition-only sort stops here too
        if (L == last_level) sp.lists.ctr = nullptr;
        if (L == last_level) sp.out16 = out16;
        t = tic(c);
        HIP_TRY(c, hipMemsetAsync(ctr, 0, kCtrBytes, c->stream));
        HIP_TRY(c, launch_seg_count(sp, c->stream));
        toc(c, PH_COUNT, t);
        t = tic(c);
        HIP_TRY(c, launch_seg_partition(sp, c->stream));
        toc(c, PH_LEVEL3 + (3 - L), t);
        if (stats) stats->keys_level[3 - L] += keys;
        ++*levels;
        if (L == last_level) break;
        ST_TRY(read_counters(c, h));
        cur = dst;
        cur_list ^= 1;
    }
    return GSORT_OK;
}


// Mailbox waits poll the stream for errors (a stream that went idle without the word) only
// every kQueryUs of waiting: each hipStreamQuery puts a marker in the stream, and one every
// 1024 spins (~1 us) during the sampled plan's eligibility wait queued dozens of them between
// K12g and K11e -- a ~6 us bubble (profiles/r04_ab_stream_query_rate.txt: 1.376 -> 1.369 ms).
constexpr int kQueryUs = 200;
struct QueryTimer {  // (every 1024 spins the waiting thread yields; the query only when due)
    std::chrono::steady_clock::time_point next = std::chrono::steady_clock::now() +
                                                 std::chrono::microseconds(kQueryUs);
    bool due() {
        const auto now = std::chrono::steady_clock::now();
        if (now < next) return false;
        next = now + std::chrono::microseconds(kQueryUs);
        return true;
    }
};

// Wait for K12p's sequence number seq in the mailbox (the counters behind it are then
// visible).  A stream error, or the stream going idle without the flag, returns GSORT_EHIP
// instead of spinning forever.
gsort_status wait_mail(gsort_ctx *c, uint64_t seq, hipStream_t s) {
    volatile uint64_t *flag = c->h_mail;
    QueryTimer qt;
    if (!s) s = c->stream;
    for (uint64_t spin = 0; *flag != seq; ++spin) {
        if ((spin & 1023) == 1023) {
            const hipError_t q = qt.due() ? hipStreamQuery(s) : hipErrorNotReady;
            if (q != hipErrorNotReady && *flag != seq) {
                if (q != hipSuccess)
                    return set_err(c, GSORT_EHIP, std::string("K12p counters: ") +
                                                      hipGetErrorString(q) + " (rank " +
                                                      std::to_string(c->rank) + ")");
                return set_err(c, GSORT_EHIP, "K12p counters: stream idle without the flag");
            }
            std::this_thread::yield();
        }
    }
    std::atomic_thread_fence(std::memory_order_acquire);
    return GSORT_OK;
}

// Levels 3 and 2 through the two-level plan (gsort_kernels.hip, "Two-level plan"): K1h (the
// 16-bit histogram) + K12a/K12b (counts, bases, bucket bounds, cursors, work lists), then K3r
// (level 3, in -> tmp, runs reserved on per-shard bucket cursors) and K3a (level 2, tmp -> out,
// or the low 16 bits -> out16 with group16).  The work-list counters are copied to the host
// right after K12b and read once levels 3 and 2 are queued, so the GPU never waits on the host
// in the common case.  Then K11 for the small level-3 buckets (three digits, tmp -> out) and
// for the level-2 children (two digits, in place in out); children still larger than kLocalMax
// go on through msd_levels from level 1.  cstart (65537 u64) receives the 16-bit bucket bounds.
gsort_status msd_sort_h16(gsort_ctx *c, const uint32_t *in, uint64_t n, uint32_t *out,
                          uint32_t *tmp, gsort_stats *stats, bool group16, uint16_t *out16,
                          uint64_t *cstart) {
    uint64_t *totals = reinterpret_cast<uint64_t *>(c->d_small + OFF_TOT);
    uint64_t *bases = reinterpret_cast<uint64_t *>(c->d_small + OFF_BASES);
    uint64_t *ctr = reinterpret_cast<uint64_t *>(c->d_small + OFF_CTR);
    uint64_t *ctr3 = reinterpret_cast<uint64_t *>(c->d_small + OFF_CTR3);
    constexpr size_t kFixBytes = (size_t)kH16Shards * kBuckets16 * 8;
    ST_TRY(ensure(c, c->m_part, (size_t)kH16Blocks * kH16PartWords * 4));
    ST_TRY(ensure(c, c->m_fix, kFixBytes));
    ST_TRY(ensure(c, c->m_cur, (size_t)kBuckets16 * 4));
    ST_TRY(ensure(c, c->m_tpfx, (kRadix + 1) * 4));
    ST_TRY(ensure(c, c->m_ccount, (size_t)kBuckets16 * 8));
    ST_TRY(ensure(c, c->m_t3, (size_t)(kH16Shards + 1) * kRadix * 8));
    ST_TRY(ensure(c, c->m_cur3, (size_t)kH16Shards * kRadix * 4));
    ST_TRY(ensure(c, c->m_tdesc, (size_t)(sweep_tiles(n) + kRadix) * kTileDescBytes));
    if (!cstart) {
        ST_TRY(ensure(c, c->m_cstart, (size_t)(kBuckets16 + 1) * 8));
        cstart = reinterpret_cast<uint64_t *>(c->m_cstart.p);
    }
    const uint64_t nchild = std::min<uint64_t>(kBuckets16, n);
    WorkLists wl2 = work_lists(c, 0), wl3 = work_lists(c, 1);
    if (!group16) {
        ST_TRY(ensure_list(c, c->m_next[0], std::min<uint64_t>(nchild, n / kLocalMax + 1)));
        ST_TRY(ensure_list(c, c->m_next[1], 1));
        for (int k = 0; k < kLocalClasses; ++k) {
            ST_TRY(ensure_list(c, c->m_local[k],
                               std::min<uint64_t>(nchild, n / (kLocalCap[k] + 1) + 1)));
            ST_TRY(ensure_list(c, c->m_local3[k], kRadix));
        }
        wl2 = work_lists(c, 0);
        wl3 = work_lists(c, 1);
        for (int k = 0; k < kLocalClasses; ++k)
            wl3.list[k + 1] = reinterpret_cast<uint64_t *>(c->m_local3[k].p);
        wl3.ctr = ctr3;
    } else {
        wl2.ctr = nullptr;
        wl3.ctr = nullptr;
    }
    uint32_t *tpfx = reinterpret_cast<uint32_t *>(c->m_tpfx.p);
    uint32_t *cur = reinterpret_cast<uint32_t *>(c->m_cur.p);
    uint32_t *cur3 = reinterpret_cast<uint32_t *>(c->m_cur3.p);
    uint64_t *t3 = reinterpret_cast<uint64_t *>(c->m_t3.p);
    uint32_t nblk = 0;
    constexpr uint32_t kCtrWords = (uint32_t)((OFF_CTR3 + kCtrBytes - OFF_CTR) / 8);
    // K12b's trivial-level word (zeroed by K12a and published with the counters); the
    // distributed sender (group16) needs every level's output, so it never skips
    uint32_t *flags = group16 ? nullptr : reinterpret_cast<uint32_t *>(c->d_small + OFF_FLAGS);
    static_assert(kCtrWords <= kRadix && kCtrWords * 8 <= kMailBytes - 64, "counter words");
    if (c->fix_clean != c->m_fix.p)  // new allocation: K12a keeps it zero from here on
        HIP_TRY(c, hipMemsetAsync(c->m_fix.p, 0, kFixBytes, c->stream));
    c->fix_clean = nullptr;
    hipEvent_t t = tic(c);
    HIP_TRY(c, launch_hist16(in, n, true, reinterpret_cast<uint32_t *>(c->m_part.p),
                             reinterpret_cast<uint64_t *>(c->m_fix.p), &nblk, c->stream));
    HIP_TRY(c, launch_plan16(reinterpret_cast<uint32_t *>(c->m_part.p), nblk,
                             reinterpret_cast<uint64_t *>(c->m_fix.p), n, group16,
                             reinterpret_cast<uint64_t *>(c->m_ccount.p), t3,
                             t3 + (size_t)kH16Shards * kRadix, bases, totals, cstart, cur, cur3,
                             tpfx, wl2, wl3, group16 ? nullptr : ctr, kCtrWords, flags,
                             c->stream));
    c->fix_clean = c->m_fix.p;
    const uint64_t seq = ++c->mail_seq;
    if (!group16)
        HIP_TRY(c, launch_publish(ctr, kCtrWords, c->d_mail + 8, c->d_mail, seq, c->stream));
    toc(c, PH_COUNT, t);
    t = tic(c);
    HIP_TRY(c, launch_partition3r(in, tmp, n, cur3, bases, flags, c->stream));
    toc(c, PH_LEVEL3, t);
    t = tic(c);
    HIP_TRY(c, launch_partition2r(tmp, out, group16 ? out16 : nullptr, n, tpfx, c->m_tdesc.p,
                                  bases, totals, cur, flags, in, c->stream));
    toc(c, PH_LEVEL2, t);
    int levels = 2;
    if (group16 && stats) { stats->keys_level[0] += n; stats->keys_level[1] += n; }
    if (!group16) {
        ST_TRY(wait_mail(c, seq));
        uint64_t h[3 * (kLocalClasses + 1)], h3[3 * (kLocalClasses + 1)];
        const char *mail = reinterpret_cast<const char *>(c->h_mail + 8);
        memcpy(h, mail, kCtrBytes);
        memcpy(h3, mail + (OFF_CTR3 - OFF_CTR), kCtrBytes);
        uint32_t fl = 0;
        memcpy(&fl, mail + (OFF_FLAGS - OFF_CTR), 4);
        const bool triv3 = fl & 1u, triv2 = fl & 2u;
        levels = 2 - (int)triv3 - (int)triv2;
        if (stats) {
            if (!triv3) stats->keys_level[0] += n;
            if (!triv2) stats->keys_level[1] += n;
            for (int k = 0; k < kLocalClasses; ++k)  // K11'd whole at level 3
                stats->keys_level[1] -= std::min<uint64_t>(h3[3 * (k + 1) + 1],
                                                           stats->keys_level[1]);
        }
        if (triv2) {  // levels 3 and 2 moved nothing: level 1 reads the int32 input
            if (stats) stats->passes_run = levels;
            ST_TRY(msd_levels(c, 1, const_cast<uint32_t *>(in), out, tmp, 0, h, stats, &levels,
                              0, nullptr, true));
            if (stats) stats->passes_run = levels;
            return GSORT_OK;
        }
        for (int k = 0; k < kLocalClasses; ++k) {
            const uint64_t *hk = h3 + 3 * (k + 1);
            if (!hk[0]) continue;
            t = tic(c);
            HIP_TRY(c, launch_local_sort(tmp, out, reinterpret_cast<uint64_t *>(c->m_local3[k].p),
                                         (uint32_t)hk[0], k + 1, 3, false, c->atomic_rank,
                                         c->stream));
            toc(c, PH_BUCKET, t);
            if (stats) { stats->buckets_local += hk[0]; stats->keys_bucket_sort += hk[1]; }
        }
        ST_TRY(msd_levels(c, 1, out, out, tmp, 0, h, stats, &levels));
    }
    if (stats) stats->passes_run = levels;
    return GSORT_OK;
}

// The sampled plan (gsort_kernels.hip, "Sampled plan"): levels 3 and 2 into gapped regions
// sized from a 1/64 sample, K11e into out.  The host reads the eligibility / overflow words
// and the K11e list counts K12g leaves in the mailbox (one wait, after level 2), then launches
// K11e; *ok = false means nothing was written to out and the caller sorts on the exact plan.
// the sampled plan's mailbox words start here (EstPlan::mail: kEstMailWords of them)
constexpr size_t kEstMailWord = 400;
static_assert((kEstMailWord + kEstMailWords) * 8 <= kMailBytes, "mailbox");

// Keys of the region buffers the caps of `nreg` regions can add up to (k_est_plan's est_cap:
// max(a, b) <= a + b, Cauchy-Schwarz on the sigma terms: sum sqrt(cnt + 1) <=
// sqrt(nreg (m + nreg)); m >= the samples of all full blocks)
uint64_t est_region_keys(uint64_t n, uint64_t nreg, double slack) {
    const double m = (double)std::max<uint64_t>((n / kEstBlockKeysHost) * 8, 8);
    const double sig = 6.0 * ((double)n / m) * std::sqrt((double)nreg * (m + (double)nreg));
    const double floor2 = 2.0 * kEstBlockKeysHost * (double)nreg;
    return n + nreg + (uint64_t)std::ceil(slack * (sig + floor2 + 64.0 * (double)nreg)) + 1024;
}

// What an ineligible first attempt saw: the key bits that vary among the samples (against key
// 0) and the samples' min / max, all as ordered u32.
struct EstRetry {
    bool valid = false;
    uint32_t vary = 0, lo = 0, hi = 0, maxc = 0;  // maxc: samples of the largest child
};

// Leading bits shared by every key of a range (clz of its span), 32 for a single value.
int span_lead(uint32_t lo, uint32_t hi) { return hi > lo ? __builtin_clz(hi - lo) : 32; }

gsort_status msd_sort_est(gsort_ctx *c, const uint32_t *in, uint64_t n, uint32_t *out,
                          gsort_stats *stats, bool *ok, int sb = 0, uint32_t koff = 0,
                          EstRetry *retry = nullptr) {
    *ok = false;
    if (retry) *retry = EstRetry{};
    const double slack = std::max(c->est_slack, 0.0);
    const uint64_t capx = est_region_keys(n, (uint64_t)kH16Shards * kRadix, slack);
    const uint64_t capy = std::min<uint64_t>(est_region_keys(n, kBuckets16, slack),
                                             (uint64_t)kBuckets16 * kLocalMax);
    // the region buffers are the plan's only large allocations: without room for them (or for
    // its small plan arrays) the exact plan sorts (it needs none of them), and the regions are
    // handed back
    constexpr size_t kPlanWords = (size_t)4 * kBuckets16 + 4 * kH16Shards * kRadix + kRadix + 1;
    {
        // busy while they are made: a refused Y must not reclaim the X just ensured (that left
        // X null and K3r wrote through it -- found by test_region_buffers_reclaimed_for_a_later_call)
        c->est_busy = true;
        gsort_status st = GSORT_OK;
        for (DevBuf *b : {&c->m_ex, &c->m_ey})
            if (st == GSORT_OK) st = ensure(c, *b, b == &c->m_ex ? capx * 4 : capy * 2);  // Y: u16
        if (st == GSORT_OK)
            st = ensure(c, c->m_epart,
                        (size_t)kEstWGs * (kBuckets16 / 4 + kH16Shards * kRadix + 4) * 4);
        if (st == GSORT_OK) st = ensure(c, c->m_eplan, kPlanWords * 4 + 4 * kRadix * 8 + 64);
        if (st == GSORT_OK)
            st = ensure(c, c->m_edesc,
                        ((size_t)est_max_tiles(n) + kH16Shards * kRadix) * kTileDescBytes);
        if (st == GSORT_OK) st = ensure(c, c->m_edump, (size_t)kSweepTile * 4);
        for (int k = 0; k < kLocalClasses && st == GSORT_OK; ++k)
            st = ensure_list(c, c->m_local[k], kBuckets16);
        if (st == GSORT_OK) st = ensure_list(c, c->m_next[0], kBuckets16);  // K18c: > kLocalMax
        c->est_busy = false;
        if (st == GSORT_OK && (!c->m_ex.p || !c->m_ey.p))
            return set_err(c, GSORT_EINVAL, "sampled plan: region buffers missing");
        if (st == GSORT_ENOMEM) {
            (void)reclaim_regions(c, DevBuf{});
            c->err.clear();
            return GSORT_OK;  // *ok stays false
        }
        ST_TRY(st);
    }
    struct Busy {
        bool &f;
        explicit Busy(bool &x) : f(x) { f = true; }
        ~Busy() { f = false; }
    } busy(c->est_busy);
    EstPlan p{};
    p.in = in;
    p.n = n;
    p.flip_in = true;
    p.x = static_cast<uint32_t *>(c->m_ex.p);
    p.y = static_cast<uint16_t *>(c->m_ey.p);
    p.out = out;
    p.capx = capx;
    p.capy = capy;
    p.part8 = static_cast<uint32_t *>(c->m_epart.p);
    p.part3 = p.part8 + (size_t)kEstWGs * (kBuckets16 / 4);
    p.msamp = p.part3 + (size_t)kEstWGs * kH16Shards * kRadix;
    uint64_t *u64 = static_cast<uint64_t *>(c->m_eplan.p);
    p.r2 = u64;
    p.r3 = u64 + kRadix;
    p.bases3 = u64 + 2 * kRadix;
    p.bases2 = u64 + 3 * kRadix;
    uint32_t *w = reinterpret_cast<uint32_t *>(u64 + 4 * kRadix);
    p.capc = w;
    p.cur2 = w + kBuckets16;
    p.lim2 = w + 2 * kBuckets16;
    p.init2 = w + 3 * kBuckets16;
    w += 4 * kBuckets16;
    p.cap3 = w;
    p.cur3 = w + kH16Shards * kRadix;
    p.lim3 = w + 2 * kH16Shards * kRadix;
    p.init3 = w + 3 * kH16Shards * kRadix;
    p.tp = w + 4 * kH16Shards * kRadix;
    p.eflag = p.tp + kRadix + 2;  // 2 words, 8-B aligned (published as one u64)
    p.tdesc = c->m_edesc.p;
    p.dump = static_cast<uint32_t *>(c->m_edump.p);
    p.wl = work_lists(c, 0);
    p.slack = slack;
    p.atomic_rank = c->atomic_rank;
    p.sb = sb;
    p.koff = koff;
    p.mail = c->d_mail + kEstMailWord;
    p.seq_elig = ++c->mail_seq;
    p.seq_done = ++c->mail_seq;
    volatile uint64_t *mail = c->h_mail + kEstMailWord;
    // poll a sequence word of the mailbox; a stream that goes idle without it is an error
    auto wait_word = [&](size_t w, uint64_t seq, const char *what) -> gsort_status {
        QueryTimer qt;
        for (uint64_t spin = 0; mail[w] != seq; ++spin) {
            if ((spin & 1023) == 1023) {
                const hipError_t q = qt.due() ? hipStreamQuery(c->stream) : hipErrorNotReady;
                if (q != hipErrorNotReady && mail[w] != seq)
                    return set_err(c, GSORT_EHIP, std::string("sampled plan: ") + what + ": " +
                                                      (q == hipSuccess ? "stream idle without it"
                                                                       : hipGetErrorString(q)));
                std::this_thread::yield();
            }
        }
        std::atomic_thread_fence(std::memory_order_acquire);
        return GSORT_OK;
    };
    hipEvent_t t = tic(c);
    HIP_TRY(c, launch_est_front(p, c->stream));
    toc(c, PH_COUNT, t);
    t = tic(c);
    HIP_TRY(c, launch_est_level3(p, c->stream));  // block 0 publishes the eligibility word; all return at once on an ineligible block
    toc(c, PH_LEVEL3, t);
    // K12f, K3a and K12g return at once on an ineligible block too, so they are queued before
    // the host looks at the eligibility word (waiting first left a launch gap behind K3r)
    t = tic(c);
    HIP_TRY(c, launch_est_level2(p, c->stream));
    toc(c, PH_LEVEL2, t);
    HIP_TRY(c, launch_est_classify(p, c->stream));
    ST_TRY(wait_word(3, p.seq_elig, "eligibility word"));
    if (c->plan_trace)
        fprintf(stderr, "gsort plan: n %llu sb %d koff %u eflag %llx children %llu maxc %llx\n",
                (unsigned long long)n, sb, koff, (unsigned long long)mail[2],
                (unsigned long long)mail[4], (unsigned long long)mail[23]);
    if (mail[2] & 4u) {  // ineligible: the exact plan sorts -- unless the samples share leading
        // key bits (a key range narrower than int32: 16-, 20-, 24-, 28-bit keys, dense or
        // sorted ranges) whose removal leaves children K11e can take: then the caller retries
        // with every digit that many bits lower (at most 16, the plan's two levels).  One or
        // two shared bits (Zipf, any non-negative keys) rarely turn an ineligible block
        // eligible and are not worth a second sample.
        if (retry) {
            retry->vary = (uint32_t)mail[5];
            retry->lo = (uint32_t)mail[6];
            retry->hi = (uint32_t)mail[7];
            retry->maxc = (uint32_t)mail[23];
            retry->valid = true;
        }
        return GSORT_OK;
    }
    // K11e of the class the average child falls in, queued right behind K12g (a grid of the
    // sampled children: at least its entries, usually exactly), so no host round trip sits
    // between K12g and the largest K11e launch; the other classes follow once the counts are in
    const uint32_t sampled = (uint32_t)std::min<uint64_t>((uint64_t)mail[4], (uint64_t)kBuckets16);
    // (class 4 children go to K18c unless the plan is shifted by 8+ bits: the speculative grid
    // then is class 3's, whose blocks past its count return at once after block 0 has
    // published the counters)
    const int kmax = sb >= 8 ? kLocalClasses : kEstCx - 1;
    const int kspec = sampled ? std::min(std::max(local_class(n / sampled), 1), kmax) : 0;
    t = tic(c);
    if (kspec) HIP_TRY(c, launch_local_sort_e(p, kspec, 0, sampled, true, c->stream));
    else HIP_TRY(c, launch_est_publish(p, c->stream));
    ST_TRY(wait_word(1, p.seq_done, "K12g counters"));
    if (mail[0] != 0) {  // a region overflowed: *ok stays false
        if (c->plan_trace) fprintf(stderr, "gsort plan: overflow %llx\n", (unsigned long long)mail[0]);
        return GSORT_OK;
    }
    uint64_t h[3 * (kLocalClasses + 1)];
    for (int i = 0; i < 3 * (kLocalClasses + 1); ++i) h[i] = mail[8 + i];
    uint64_t keys = 0, ent = 0;  // (list 0: the children past kLocalMax, K18c)
    for (int k = 0; k <= kLocalClasses; ++k) { keys += h[3 * k + 1]; ent += h[3 * k]; }
    if (keys != n || ent > kBuckets16)  // every key in exactly one K11e entry
        return set_err(c, GSORT_EINVAL, "sampled plan: K11e lists hold " + std::to_string(keys) +
                                            " keys in " + std::to_string(ent) + " entries, want " +
                                            std::to_string(n) + " keys");
    for (int k = 1; k <= kmax; ++k) {
        const uint32_t done = k == kspec ? sampled : 0u, cnt = (uint32_t)h[3 * k];
        if (cnt > done) HIP_TRY(c, launch_local_sort_e(p, k, done, cnt - done, false, c->stream));
    }
    if (h[0]) HIP_TRY(c, launch_est_oversized(p, (uint32_t)h[0], c->ncu, c->stream));
    toc(c, PH_BUCKET, t);
    *ok = true;
    if (stats) stats->buckets_local += ent;
    if (*ok && stats) {
        stats->keys_level[0] += n;
        stats->keys_level[1] += n;
        stats->keys_bucket_sort += n;
        stats->passes_run = 2;
    }
    return GSORT_OK;
}

gsort_status msd_sort(gsort_ctx *c, const uint32_t *in, uint64_t n, uint32_t *out,
                      uint32_t *tmp, gsort_stats *stats, bool group16, uint16_t *out16,
                      uint64_t *gb, bool allow_est, bool allow_giant);

// One dominant 16-bit child (gsort_kernels.hip, "giant child"): K1m found child `child` in at
// least half of the samples.  K1g histograms its keys' low 16 bits and compacts the other
// (cold) keys per XCD shard into S_TMP; K12m / K12s turn the partials into output starts; the
// cold keys are gathered, sorted by the regular local sort into out + n_child (below-child keys
// then move to the front) and K18g writes the child's keys from the counts.  *ok = false: the
// child held fewer than half of the keys after all (nothing is written; the caller goes on).
gsort_status giant_sort(gsort_ctx *c, const uint32_t *in, uint64_t n, uint32_t *out,
                        uint32_t child, gsort_stats *stats, bool *ok) {
    *ok = false;
    uint32_t g = 0;
    const uint64_t cap = (uint64_t)giant_wg_cap(n, &g) * g;
    ST_TRY(ensure(c, c->slot[S_TMP], cap * 4));
    ST_TRY(ensure(c, c->m_part, (size_t)kH16Blocks * kH16PartWords * 4));
    constexpr size_t kFixBytes = (size_t)kH16Shards * kBuckets16 * 8;
    ST_TRY(ensure(c, c->m_fix, kFixBytes));
    const uint64_t nchunks_max = n / 2048 + 2;  // K18g chunks of >= 2048 keys
    ST_TRY(ensure(c, c->m_gplan, ((size_t)2 * kBuckets16 + 1 + 64) * 8 + nchunks_max * 4));
    if (c->fix_clean != c->m_fix.p) HIP_TRY(c, hipMemsetAsync(c->m_fix.p, 0, kFixBytes, c->stream));
    c->fix_clean = nullptr;
    // ctr: [0] cold keys below the child, [1 + b] workgroup b's cold keys (1 + g <= 257 u64,
    // inside OFF_GIANT's 4 KiB)
    static_assert(OFF_GIANT + (4 + 1 + kH16Blocks) * 8 <= OFF_PLAN, "giant counters");
    uint64_t *d_ctr = reinterpret_cast<uint64_t *>(c->d_small + OFF_GIANT) + 4;
    uint64_t *h_ctr = reinterpret_cast<uint64_t *>(c->h_small + OFF_GIANT) + 4;
    uint64_t *counts = static_cast<uint64_t *>(c->m_gplan.p), *starts = counts + kBuckets16;
    uint32_t *chunk_bin = reinterpret_cast<uint32_t *>(starts + kBuckets16 + 1 + 64);  // (K12s scratch before it)
    uint32_t *cold = slot_ptr<uint32_t>(c, S_TMP);
    HIP_TRY(c, hipMemsetAsync(d_ctr, 0, (1 + g) * 8, c->stream));
    hipEvent_t t = tic(c);
    HIP_TRY(c, launch_giant_hist(in, n, child, reinterpret_cast<uint32_t *>(c->m_part.p),
                                 reinterpret_cast<uint64_t *>(c->m_fix.p), cold, d_ctr, c->stream));
    HIP_TRY(c, launch_giant_plan(reinterpret_cast<uint32_t *>(c->m_part.p), g,
                                 reinterpret_cast<uint64_t *>(c->m_fix.p), d_ctr, counts, starts,
                                 c->stream));
    c->fix_clean = c->m_fix.p;  // K12m left it zeroed
    toc(c, PH_COUNT, t);
    HIP_TRY(c, hipMemcpyAsync(h_ctr, d_ctr, (1 + g) * 8, hipMemcpyDeviceToHost, c->stream));
    HIP_TRY(c, hipStreamSynchronize(c->stream));
    uint64_t n_cold = 0;
    const uint64_t n_lo = h_ctr[0];
    for (uint32_t b = 0; b < g; ++b) n_cold += h_ctr[1 + b];
    const uint64_t n_child = n - n_cold;
    if (c->plan_trace)
        fprintf(stderr, "gsort plan: giant child %x n %llu cold %llu below %llu\n", child,
                (unsigned long long)n, (unsigned long long)n_cold, (unsigned long long)n_lo);
    if (n_cold > n || n_lo > n_cold)
        return set_err(c, GSORT_EINVAL, "giant child: inconsistent cold counts");
    // the sample misjudged: not worth it.  2 n_child >= n also gives n_cold <= n_child, which
    // the cold-key sort below relies on (odd n with n_child = (n - 1) / 2 would overlap)
    if (2 * n_child < n) return GSORT_OK;
    // the cold keys: gathered from the workgroups' segments into out[0, n_cold), sorted into
    // out[n_child, n) (disjoint: n_cold <= n_child) with S_TMP as scratch, and their part below
    // the child moved to the front (n_lo <= n_cold <= n_child: no overlap either); the child's
    // keys then fill [n_lo, n_lo + n_child)
    if (n_cold) {
        HIP_TRY(c, launch_giant_gather(cold, n, d_ctr, out, c->stream));
        gsort_stats cst;
        memset(&cst, 0, sizeof(cst));
        const int lp = c->last_plan;
        ST_TRY(msd_sort(c, out, n_cold, out + n_child, cold, &cst, false, nullptr, nullptr, true,
                        false));
        c->last_plan = lp;
        if (n_lo)
            HIP_TRY(c, hipMemcpyAsync(out, out + n_child, n_lo * 4, hipMemcpyDeviceToDevice,
                                      c->stream));
        if (stats) stats->keys_bucket_sort += n_cold;
    }
    t = tic(c);
    HIP_TRY(c, launch_giant_expand(starts, n_child, child, chunk_bin, out, c->stream));
    toc(c, PH_BUCKET, t);
    if (stats) {
        stats->passes_run = 1;
        stats->keys_level[0] += n;
        stats->keys_bucket_sort += n_child;
        stats->buckets_local += 1;
    }
    *ok = true;
    return GSORT_OK;
}

// group16: stop after level 2 -- out holds the keys (int32) grouped by their top 16 bits
// (ordered u32) but not sorted inside a group (the sender side of the distributed radix);
// with out16 and n > kLocalMax, level 2 stores only the low 16 bits of every key, at out16.
// With the two-level plan (c->plan16) and group16, gb (65537 u64) receives the 16-bit bucket
// bounds of the grouped block.
// allow_est: the sampled plan may run (it waits on the host for its mailbox words mid-sort, so
// callers that must not block -- the distributed sender's grouping -- keep it off).
// allow_giant: an ineligible block may take the one-dominant-child path (its cold keys are
// sorted with allow_giant off).
gsort_status msd_sort(gsort_ctx *c, const uint32_t *in, uint64_t n, uint32_t *out,
                      uint32_t *tmp, gsort_stats *stats, bool group16,
                      uint16_t *out16, uint64_t *gb, bool allow_est,
                      bool allow_giant) {
    c->last_plan = 0;
    if (n == 0) return GSORT_OK;
    if (allow_est && c->plan_est && c->plan16 && !group16 && n >= kEstMinKeys &&
        n <= kEstMaxKeys) {
        bool ok = false;
        EstRetry r;
        ST_TRY(msd_sort_est(c, in, n, out, stats, &ok, 0, 0, &r));
        c->last_plan = ok ? 1 : 2;
        if (ok) return GSORT_OK;
        // the block's exact min / max (one read pass + a host round trip), once
        bool have_mm = false;
        uint32_t mlo = 0, mhi = 0;
        auto minmax = [&]() -> gsort_status {
            if (have_mm) return GSORT_OK;
            int *d_mm = reinterpret_cast<int *>(c->d_small + OFF_MINMAX);
            int *h_mm = reinterpret_cast<int *>(c->h_small + OFF_MINMAX);
            HIP_TRY(c, hipStreamSynchronize(c->stream));  // h_mm may still feed an earlier copy
            h_mm[0] = 2147483647;
            h_mm[1] = -2147483647 - 1;
            HIP_TRY(c, hipMemcpyAsync(d_mm, h_mm, 8, hipMemcpyHostToDevice, c->stream));
            HIP_TRY(c, launch_minmax(reinterpret_cast<const int32_t *>(in), n, d_mm, c->stream));
            HIP_TRY(c, hipMemcpyAsync(h_mm, d_mm, 8, hipMemcpyDeviceToHost, c->stream));
            HIP_TRY(c, hipStreamSynchronize(c->stream));
            mlo = (uint32_t)h_mm[0] ^ 0x80000000u;
            mhi = (uint32_t)h_mm[1] ^ 0x80000000u;
            have_mm = true;
            return GSORT_OK;
        };
        // one value: the sorted block is the block (copied)
        auto one_value = [&]() -> gsort_status {
            HIP_TRY(c, hipMemcpyAsync(out, in, n * 4, hipMemcpyDeviceToDevice, c->stream));
            ok = true;
            if (stats) {  // one bucket, finished without a partition level
                stats->passes_run = 0;
                stats->buckets_local += 1;
                stats->keys_bucket_sort += n;
            }
            return GSORT_OK;
        };
        // every sample one value: most likely the whole block is (all-equal 2^28 keys: the
        // copy 0.60 ms, the counted child below 1.11 ms)
        if (r.valid && span_lead(r.lo, r.hi) == 32) {
            ST_TRY(minmax());
            if (mlo == mhi) {
                ST_TRY(one_value());
                c->last_plan = 3;
                return GSORT_OK;
            }
        }
        // one 16-bit child holding at least half of the keys (Zipf, 8- / 16-bit keys, one
        // frequent value): counted, not partitioned (K1m decides from 16384 strided samples)
        // (skipped when the first sample's child counts are known -- no u8 counter wrapped --
        // and its largest child holds well under half of the samples: K1m is a 40 us strided
        // read; a dominant child always wraps, >= 512 samples in one workgroup's counter)
        const bool known = r.maxc != 0xffffffffu;
        if (allow_giant && c->plan_giant && r.valid && !(known && (uint64_t)r.maxc * 160 < n)) {
            uint64_t *d_res = reinterpret_cast<uint64_t *>(c->d_small + OFF_GIANT);
            uint64_t *h_res = reinterpret_cast<uint64_t *>(c->h_small + OFF_GIANT);
            HIP_TRY(c, launch_est_mode(in, n, d_res, c->stream));
            HIP_TRY(c, hipMemcpyAsync(h_res, d_res, 24, hipMemcpyDeviceToHost, c->stream));
            HIP_TRY(c, hipStreamSynchronize(c->stream));
            if (c->plan_trace)
                fprintf(stderr, "gsort plan: mode child %llx %llu of %llu samples\n",
                        (unsigned long long)h_res[0], (unsigned long long)h_res[1],
                        (unsigned long long)h_res[2]);
            // (strictly more than half: all a Boyer-Moore vote guarantees to find -- at an
            // exact 50 / 50 split of two children it may end on either or on neither)
            if (h_res[2] && 2 * h_res[1] > h_res[2]) {
                ST_TRY(giant_sort(c, in, n, out, (uint32_t)h_res[0], stats, &ok));
                if (ok) {
                    c->last_plan = 4;
                    return GSORT_OK;
                }
            }
        }
        // An ineligible block whose keys span a narrow range: retry with every digit below the
        // bits the range's keys share (children of at most kLocalMax / 2 on average), either
        // a prefix the samples share (free: K3r checks it on every key) or -- when the range
        // crosses a power of two, e.g. around zero -- the exact min / max (one read pass) as an
        // offset.  One or two shared bits (Zipf, any non-negative keys) rarely make a block
        // eligible and are not worth a second sample.
        // fits: the children after a shift by min(lead, 16) bits average at most kLocalMax / 2,
        // and -- when the first sample's child counts are known (no u8 counter wrapped) -- the
        // largest one now (~64 keys per sample) split 2^shift ways stays below 5/8 of it.  The
        // prefix retry costs a failed sample when wrong; the offset retry also a read pass, so
        // it needs known counts (no u8 counter wrapped) and a fit after the shift, or -- counts
        // wrapped, i.e. a peaked block -- a span of at most 24 bits (>= 8 shared): Gaussian keys
        // (the first sample wraps on their peak; after the offset their children hold <= ~27K
        // keys at 2^28, sigma 1e6) pass it, Zipf keys, whose densest child holds ~29 % of the
        // block, do not.
        auto fits = [&](int lead) {
            const int sb = std::min(lead, 16);
            const int fixed = std::max(0, std::min(lead - sb, 16));  // bits fixed below the shift
            return n / (1ull << (16 - fixed)) <= kLocalMax / 2 &&
                   (!known || ((uint64_t)r.maxc * 64) >> sb <= kLocalMax * 5 / 8);
        };
        if (r.valid) {
            const int lead = r.vary ? __builtin_clz(r.vary) : 32;
            const int slead = span_lead(r.lo, r.hi);
            const bool by_prefix = lead >= 3 && lead < 32 && fits(lead);
            const bool by_offset =
                !by_prefix && (slead == 32 || ((known || slead >= 8) && slead >= 4 && fits(slead - 1)));
            if (by_prefix) {
                ST_TRY(msd_sort_est(c, in, n, out, stats, &ok, std::min(lead, 16)));
            } else if (by_offset) {
                // (the samples' span, one bit of margin: the block's may be wider)
                // First the samples' range widened by an eighth of its width each way as the
                // offset (no read pass: K3r checks every key against the constant prefix, so a
                // key outside the guess fails the attempt); then the exact min / max.
                if (slead < 32) {
                    const uint64_t m = ((uint64_t)r.hi - r.lo) / 8 + 1;
                    const uint32_t glo = r.lo > m ? (uint32_t)(r.lo - m) : 0u;
                    const uint32_t ghi = (uint32_t)std::min<uint64_t>((uint64_t)r.hi + m, 0xffffffffull);
                    const int gl = span_lead(glo, ghi);
                    if (gl >= 3 && fits(gl))
                        ST_TRY(msd_sort_est(c, in, n, out, stats, &ok, std::min(gl, 16), glo));
                    if (c->plan_trace)
                        fprintf(stderr, "gsort plan: offset guess %x..%x lead %d ok %d\n", glo, ghi,
                                gl, (int)ok);
                }
            }
            if (by_offset && !ok) {
                ST_TRY(minmax());
                const uint32_t lo = mlo, hi = mhi;
                const int lead = span_lead(lo, hi);
                if (lead == 32) {
                    ST_TRY(one_value());
                } else if (lead >= 3 && fits(lead)) {
                    ST_TRY(msd_sort_est(c, in, n, out, stats, &ok, std::min(lead, 16), lo));
                }
            }
        }
        if (ok) {
            c->last_plan = 3;
            return GSORT_OK;
        }
    }
    uint64_t *ctr = reinterpret_cast<uint64_t *>(c->d_small + OFF_CTR);
    if (n <= kLocalMax) {  // one bucket: all four digits in LDS
        uint64_t *h_one = reinterpret_cast<uint64_t *>(c->h_small + OFF_ONE);
        uint64_t *d_one = reinterpret_cast<uint64_t *>(c->d_small + OFF_ONE);
        HIP_TRY(c, hipStreamSynchronize(c->stream));  // h_one may feed an earlier copy
        h_one[0] = 0;
        h_one[1] = n;
        HIP_TRY(c, hipMemcpyAsync(d_one, h_one, 16, hipMemcpyHostToDevice, c->stream));
        hipEvent_t t = tic(c);
        HIP_TRY(c, launch_local_sort(in, out, d_one, 1, local_class(n), 4, true, c->atomic_rank,
                                     c->stream));
        toc(c, PH_BUCKET, t);
        if (stats) { stats->buckets_local += 1; stats->keys_bucket_sort += n; }
        return GSORT_OK;
    }
    if (!tmp) {  // the exact plans' ping-pong buffer, allocated only when one of them runs
        ST_TRY(ensure(c, c->slot[S_TMP], n * 4));
        tmp = slot_ptr<uint32_t>(c, S_TMP);
    }
    if (c->plan16 && (!group16 || out16) && n < (1ull << 32)) {
        const int lp = c->last_plan;
        const gsort_status st =
            msd_sort_h16(c, in, n, out, tmp, stats, group16, out16, group16 ? gb : nullptr);
        c->last_plan = lp;
        return st;
    }
    ST_TRY(ensure_pass_scratch(c, n));
    uint64_t *totals = reinterpret_cast<uint64_t *>(c->d_small + OFF_TOT);
    uint64_t *bases = reinterpret_cast<uint64_t *>(c->d_small + OFF_BASES);
    ST_TRY(ensure_list(c, c->m_next[0], kRadix));
    for (auto &b : c->m_local) ST_TRY(ensure_list(c, b, kRadix));
    auto lists = [&](int next) { return work_lists(c, next); };

    // level 3: global tiles
    hipEvent_t t = tic(c);
    HIP_TRY(c, launch_tile_counts1(in, n, 24, true, d_tcounts(c), c->stream));
    HIP_TRY(c, launch_scan_tiles(d_tcounts(c), n, d_gsum(c), totals, bases, c->stream));
    toc(c, PH_COUNT, t);
    t = tic(c);
    HIP_TRY(c, launch_partition(in, tmp, n, 24, d_tcounts(c), d_gsum(c), bases, true, c->stream));
    toc(c, PH_LEVEL3, t);
    if (stats) stats->keys_level[0] += n;
    HIP_TRY(c, hipMemsetAsync(ctr, 0, kCtrBytes, c->stream));
    WorkLists wl3 = lists(0);
    wl3.force_next = group16;  // every level-3 bucket goes through level 2
    HIP_TRY(c, launch_classify_buckets(bases, totals, wl3, c->stream));
    uint64_t h[3 * (kLocalClasses + 1)];  // {entries, keys, longest}: next level, K11 classes
    ST_TRY(read_counters(c, h));
    c->group16_nseg = h[0];
    int levels = 1;
    ST_TRY(msd_levels(c, 2, tmp, out, tmp, 0, h, stats, &levels, group16 ? 2 : 0,
                      group16 ? out16 : nullptr));
    if (stats) stats->passes_run = levels;
    return GSORT_OK;
}

// tmp == nullptr: S_TMP, ensured only if the plan that runs needs a second buffer
gsort_status local_sort(gsort_ctx *c, const uint32_t *in, uint64_t n, uint32_t *out,
                        uint32_t *tmp, int *passes_run, gsort_stats *stats,
                        bool allow_est) {
    if (stats) stats->local_algo = c->local_algo;
    if (c->local_algo == GSORT_LOCAL_LSD) {
        if (!tmp) {
            ST_TRY(ensure(c, c->slot[S_TMP], std::max<uint64_t>(n, 1) * 4));
            tmp = slot_ptr<uint32_t>(c, S_TMP);
        }
        return lsd_sort(c, in, n, out, tmp, passes_run);
    }
    gsort_stats tmp_st;
    memset(&tmp_st, 0, sizeof(tmp_st));
    gsort_stats *st = stats ? stats : &tmp_st;
    const int before = st->passes_run;
    ST_TRY(msd_sort(c, in, n, out, tmp, st, false, nullptr, nullptr, allow_est));
    if (passes_run) *passes_run = st->passes_run;
    if (stats) stats->passes_run = std::max(before, st->passes_run);
    return GSORT_OK;
}

}  // namespace rt
}  // namespace gsort
