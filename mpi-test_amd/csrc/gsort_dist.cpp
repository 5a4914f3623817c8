// gsort_dist.cpp -- the distributed sorts of libgsort: the receive side (P
// sorted runs -> one sorted block), the distributed radix (radix select + one packed exchange;
// the LSD-pass form; the reference-compat order) and the sample sort.
// Reference being replaced: mpi_radix_sort.c:133-195 (per-pass all-to-all through rank 0) and
// mpi_sample_sort.c:89-174 (samples, splitters, buckets, all-to-all, final qsort).
#include "gsort_ctx.h"

namespace gsort {
namespace rt {

// ---- receive side: P sorted runs (after an exchange) -> one sorted block ---------------------
// Replaces the re-sort of the received keys (the reference's final qsort, mpi_sample_sort.c:174;
// for the radix path the last pass's placement, mpi_radix_sort.c:185-192).  The runs are
// bucketed by their top 16 bits with binary searches (no pass over the keys), and K11g sorts
// every bucket's low 16 bits straight from the P pieces: one read + one write per key.  Buckets
// larger than kLocalMax are gathered into place and finish through the MSD levels 1 and 0.
// recv holds the P runs back to back (run p has rlen[p] keys), each grouped by the top 16 bits
// (ordered u32): int32 keys, or with packed16 only their low 16 bits, in which case the caller
// has already filled c->m_rpos (pos[p][h], launch_pos_from_meta).
// bucket sizes (65536) + starts (65537) + row-scan partials / K15s status words (65 x 64), u64,
// + K15s's ticket (one u64 slot)
constexpr size_t kBsizeBytes = ((size_t)2 * kBuckets16 + 1 + kRecvScanStatusWords + 1) * 8;

// (a - b) / sizeof(T) for pointers into different allocations, as a u64 (two's complement for
// a negative offset): integer arithmetic, never a pointer difference across allocations
template <typename T>
uint64_t elem_offset(const T *a, const T *b) {
    const int64_t d = (int64_t)(reinterpret_cast<uintptr_t>(a) - reinterpret_cast<uintptr_t>(b));
    return (uint64_t)(d / (int64_t)sizeof(T));
}

// K18c's lists: the K11 classes >= recv_cx, and list 0 (with list0)
bool cx_class(const gsort_ctx *c, int k) { return c->recv_cx > 0 && k >= c->recv_cx; }

// K18c over cl: with u8 bins (recv_cb 8) the wrapped buckets collect in m_fb (count at
// OFF_FBCTR, at most cl.bound() of them) and one u16 launch right behind redoes them, reading
// their count on the device (usually none: its workgroups return at once).
gsort_status count_expand_lists(gsort_ctx *c, const void *recv, bool packed16, const uint64_t *pos,
                                const uint64_t *roff, int P, const uint64_t *bstart,
                                const CxLists &cl, uint32_t *out) {
    const uint32_t bound = cl.bound();
    if (!bound) return GSORT_OK;
    if (c->recv_cb != 8) {
        HIP_TRY(c, launch_count_expand_lists(recv, packed16, pos, roff, P, bstart, cl, c->ncu,
                                             out, c->stream));
        return GSORT_OK;
    }
    uint32_t *fb_ctr = reinterpret_cast<uint32_t *>(c->d_small + OFF_FBCTR);
    // (room for every bucket: with device-read list lengths the bound is only the grid's guess)
    ST_TRY(ensure_list(c, c->m_fb, kBuckets16));
    uint64_t *fb = reinterpret_cast<uint64_t *>(c->m_fb.p);
    HIP_TRY(c, hipMemsetAsync(fb_ctr, 0, 4, c->stream));
    HIP_TRY(c, launch_count_expand_lists(recv, packed16, pos, roff, P, bstart, cl, c->ncu, out,
                                         c->stream, fb, fb_ctr));
    HIP_TRY(c, launch_count_expand(recv, packed16, pos, roff, P, bstart, fb, bound, c->ncu, out,
                                   c->stream, nullptr, nullptr, fb_ctr));
    return GSORT_OK;
}

// self (int32 runs only): run `self_rank` was not received -- it lies at self_src (the
// sender's sorted block), and the kernels read it there through a run offset taken relative to
// recv (mod 2^64); the MSD fallback, which needs the runs back to back, copies it in first.
// Every receive bucket of the lists wl (counts h, read_counters layout) sorted from its P
// pieces into out: K11g by size class, K18c (or, GSORT_RECV_CX=-1, the two-read K18) past
// kLocalMax; classes >= c->recv_cx go to K18c as well.  With list0, list 0 is sorted too (it
// must then hold no bucket past kHxMax).
// What spec_recv_launch queued before the list counts were known: per K11g class the entries
// [0, k11g[k]) (device-bounded), and the lists (index = class, 0 = list 0) one K18c launch took
// whole with device-read lengths.
struct RecvSpec {
    uint32_t k11g[kLocalClasses + 1] = {};
    bool cx[kLocalClasses + 1] = {};
};

gsort_status sort_recv_lists(gsort_ctx *c, const void *recv, bool packed16, const uint64_t *pos,
                             const uint64_t *roff, int P, const uint64_t *bstart,
                             const WorkLists &wl, const uint64_t *h, uint32_t *out,
                             gsort_stats *stats, bool list0 = true, const RecvSpec *sp = nullptr) {
    CxLists cl;  // every K18c list in ONE persistent launch (a tail per launch otherwise)
    for (int k = 1; k <= kLocalClasses; ++k) {
        const uint64_t *hk = h + 3 * k;
        if (!hk[0]) continue;
        if (stats) { stats->buckets_local += hk[0]; stats->keys_bucket_sort += hk[1]; }
        if (cx_class(c, k)) {
            if (!(sp && sp->cx[k])) cl.add(wl.list[k], (uint32_t)hk[0]);
        } else {
            const uint32_t first = sp ? std::min<uint32_t>(sp->k11g[k], (uint32_t)hk[0]) : 0u;
            if ((uint32_t)hk[0] > first)
                HIP_TRY(c, launch_gather_sort(recv, packed16, pos, roff, P, bstart, wl.list[k],
                                              (uint32_t)hk[0] - first, k, c->atomic_rank, out,
                                              c->stream, nullptr, first));
        }
    }
    if (h[0] && list0) {
        if (stats) { stats->buckets_local += h[0]; stats->keys_bucket_sort += h[1]; }
        if (c->recv_cx > 0) {
            if (!(sp && sp->cx[0])) cl.add(wl.list[0], (uint32_t)h[0]);
        } else {
            HIP_TRY(c, launch_hist_expand(recv, packed16, pos, roff, P, bstart, wl.list[0],
                                          (uint32_t)h[0], out, c->stream));
        }
    }
    return count_expand_lists(c, recv, packed16, pos, roff, P, bstart, cl, out);
}

// The receive sort's launches queued BEFORE the host has read the list counts (VERDICT r5 item
// 3: no host wait between the exchange and the first receive kernel), shaped by the previous
// call's counts (c->recv_hint; none on a context's first call): a K11g grid of that many
// entries per class, each block reading the list's true length on the device and returning
// past it, and one persistent K18c walking its lists to their device-read lengths (list 0
// skipped on the device if it holds a bucket past kHxMax: the caller then re-sorts the block
// through recv_sort).  Whatever the guess missed -- K11g entries past it, a list it did not
// expect -- sort_recv_lists launches once the counts are in.  The guess shapes launches only:
// every bucket is sorted exactly once either way.
gsort_status spec_recv_launch(gsort_ctx *c, const void *recv, bool packed16, const uint64_t *pos,
                              const uint64_t *roff, int P, const uint64_t *bstart,
                              const WorkLists &wl, uint32_t *out, RecvSpec *sp) {
    if (!c->recv_hint_ok || c->recv_cx <= 0) return GSORT_OK;
    const uint64_t *ctr = reinterpret_cast<const uint64_t *>(c->d_small + OFF_CTR);
    auto nd = [&](int k) { return reinterpret_cast<const uint32_t *>(ctr + 3 * k); };  // (low word)
    CxLists cl;
    for (int k = 1; k <= kLocalClasses; ++k) {
        const uint32_t hint = c->recv_hint[k];
        if (!hint) continue;
        if (cx_class(c, k)) {
            cl.add(wl.list[k], hint, nd(k));
            sp->cx[k] = true;
        } else {
            HIP_TRY(c, launch_gather_sort(recv, packed16, pos, roff, P, bstart, wl.list[k], hint, k,
                                          c->atomic_rank, out, c->stream, nd(k), 0));
            sp->k11g[k] = hint;
        }
    }
    if (c->recv_hint[0]) {
        cl.add(wl.list[0], c->recv_hint[0], nd(0));
        cl.skip = cl.nl - 1;
        cl.skip_max = ctr + 2;  // list 0's longest bucket
        sp->cx[0] = true;
    }
    return count_expand_lists(c, recv, packed16, pos, roff, P, bstart, cl, out);
}

gsort_status recv_sort(gsort_ctx *c, const void *recv, bool packed16,
                       const std::vector<uint64_t> &rlen, uint64_t n, uint32_t *out,
                       uint32_t *tmp, gsort_stats *stats, int self_rank = -1,
                       const int32_t *self_src = nullptr) {
    const int P = (int)rlen.size();
    if (n == 0) return GSORT_OK;
    if (!packed16 && (P > 64 || c->local_algo == GSORT_LOCAL_LSD)) {  // K11g: <= 64 pieces
        if (self_src && rlen[self_rank]) {
            uint64_t o = 0;
            for (int p = 0; p < self_rank; ++p) o += rlen[p];
            HIP_TRY(c, hipMemcpyAsync(static_cast<int32_t *>(const_cast<void *>(recv)) + o,
                                      self_src, rlen[self_rank] * 4, hipMemcpyDeviceToDevice,
                                      c->stream));
        }
        int pr = 0;
        return local_sort(c, reinterpret_cast<const uint32_t *>(recv), n, out, tmp, &pr, stats);
    }
    if (P > 64) return set_err(c, GSORT_EINVAL, "packed exchange supports at most 64 ranks");
    hipEvent_t t = tic(c);
    ST_TRY(ensure(c, c->m_rpos, (size_t)P * (kBuckets16 + 1) * 8));
    ST_TRY(ensure(c, c->m_bsize, kBsizeBytes));
    ST_TRY(ensure_list(c, c->m_next[0], kBuckets16));
    for (auto &b : c->m_local) ST_TRY(ensure_list(c, b, kBuckets16));
    uint64_t *h_r = reinterpret_cast<uint64_t *>(c->h_small + OFF_PLAN);
    uint64_t *d_r = reinterpret_cast<uint64_t *>(c->d_small + OFF_PLAN);
    HIP_TRY(c, hipStreamSynchronize(c->stream));  // h_r may still feed an earlier copy
    uint64_t off = 0;
    for (int p = 0; p < P; ++p) { h_r[p] = off; h_r[P + p] = rlen[p]; off += rlen[p]; }
    if (self_src)
        h_r[self_rank] = elem_offset(self_src, static_cast<const int32_t *>(recv));
    HIP_TRY(c, hipMemcpyAsync(d_r, h_r, (size_t)2 * P * 8, hipMemcpyHostToDevice, c->stream));
    uint64_t *pos = reinterpret_cast<uint64_t *>(c->m_rpos.p);
    uint64_t *bsize = reinterpret_cast<uint64_t *>(c->m_bsize.p), *bstart = bsize + kBuckets16;
    uint64_t *ctr = reinterpret_cast<uint64_t *>(c->d_small + OFF_CTR);
    HIP_TRY(c, hipMemsetAsync(ctr, 0, kCtrBytes, c->stream));
    if (!packed16)
        HIP_TRY(c, launch_run_bounds(reinterpret_cast<const int32_t *>(recv), d_r, d_r + P, P, pos,
                                     c->stream));
    HIP_TRY(c, launch_recv_classify(pos, P, bsize, bstart, work_lists(c, 0),
                                    bstart + kBuckets16 + 1, c->stream));
    toc(c, PH_COUNT, t);
    uint64_t h[3 * (kLocalClasses + 1)];
    ST_TRY(read_counters(c, h));
    if (check_mode()) {
        uint64_t keys = h[1];
        for (int k = 0; k < kLocalClasses; ++k) keys += h[3 * (k + 1) + 1];
        if (keys != n)
            return set_err(c, GSORT_EINVAL, "GSORT_CHECK receive lists hold " +
                                                std::to_string(keys) + " keys, want " +
                                                std::to_string(n) + " (rank " +
                                                std::to_string(c->rank) + ")");
        ST_TRY(check_bounds(c, bstart, kBuckets16 + 1, n, "receive bucket starts"));
    }
    const bool list0 = h[0] && h[2] <= kHxMax;  // else: a bucket past kHxMax (below)
    // buckets past kHxMax (skewed keys: a Zipf block's frequent values) are counted in place
    // (round 6): K18c takes list 0 and leaves them empty, then each is gathered as int32 into its
    // place and sorted there by giant_sort -- all its keys share the bucket's top 16 bits, so
    // that is one 65 536-bin count and an expansion (8 B/key), no cold keys.  Without K18c
    // (GSORT_RECV_CX <= 0) or GSORT_GIANT=0, list 0 goes through the MSD levels 1 and 0.
    const bool counted = h[0] && !list0 && c->recv_cx > 0 && c->plan_giant;
    t = tic(c);
    ST_TRY(sort_recv_lists(c, recv, packed16, pos, d_r, P, bstart, work_lists(c, 0), h, out, stats,
                           list0 || counted));
    toc(c, PH_BUCKET, t);
    if (counted) {
        t = tic(c);
        HIP_TRY(c, launch_gather_copy(recv, packed16, pos, d_r, P, bstart, n, out, c->stream, kHxMax,
                                      true));
        std::vector<uint64_t> l0(2 * h[0]);
        HIP_TRY(c, hipMemcpyAsync(l0.data(), c->m_next[0].p, l0.size() * 8, hipMemcpyDeviceToHost,
                                  c->stream));
        HIP_TRY(c, hipStreamSynchronize(c->stream));
        for (uint64_t e = 0; e < h[0]; ++e) {
            const uint64_t len = (uint32_t)l0[2 * e + 1];
            if (len <= kHxMax) continue;
            uint32_t *b = out + (l0[2 * e] >> 16);  // (entry: h | bstart[h] << 16)
            bool ok = false;
            ST_TRY(giant_sort(c, b, len, b, (uint32_t)(l0[2 * e] & 0xFFFFu), nullptr, &ok));
            if (!ok) return set_err(c, GSORT_EINVAL, "receive bucket past kHxMax: counted sort refused");
        }
        toc(c, PH_BUCKET, t);
    } else if (h[0] && !list0) {  // all of list 0 into place, then MSD levels 1 and 0
        HIP_TRY(c, launch_list_to_segments(reinterpret_cast<uint64_t *>(c->m_next[0].p),
                                           (uint32_t)h[0], bstart, c->stream));
        HIP_TRY(c, launch_gather_copy(recv, packed16, pos, d_r, P, bstart, n, out, c->stream));
        for (int k = 3; k < 3 * (kLocalClasses + 1); ++k) h[k] = 0;
        int levels = 0;
        ST_TRY(msd_levels(c, 1, out, out, tmp, 0, h, stats, &levels));
    }
    return GSORT_OK;
}

// Allgather one u64 per rank into host memory (counts used to size RCCL messages).
gsort_status allgather_u64(gsort_ctx *c, uint64_t v, std::vector<uint64_t> &out) {
    out.assign(c->nranks, 0);
    if (c->nranks == 1) { out[0] = v; return GSORT_OK; }
    uint64_t *h = reinterpret_cast<uint64_t *>(c->h_small + OFF_PLAN);
    uint64_t *d = reinterpret_cast<uint64_t *>(c->d_small + OFF_PLAN);
    h[0] = v;
    HIP_TRY(c, hipMemcpyAsync(d, h, 8, hipMemcpyHostToDevice, c->stream));
    ST_TRY(comm_try(c, c->comm->allgather(d, d + 1, 8, c->stream)));
    HIP_TRY(c, hipMemcpyAsync(h + 1, d + 1, 8 * c->nranks, hipMemcpyDeviceToHost, c->stream));
    HIP_TRY(c, hipStreamSynchronize(c->stream));
    for (int r = 0; r < c->nranks; ++r) out[r] = h[1 + r];
    return GSORT_OK;
}

void block_of(uint64_t N, int P, int r, uint64_t *B, uint64_t *len) {
    *B = P ? (N + P - 1) / P : 0;
    const uint64_t lo = (uint64_t)r * *B;
    *len = lo >= N ? 0 : std::min(*B, N - lo);
}

// Sort the listed groups {start, len} of an int32 block in place on their low 16 bits (their
// top 16 bits are equal, ids[i] = group i's as ordered u32 >> 16 when given): K11 for groups of
// <= kLocalMax keys; past that the counted-child sort (giant_sort: one 65 536-bin histogram of
// the low halves and an expansion, 8 B/key -- round 6: a Zipf block's giant group took two LSD
// passes, ~30 B/key, 93 ms of every rank's 135 ms step at P = 8, profiles/r06_zipf_p8.txt), or
// the LSD passes without ids or with GSORT_GIANT=0.
gsort_status sort_groups(gsort_ctx *c, int32_t *a,
                         const std::vector<std::pair<uint64_t, uint64_t>> &groups,
                         const std::vector<uint32_t> *ids = nullptr) {
    std::vector<uint64_t> small[kLocalClasses];
    for (size_t gi = 0; gi < groups.size(); ++gi) {
        const auto &gr = groups[gi];
        const int k = local_class(gr.second);
        if (k) {
            small[k - 1].push_back(gr.first);
            small[k - 1].push_back(gr.second);
            continue;
        }
        ST_TRY(ensure(c, c->m_bseg, gr.second * 8));
        uint32_t *t0 = reinterpret_cast<uint32_t *>(c->m_bseg.p), *t1 = t0 + gr.second;
        bool counted = false;
        if (ids && c->plan_giant) {  // every key in the one child: counted, never "misjudged"
            const int lp = c->last_plan;
            ST_TRY(giant_sort(c, reinterpret_cast<const uint32_t *>(a + gr.first), gr.second, t0,
                              (*ids)[gi], nullptr, &counted));
            c->last_plan = lp;
        }
        int pr = 0;  // lsd_sort leaves its result in its `out` (t0)
        if (!counted)
            ST_TRY(lsd_sort(c, reinterpret_cast<const uint32_t *>(a + gr.first), gr.second, t0, t1,
                            &pr));
        HIP_TRY(c, hipMemcpyAsync(a + gr.first, t0, gr.second * 4, hipMemcpyDeviceToDevice,
                                  c->stream));
    }
    for (int k = 0; k < kLocalClasses; ++k) {
        if (small[k].empty()) continue;
        ST_TRY(ensure(c, c->m_blist, small[k].size() * 8));
        HIP_TRY(c, hipMemcpyAsync(c->m_blist.p, small[k].data(), small[k].size() * 8,
                                  hipMemcpyHostToDevice, c->stream));
        uint32_t *ab = reinterpret_cast<uint32_t *>(a);
        HIP_TRY(c, launch_local_sort(ab, ab, reinterpret_cast<uint64_t *>(c->m_blist.p),
                                     (uint32_t)(small[k].size() / 2), k + 1, 2, true,
                                     c->atomic_rank, c->stream));
        HIP_TRY(c, hipStreamSynchronize(c->stream));  // small[k] is host memory
    }
    return GSORT_OK;
}

// The same on the packed send buffer: groups = {16-bit bucket h, first position}, ends[i] =
// the group's end (gb[h + 1]).  Each group is rebuilt as int32 keys in scratch, sorted by
// sort_groups (K11 or LSD passes by size), and packed back in place.
gsort_status sort_groups16(gsort_ctx *c, uint16_t *pack,
                           const std::vector<std::pair<uint64_t, uint64_t>> &groups,
                           const std::vector<uint64_t> &ends) {
    uint64_t total = 0;
    for (size_t i = 0; i < groups.size(); ++i) total += ends[i] - groups[i].second;
    ST_TRY(ensure(c, c->m_g16, std::max<uint64_t>(total, 1) * 4));
    int32_t *scr = reinterpret_cast<int32_t *>(c->m_g16.p);
    std::vector<std::pair<uint64_t, uint64_t>> local;
    std::vector<uint32_t> ids;
    uint64_t off = 0;
    for (size_t i = 0; i < groups.size(); ++i) {
        const uint64_t a = groups[i].second, len = ends[i] - a;
        HIP_TRY(c, launch_unpack16(pack + a, len, (uint32_t)groups[i].first, scr + off,
                                   c->stream));
        local.push_back({off, len});
        ids.push_back((uint32_t)groups[i].first);
        off += len;
    }
    ST_TRY(sort_groups(c, scr, local, &ids));
    for (size_t i = 0; i < groups.size(); ++i)
        HIP_TRY(c, launch_pack16(scr + local[i].first, local[i].second, pack + groups[i].second,
                                 c->stream));
    return GSORT_OK;
}

// The listed 16-bit groups of the packed block (ids < 65536, any order, duplicates allowed)
// sorted in place through sort_groups16 -- the host path for groups past K13g's 32 768 keys
// (their bounds read from gb: one host round trip).
gsort_status sort_groups16_host(gsort_ctx *c, uint16_t *pack, const uint64_t *gb,
                                std::vector<uint64_t> hs) {
    std::sort(hs.begin(), hs.end());
    hs.erase(std::unique(hs.begin(), hs.end()), hs.end());
    if (hs.empty()) return GSORT_OK;
    std::vector<uint64_t> h_gb(2 * hs.size());
    for (size_t i = 0; i < hs.size(); ++i)
        HIP_TRY(c, hipMemcpyAsync(&h_gb[2 * i], gb + hs[i], 16, hipMemcpyDeviceToHost, c->stream));
    HIP_TRY(c, hipStreamSynchronize(c->stream));
    std::vector<std::pair<uint64_t, uint64_t>> nonempty;  // {h, first position}
    std::vector<uint64_t> ends;
    for (size_t i = 0; i < hs.size(); ++i)
        if (h_gb[2 * i + 1] > h_gb[2 * i]) {
            nonempty.push_back({hs[i], h_gb[2 * i]});
            ends.push_back(h_gb[2 * i + 1]);
        }
    if (!nonempty.empty()) ST_TRY(sort_groups16(c, pack, nonempty, ends));
    return GSORT_OK;
}


// ---- the packed distributed sorts (P ranks, one exchange of 2 B per key) ----------------------
// Both distributed sorts share one sender and one receiver; they differ only in how the block
// boundaries are found:
//   radix  (mpi_radix_sort.c:133-195): rank q ends with global positions [qB, (q+1)B) -- the
//          boundary keys by an exact radix select;
//   sample (mpi_sample_sort.c:85-174): rank q ends with the keys in (s_{q-1}, s_q] of the
//          reference's splitters -- regular samples, splitters on the root, bucket bounds.
// (1) group_block16: the block grouped by its top 16 bits (MSD levels 3 and 2 only: every
//     receiver sorts the low 16 bits anyway), the low 16 bits of every key stored as the packed
//     send buffer, the 65 537 group bounds from the plan;
// (2) the boundaries (select_radix / select_sample): small device kernels + collectives on the
//     grouped block; only the groups holding a boundary (and, for the sample sort, a regular
//     sample) are sorted, in place, by K13g -- never the whole block;
// (3) the cut of every rank's block into P contiguous runs (host, from the gathered counts);
// (4) packed_exchange_sort: one u32 count per (destination, 16-bit bucket) and the packed keys
//     in two grouped send/recv rounds, then every received bucket sorted from its P pieces.

// The block of n_in keys grouped by its top 16 bits (ordered u32): *pack (n_in u16, m_pack) =
// the low 16 bits, grouped; *gb (65 537 u64, m_gb) = the group bounds.  A block of <= kLocalMax
// keys is sorted whole in LDS instead, then bounded and packed.
gsort_status group_block16(gsort_ctx *c, const int32_t *d_keys, uint64_t n_in,
                           gsort_stats *stats, uint16_t **pack_out, uint64_t **gb_out) {
    ST_TRY(ensure(c, c->slot[S_TMP], std::max<uint64_t>(n_in, 1) * 4));
    ST_TRY(ensure(c, c->m_gb, (size_t)(kBuckets16 + 1) * 8));
    ST_TRY(ensure(c, c->m_pack, std::max<uint64_t>(n_in, 1) * 2));
    uint64_t *gb = reinterpret_cast<uint64_t *>(c->m_gb.p);
    uint16_t *pack = reinterpret_cast<uint16_t *>(c->m_pack.p);
    if (stats) stats->local_algo = c->local_algo;
    const bool packed_msd = n_in > kLocalMax;
    gsort_stats tmp_st;
    memset(&tmp_st, 0, sizeof(tmp_st));
    int32_t *sorted = nullptr;
    if (!packed_msd) {
        ST_TRY(ensure(c, c->slot[S_SORTED], std::max<uint64_t>(n_in, 1) * 4));
        sorted = slot_ptr<int32_t>(c, S_SORTED);
    }
    ST_TRY(msd_sort(c, reinterpret_cast<const uint32_t *>(d_keys), n_in,
                    reinterpret_cast<uint32_t *>(sorted), slot_ptr<uint32_t>(c, S_TMP),
                    stats ? stats : &tmp_st, true, packed_msd ? pack : nullptr, gb));
    hipEvent_t t = tic(c);
    if (packed_msd && c->plan16) {
        // gb written by the two-level plan
    } else if (packed_msd) {
        HIP_TRY(c, launch_gb_from_plan(reinterpret_cast<uint64_t *>(c->d_small + OFF_BASES),
                                       reinterpret_cast<uint64_t *>(c->d_small + OFF_TOT),
                                       reinterpret_cast<uint64_t *>(c->m_next[0].p),
                                       (uint32_t)c->group16_nseg,
                                       reinterpret_cast<uint64_t *>(c->m_cstart.p), n_in, gb,
                                       c->stream));
    } else {
        uint64_t *h_one = reinterpret_cast<uint64_t *>(c->h_small + OFF_ONE);
        uint64_t *d_one = reinterpret_cast<uint64_t *>(c->d_small + OFF_ONE);
        HIP_TRY(c, hipStreamSynchronize(c->stream));  // h_one may feed an earlier copy
        h_one[0] = 0;
        h_one[1] = n_in;
        HIP_TRY(c, hipMemcpyAsync(d_one, h_one, 16, hipMemcpyHostToDevice, c->stream));
        HIP_TRY(c, launch_run_bounds(sorted, d_one, d_one + 1, 1, gb, c->stream));
        HIP_TRY(c, launch_pack16(sorted, n_in, pack, c->stream));
    }
    toc(c, PH_PLACE, t);
    if (check_mode()) ST_TRY(check_bounds(c, gb, kBuckets16 + 1, n_in, "sender bucket bounds"));
    *pack_out = pack;
    *gb_out = gb;
    return GSORT_OK;
}

// Every rank's block size must stay within what the transport can carry in one alltoallv
// (the IPC group's staging limit), bytes_per_key of it: checked on all ranks from the gathered
// sizes, so all of them fail alike before any key moves.
gsort_status check_send_limit(gsort_ctx *c, const std::vector<uint64_t> &n_all,
                              uint64_t bytes_per_key, const char *what) {
    const uint64_t lim = c->comm ? c->comm->max_send_bytes() : ~0ull;
    for (size_t r = 0; r < n_all.size(); ++r)
        if (n_all[r] > lim / bytes_per_key)
            return set_err(c, GSORT_EINVAL, std::string(what) + ": rank " + std::to_string(r) +
                                                " would send up to " +
                                                std::to_string(n_all[r] * bytes_per_key) +
                                                " bytes, over the transport's " +
                                                std::to_string(lim) + "-byte limit");
    return GSORT_OK;
}

// (4)-(6): the packed exchange and the receive sort.  cut (P + 1): this rank's runs, run q =
// [cut[q], cut[q+1]) of the grouped block goes to rank q; recv[p] = the keys rank p sends here;
// destination q's keys lie in the 16-bit buckets [hlo[q], hlo[q] + nh[q]) (every rank computes
// the same hlo / nh).  The sorted result (sum of recv keys) is left in S_OUT.
gsort_status packed_exchange_sort(gsort_ctx *c, uint16_t *pack, const uint64_t *gb,
                                  const std::vector<uint64_t> &cut,
                                  const std::vector<uint64_t> &recv,
                                  const std::vector<uint64_t> &hlo,
                                  const std::vector<uint64_t> &nh, gsort_stats *stats,
                                  int32_t **d_out, uint64_t *n_out) {
    const int P = c->nranks, me = c->rank;
    std::vector<uint64_t> send(P);
    for (int q = 0; q < P; ++q) send[q] = cut[q + 1] - cut[q];
    uint64_t mine = 0;
    for (int p = 0; p < P; ++p) mine += recv[p];
    ST_TRY(ensure(c, c->slot[S_RECV], std::max<uint64_t>(mine, 1) * 2));
    ST_TRY(ensure(c, c->slot[S_OUT], std::max<uint64_t>(mine, 1) * 4));
    // test hook GSORT_RCCL_SELF=1: the self pieces do go through the transport (RcclComm then
    // sends them through ncclSend / ncclRecv: tests/test_gpu_rccl.py pins RCCL's message limit)
    static const bool self_moved = getenv("GSORT_RCCL_SELF") && getenv("GSORT_RCCL_SELF")[0] == '1';
    uint64_t meta_n = 0, meta_self = ~0ull;  // meta_self: this rank's own count section
    std::vector<uint64_t> rng;
    for (int q = 0; q < P; ++q)
        if (send[q]) {
            rng.insert(rng.end(), {cut[q], cut[q + 1], hlo[q], nh[q], meta_n});
            if (q == me) meta_self = meta_n;
            meta_n += nh[q];
        }
    uint64_t nsrc = 0;
    for (int p = 0; p < P; ++p) nsrc += recv[p] ? 1 : 0;
    // the receive plan's buffers first (host-side allocations, none once warm)
    ST_TRY(ensure(c, c->m_rpos, (size_t)P * (kBuckets16 + 1) * 8));
    ST_TRY(ensure(c, c->m_bsize, kBsizeBytes));
    ST_TRY(ensure_list(c, c->m_next[0], kBuckets16));
    for (auto &b : c->m_local) ST_TRY(ensure_list(c, b, kBuckets16));
    ST_TRY(ensure(c, c->m_meta, (std::max<uint64_t>(meta_n, 1) + nsrc * nh[me] + 1) * 4 +
                                    (rng.size() + 3 * P + 2) * 8));
    uint32_t *meta_s = reinterpret_cast<uint32_t *>(c->m_meta.p);
    // (one word of gap: an in-place self offset below, meta_self - (meta_r - meta_s), is then
    // at most -2 and never the "no source" mark ~0)
    uint32_t *meta_r = meta_s + std::max<uint64_t>(meta_n, 1) + 1;
    // table (device, one H2D copy): the K15 ranges (5 per destination) | moff (P) | the receive
    // runs' offsets roff (P) and lengths (P)
    uint64_t *d_tab = reinterpret_cast<uint64_t *>(
        reinterpret_cast<char *>(c->m_meta.p) +
        (((std::max<uint64_t>(meta_n, 1) + nsrc * nh[me] + 1) * 4 + 7) & ~size_t(7)));
    std::vector<uint64_t> tab(rng);
    std::vector<uint64_t> moff(P, ~0ull);
    {
        uint64_t k = 0;
        for (int p = 0; p < P; ++p)
            if (recv[p]) moff[p] = (k++) * nh[me];
    }
    // the rank's own counts are read where K15 writes them (an offset relative to meta_r, mod
    // 2^64), like its own keys below: no self copy in the count exchange either
    const bool meta_in_place = !self_moved && recv[me] && meta_self != ~0ull;
    if (meta_in_place) moff[me] = meta_self - (uint64_t)(meta_r - meta_s);
    tab.insert(tab.end(), moff.begin(), moff.end());
    std::vector<uint64_t> roffs(P + 1, 0);
    for (int p = 0; p < P; ++p) roffs[p + 1] = roffs[p] + recv[p];
    uint16_t *rbuf = slot_ptr<uint16_t>(c, S_RECV);
    const size_t r0 = tab.size();
    for (int p = 0; p < P; ++p) tab.push_back(roffs[p]);
    for (int p = 0; p < P; ++p) tab.push_back(recv[p]);
    // the self piece is read in place: its offset from rbuf in keys, from integer addresses
    // (mod 2^64, run_ptr)
    if (!self_moved) tab[r0 + me] = elem_offset(pack + cut[me], rbuf);
    // staged through pinned memory (a pageable copy blocks the host in the runtime's staging):
    // OFF_PLAN + 8 KiB is free here -- the select's host reads synchronised the stream, and
    // nothing else stages there
    uint64_t *h_tab = reinterpret_cast<uint64_t *>(c->h_small + OFF_PLAN + 8192);
    if (OFF_PLAN + 8192 + tab.size() * 8 > kSmallBytes)
        return set_err(c, GSORT_EINVAL, "exchange table too large");
    std::copy(tab.begin(), tab.end(), h_tab);
    HIP_TRY(c, hipMemcpyAsync(d_tab, h_tab, tab.size() * 8, hipMemcpyHostToDevice, c->stream));
    const uint64_t *d_rng = d_tab, *d_moff = d_tab + rng.size();
    const uint64_t *d_r = d_tab + r0;  // roff (P) | rlen (P)
    hipEvent_t t = tic(c);
    HIP_TRY(c, launch_meta_counts(gb, d_rng, (int)(rng.size() / 5), meta_s, c->stream));
    toc(c, PH_PLACE, t);
    std::vector<size_t> sc(P, 0), sd(P, 0), rc(P, 0), rd(P, 0);
    {
        uint64_t mo = 0, ro = 0;
        for (int q = 0; q < P; ++q) {
            if (send[q]) { sc[q] = nh[q] * 4; sd[q] = mo * 4; mo += nh[q]; }
            if (recv[q]) { rc[q] = nh[me] * 4; rd[q] = ro * 4; ro += nh[me]; }
        }
        if (meta_in_place) sc[me] = rc[me] = 0;
    }
    t = tic_rec(c);
    ST_TRY(comm_try(c, c->comm->alltoallv(meta_s, sc.data(), sd.data(), meta_r, rc.data(),
                                          rd.data(), c->stream)));
    toc_rec(c, PH_EXCH, t);
    // (no payload from or to a peer -- one rank -- leaves nothing to overlap: the plan then
    // stays on the main stream, where the cross-stream hand-off cost ~13 us of idle, and even
    // the event record alone ~5 us)
    bool peers = false;
    for (int q = 0; q < P; ++q) peers |= q != me && (send[q] || recv[q]);
    if (peers) HIP_TRY(c, hipEventRecord(c->ev_meta, c->stream));
    for (int q = 0; q < P; ++q)
        if (stats && q != me) {
            stats->bytes_sent += send[q] * 2;
            stats->max_pair_bytes = std::max<uint64_t>(stats->max_pair_bytes, send[q] * 2);
        }
    // the payload, queued right behind the counts.  The rank's own piece is not moved at all:
    // the receive kernels read it where it lies in the send buffer (its run offset above is
    // taken relative to rbuf, mod 2^64) -- at P = 1 that is the whole 512 MiB of a 2^28-key
    // block, at P = 8 an eighth of it
    t = tic_rec(c);
    for (int q = 0; q < P; ++q) {
        const bool self = q == me && !self_moved;
        sc[q] = self ? 0 : send[q] * 2;
        sd[q] = cut[q] * 2;
        rc[q] = self ? 0 : recv[q] * 2;
        rd[q] = roffs[q] * 2;
    }
    ST_TRY(comm_try(c, c->comm->alltoallv(pack, sc.data(), sd.data(), rbuf, rc.data(), rd.data(),
                                          c->stream)));
    toc_rec(c, PH_EXCH, t);
    if (stats) stats->exchanges = 1;
    // (5) the receive plan from the counts alone -- run bounds, bucket starts, the K11g / K18c
    // work lists of this rank's bucket range -- on the side stream behind the count exchange,
    // while the payload is in flight on the main one (round 6: on one stream it queued behind
    // the payload, and the host's read of the list counts then idled the GPU before the first
    // receive kernel).  The first kernel clears the list counters, the classification hands
    // them to the host through the pinned mailbox (K12p: no copy, no stream synchronisation),
    // and the main stream waits for the plan before the receive sort.
    uint64_t *pos = reinterpret_cast<uint64_t *>(c->m_rpos.p);
    uint64_t *bsize = reinterpret_cast<uint64_t *>(c->m_bsize.p), *bstart = bsize + kBuckets16;
    uint64_t *ctr = reinterpret_cast<uint64_t *>(c->d_small + OFF_CTR);
    uint64_t *scan_scratch = bstart + kBuckets16 + 1;  // K15s status words, then its ticket
    hipStream_t ps = peers ? c->stream2 : c->stream;
    t = tic(c);
    if (peers) HIP_TRY(c, hipStreamWaitEvent(c->stream2, c->ev_meta, 0));
    if (c->scan_clean != c->m_bsize.p) {  // a new allocation: status words and ticket zeroed
        // once, on the stream the scan runs on (queued on the other one, behind the count
        // exchange's event, it raced the scan: a ticket cleared mid-launch hung the IPC group)
        HIP_TRY(c, hipMemsetAsync(scan_scratch, 0, (kRecvScanStatusWords + 1) * 8, ps));
        c->scan_clean = c->m_bsize.p;
    }
    // the runs' bucket bounds and the bucket starts in one row scan of P + 1 rows (the last
    // row is every bucket's total over the sources); classify reads the sizes off bstart
    HIP_TRY(c, launch_recv_plan_from_meta(meta_r, d_moff, (uint32_t)hlo[me], (uint32_t)nh[me], P,
                                          pos, bstart, scan_scratch, ps, ctr,
                                          (uint32_t)(kCtrBytes / 8), ++c->scan_epoch));
    const WorkLists wl = work_lists(c, 0);
    HIP_TRY(c, launch_classify_range(nullptr, bstart, wl, (uint32_t)hlo[me],
                                     (uint32_t)(hlo[me] + nh[me]), ps));
    const uint64_t seq = ++c->mail_seq;
    HIP_TRY(c, launch_publish(ctr, (uint32_t)(kCtrBytes / 8), c->d_mail + 8, c->d_mail, seq, ps));
    if (peers) {
        HIP_TRY(c, hipEventRecord(c->ev_plan, c->stream2));
        HIP_TRY(c, hipStreamWaitEvent(c->stream, c->ev_plan, 0));
    }
    toc(c, PH_COUNT, t);
    t = tic(c);
    RecvSpec sp;
    uint32_t *out = slot_ptr<uint32_t>(c, S_OUT);
    ST_TRY(spec_recv_launch(c, rbuf, true, pos, d_r, P, bstart, wl, out, &sp));
    uint64_t h[3 * (kLocalClasses + 1)];
    ST_TRY(wait_mail(c, seq, ps));
    memcpy(h, reinterpret_cast<const char *>(c->h_mail + 8), kCtrBytes);
    for (int k = 0; k <= kLocalClasses; ++k)  // the next call's launch shapes
        c->recv_hint[k] = (uint32_t)std::min<uint64_t>(h[3 * k], kBuckets16);
    c->recv_hint_ok = true;
    if (check_mode()) {
        for (int p = 0; p < P; ++p)
            ST_TRY(check_bounds(c, pos + (size_t)p * (kBuckets16 + 1), kBuckets16 + 1, recv[p],
                                "received run bounds"));
        uint64_t keys = 0;
        for (int l = 0; l <= kLocalClasses; ++l) keys += h[3 * l + 1];
        if (keys != mine)
            return set_err(c, GSORT_EINVAL, "GSORT_CHECK receive lists hold " +
                                                std::to_string(keys) + " keys, want " +
                                                std::to_string(mine) + " (rank " +
                                                std::to_string(me) + ")");
    }
    // (6) every bucket sorted from its P pieces: K11g by size class, K18c past them (classes
    // >= recv_cx and list 0, one persistent launch) -- what spec_recv_launch did not already
    // queue; a bucket past K18c's reach sends the block through recv_sort's MSD levels 1 and 0
    if (h[0] && h[2] > kHxMax) {  // recv_sort wants the P runs back to back in rbuf
        if (recv[me] && !self_moved)
            HIP_TRY(c, hipMemcpyAsync(rbuf + roffs[me], pack + cut[me], recv[me] * 2,
                                      hipMemcpyDeviceToDevice, c->stream));
        ST_TRY(ensure(c, c->slot[S_TMP], std::max<uint64_t>(mine, 1) * 4));
        ST_TRY(recv_sort(c, rbuf, true, recv, mine, out, slot_ptr<uint32_t>(c, S_TMP), stats));
    } else {
        ST_TRY(sort_recv_lists(c, rbuf, true, pos, d_r, P, bstart, wl, h, out, stats, true, &sp));
    }
    toc(c, PH_MERGE, t);
    *d_out = slot_ptr<int32_t>(c, S_OUT);
    *n_out = mine;
    return GSORT_OK;
}

// ---- distributed radix (P > 1): group, exact splitters, ONE exchange, receive sort --------
// The reference keeps rank q on global positions [qB, (q+1)B) by routing every key through
// rank 0 on each of its base-P passes (mpi_radix_sort.c:139 Scatter, :150-173 all-to-all,
// :180-192 Gatherv).  Here: (1) each rank groups its block by the top 16 bits; (2) radix select
// of the exact boundary keys: 4 rounds of 8 bits, each counting the keys below 257 thresholds
// per boundary by binary search on the grouped block (K13) and all-gathering the counts; (3) the
// cut of every block (gsort_plan_split: copies of a boundary key go left in rank order); (4) one
// grouped send/recv of contiguous runs; (5) the received runs are bucketed by their top 16 bits
// and every bucket is finished in LDS (packed_exchange_sort).
gsort_status radix_dist_exact(gsort_ctx *c, const int32_t *d_keys, uint64_t n_in,
                              int32_t **d_out, uint64_t *n_out, gsort_stats *stats) {
    const int P = c->nranks, me = c->rank;
    std::vector<uint64_t> n_all;
    ST_TRY(allgather_u64(c, n_in, n_all));
    uint64_t N = 0;
    for (uint64_t v : n_all) N += v;
    uint64_t B, mine;
    block_of(N, P, me, &B, &mine);
    // the packed exchange sends one u32 count per (destination, 16-bit bucket): every rank's
    // block, and so every count, must stay below 2^32 keys (decided identically on all ranks)
    for (int r = 0; r < P; ++r)
        if (n_all[r] >= (1ull << 32))
            return set_err(c, GSORT_EINVAL, "radix: a rank holds >= 2^32 keys (rank " +
                                                std::to_string(r) + "); split the input further");
    ST_TRY(check_send_limit(c, n_all, 2, "radix"));
    // (the receive side's buffers first: allocated before the grouping, as they always were)
    ST_TRY(ensure(c, c->slot[S_RECV], std::max<uint64_t>(mine, 1) * 2));
    ST_TRY(ensure(c, c->slot[S_OUT], std::max<uint64_t>(mine, 1) * 4));
    uint16_t *pack = nullptr;
    uint64_t *gb = nullptr;
    ST_TRY(group_block16(c, d_keys, n_in, stats, &pack, &gb));
    const int pr = stats ? stats->passes_run : 0;

    // (2) radix select of v_q, the g_q-th smallest key, for the P-1 inner boundaries: 4 rounds of
    // 8 bits, every round decided on the device (K13s sums the all-gathered counts, picks the
    // digit and writes the next round's thresholds), and after round 1 -- the boundaries'
    // 16-bit groups known -- K13g sorts each boundary group in place in the packed buffer, so
    // rounds 2 and 3 binary-search it and the cut splits it by value.  The host waits ONCE, for
    // the last round's counts (the cut and the exchange sizes RCCL needs on the host).  A
    // boundary group past K13g's 32 768 keys (skewed input) is flagged in the count rows of
    // rounds 2 and 3, so every rank sees it: all ranks then sort the groups on the host path and
    // repeat rounds 2 and 3 with the host between them (select_rounds below).
    const int nb = P - 1, M = 257, W = nb * M + nb;  // count row: nb x M counts + nb K13g flags
    std::vector<uint64_t> g(nb), prefix(nb, 0), all((size_t)P * W);
    std::vector<int> dsel(nb, 0);
    for (int q = 0; q < nb; ++q) g[q] = std::min<uint64_t>((uint64_t)(q + 1) * B, N);
    ST_TRY(ensure(c, c->m_split, (size_t)std::max(nb, 1) * (M * 16 + 32)));
    ST_TRY(ensure(c, c->slot[S_STAGE], (size_t)P * std::max(W, 1) * 8));
    // m_split: prefix (nb) | g (nb) | thresholds (nb x M) | counts (nb x M) + flags (nb), u64
    uint64_t *d_pref = reinterpret_cast<uint64_t *>(c->m_split.p), *d_g = d_pref + nb;
    uint64_t *d_xs = d_g + nb;
    uint64_t *d_cnt = d_xs + (size_t)nb * M;
    const uint64_t *d_all = reinterpret_cast<const uint64_t *>(c->slot[S_STAGE].p);
    // rounds k0 .. 3 from the thresholds in d_xs (K13g after round 1 when k0 == 0), then the last
    // round's rows and the boundary keys to the host
    auto select_rounds = [&](int k0) -> gsort_status {
        for (int k = k0; k < 4; ++k) {
            HIP_TRY(c, launch_count_below16(pack, gb, d_xs, nb * M, d_cnt, c->stream));
            ST_TRY(comm_try(c, c->comm->allgather(d_cnt, c->slot[S_STAGE].p, (size_t)W * 8,
                                                  c->stream)));
            HIP_TRY(c, launch_select_digit(d_all, W, d_g, N, P, nb, M, 24 - 8 * k, d_pref, d_xs,
                                           c->stream));
            if (k == 1)
                HIP_TRY(c, launch_boundary_sort16(pack, gb, d_pref, d_g, N, nb, c->atomic_rank,
                                                  d_cnt + (size_t)nb * M, c->stream));
        }
        HIP_TRY(c, hipMemcpyAsync(all.data(), d_all, all.size() * 8, hipMemcpyDeviceToHost,
                                  c->stream));
        HIP_TRY(c, hipMemcpyAsync(prefix.data(), d_pref, (size_t)nb * 8, hipMemcpyDeviceToHost,
                                  c->stream));
        HIP_TRY(c, hipStreamSynchronize(c->stream));
        return GSORT_OK;
    };
    // the thresholds of round 0 (prefix 0) and of round 2 after the host path (prefix: the top
    // 16 bits); prefix and g go along.  Staged in pinned memory at OFF_PLAN + 8 KiB (free: the
    // exchange table reuses it after select_rounds' synchronisation): a pageable copy would
    // hold the host in the runtime's staging until the stream had drained the sender's K1h ..
    // K3a, and the select's kernels would then be queued behind an idle GPU
    const size_t nx = (size_t)2 * nb + (size_t)nb * M;
    if (OFF_PLAN + 8192 + nx * 8 > kSmallBytes)
        return set_err(c, GSORT_EINVAL, "select thresholds too large");
    uint64_t *hx = reinterpret_cast<uint64_t *>(c->h_small + OFF_PLAN + 8192);
    auto put_thresholds = [&](int shift) -> gsort_status {
        for (int q = 0; q < nb; ++q) { hx[q] = prefix[q]; hx[nb + q] = g[q]; }
        for (int q = 0; q < nb; ++q)
            for (int d = 0; d < M; ++d)
                hx[2 * nb + (size_t)q * M + d] = prefix[q] + ((uint64_t)d << shift);
        HIP_TRY(c, hipMemcpyAsync(d_pref, hx, nx * 8, hipMemcpyHostToDevice, c->stream));
        return GSORT_OK;
    };
    hipEvent_t t = tic_rec(c);
    if (nb > 0) {  // (one rank: no boundary, nothing to select)
        ST_TRY(put_thresholds(24));
        ST_TRY(select_rounds(0));
        bool big = false;
        for (int p = 0; p < P; ++p)
            for (int q = 0; q < nb; ++q) big |= all[(size_t)p * W + (size_t)nb * M + q] != 0;
        if (big) {  // a boundary group past K13g's reach on some rank: every rank takes this
            std::vector<uint64_t> hs;
            for (int q = 0; q < nb; ++q)
                if (g[q] < N) hs.push_back(prefix[q] >> 16);
            ST_TRY(sort_groups16_host(c, pack, gb, hs));
            for (int q = 0; q < nb; ++q) prefix[q] = prefix[q] >> 16 << 16;
            ST_TRY(put_thresholds(8));
            ST_TRY(select_rounds(2));
        }
        for (int q = 0; q < nb; ++q) dsel[q] = (int)(prefix[q] & 255u);
    }
    toc_rec(c, PH_SAMPLE, t);
    // (3) cut points from the last round: lt = count(< v_q), le = count(< v_q + 1)
    std::vector<uint64_t> lt((size_t)P * nb), le((size_t)P * nb), send(P), recv(P);
    for (int p = 0; p < P; ++p)
        for (int q = 0; q < nb; ++q) {
            const uint64_t *row = &all[(size_t)p * W + (size_t)q * M];
            lt[(size_t)p * nb + q] = g[q] >= N ? n_all[p] : row[dsel[q]];
            le[(size_t)p * nb + q] = g[q] >= N ? n_all[p] : row[dsel[q] + 1];
        }
    gsort_status ps = gsort_plan_split(P, n_all.data(), lt.data(), le.data(), me, send.data(),
                                       recv.data());
    if (ps != GSORT_OK) return set_err(c, ps, "inconsistent splitter counts");
    // every destination block's keys lie in a known range of 16-bit buckets (from the boundary
    // keys), so the top 16 bits travel as one count per (destination, bucket)
    std::vector<uint64_t> hlo(P), nh(P), cut(P + 1, 0);
    for (int q = 0; q < P; ++q) {
        const uint64_t lo = q == 0 ? 0 : (g[q - 1] >= N ? 0xFFFFFFFFull : prefix[q - 1]);
        const uint64_t hi = q == P - 1 ? 0xFFFFFFFFull : (g[q] >= N ? 0xFFFFFFFFull : prefix[q]);
        hlo[q] = lo >> 16;
        nh[q] = (hi >> 16) - hlo[q] + 1;
        cut[q + 1] = cut[q] + send[q];
    }
    uint64_t got = 0;
    for (int p = 0; p < P; ++p) got += recv[p];
    if (got != mine) return set_err(c, GSORT_EINVAL, "exchange plan does not fill the block");
    ST_TRY(packed_exchange_sort(c, pack, gb, cut, recv, hlo, nh, stats, d_out, n_out));
    if (stats) stats->passes_run = pr;
    return GSORT_OK;
}

// ---- distributed LSD radix (P > 1, GSORT_LOCAL_LSD) ----------------------------------------
// Per non-trivial digit: local K1/K2 (tile counts; the digit totals of this rank), all-gather
// of the P x 256 per-rank digit counts, local K3 (stable by digit), route contiguous slices to
// the ranks owning their global positions (one grouped send/recv round), then place the
// received runs (K8).  Keeps the reference's invariant that rank q holds positions
// [qB, (q+1)B) after each pass (mpi_radix_sort.c:139,:192) without moving keys through rank 0.
// sort_keys != nullptr (the reference-compat sort): the passes sort the u32 keys sort_keys[i]
// (never flipped) stably and d_keys[i] travels with them as the value; the output is the
// values.  Keys and values go through the same exchange and placement, so the order is
// (key, source rank, source order), the reference's per-pass order (mpi_radix_sort.c:164-192).
gsort_status radix_dist(gsort_ctx *c, const int32_t *d_keys, uint64_t n_in, int32_t **d_out,
                        uint64_t *n_out, gsort_stats *stats, const uint32_t *sort_keys) {
    const int P = c->nranks, me = c->rank;
    const bool kv = sort_keys != nullptr, fl = !kv;
    std::vector<uint64_t> n_all;
    ST_TRY(allgather_u64(c, n_in, n_all));
    uint64_t N = 0;
    for (uint64_t v : n_all) N += v;
    uint64_t B, mine;
    block_of(N, P, me, &B, &mine);
    // a pass sends at most a rank's block (n_in, then B) of int32 keys
    ST_TRY(check_send_limit(c, std::vector<uint64_t>(1, std::max<uint64_t>(
                                   *std::max_element(n_all.begin(), n_all.end()), B)),
                            4, "radix (LSD passes)"));
    const uint64_t cap = std::max<uint64_t>(std::max(n_in, B), 1);
    for (Slot s : {S_CUR, S_SORTED, S_RECV, S_OUT}) ST_TRY(ensure(c, c->slot[s], cap * 4));
    if (kv)
        for (DevBuf *b : {&c->slot[S_TMP], &c->m_vtmp[0], &c->m_vtmp[1], &c->m_vtmp[2]})
            ST_TRY(ensure(c, *b, cap * 4));
    ST_TRY(ensure_pass_scratch(c, cap));
    if (N == 0) { *d_out = slot_ptr<int32_t>(c, S_OUT); *n_out = 0; return GSORT_OK; }

    // K1 on the input: tile counts of digit 0 + all four digit histograms; all-gathered they
    // give the global digit totals (invariant under the exchange), so every rank skips the
    // same trivial digits.
    uint64_t *d_hist = reinterpret_cast<uint64_t *>(c->d_small + OFF_HIST);
    uint64_t *d_tot = reinterpret_cast<uint64_t *>(c->d_small + OFF_TOT);
    const uint32_t *src = kv ? sort_keys : reinterpret_cast<const uint32_t *>(d_keys);
    HIP_TRY(c, hipMemsetAsync(d_hist, 0, 4 * kRadix * 8, c->stream));
    hipEvent_t t = tic(c);
    HIP_TRY(c, launch_tile_counts(src, n_in, 0, fl, d_tcounts(c), d_hist, c->stream));
    toc(c, PH_COUNT, t);
    DevBuf &allh = c->slot[S_STAGE];
    ST_TRY(ensure(c, allh, (size_t)P * 4 * kRadix * 8));
    ST_TRY(comm_try(c, c->comm->allgather(d_hist, allh.p, 4 * kRadix * 8, c->stream)));
    std::vector<uint64_t> H((size_t)P * 4 * kRadix);
    HIP_TRY(c, hipMemcpyAsync(H.data(), allh.p, H.size() * 8, hipMemcpyDeviceToHost, c->stream));
    HIP_TRY(c, hipStreamSynchronize(c->stream));
    std::vector<int> active;
    for (int p = 0; p < 4; ++p) {
        uint64_t mx = 0;
        for (int d = 0; d < kRadix; ++d) {
            uint64_t tot = 0;
            for (int r = 0; r < P; ++r) tot += H[((size_t)r * 4 + p) * kRadix + d];
            mx = std::max(mx, tot);
        }
        if (mx < N) active.push_back(p);
    }
    if (active.empty()) active.push_back(0);  // still redistribute to balanced blocks

    std::vector<uint64_t> hp((size_t)P * kRadix), send(P), recv(P), seg((size_t)4 * P * kRadix);
    std::vector<size_t> sc(P), sd(P), rc(P), rd(P);
    uint64_t n_src = n_in;
    uint32_t *placed[2] = {slot_ptr<uint32_t>(c, S_CUR), slot_ptr<uint32_t>(c, kv ? S_TMP : S_OUT)};
    // kv: the values' source, sorted / received copies and placed blocks (the last into S_OUT)
    const uint32_t *vsrc = reinterpret_cast<const uint32_t *>(d_keys);
    uint32_t *vsorted = reinterpret_cast<uint32_t *>(c->m_vtmp[0].p);
    uint32_t *vrecv = reinterpret_cast<uint32_t *>(c->m_vtmp[1].p);
    uint32_t *vplaced = reinterpret_cast<uint32_t *>(c->m_vtmp[2].p);
    const int k = (int)active.size();
    for (int i = 0; i < k; ++i) {
        const int p = active[i];
        const bool first = i == 0, last = i == k - 1;
        // this rank's tile counts and totals of digit p, then everyone's totals
        if (!(first && p == 0)) ST_TRY(count_tiles(c, src, n_src, p, first && fl));
        uint32_t *sorted = slot_ptr<uint32_t>(c, S_SORTED);
        ST_TRY(scan_and_scatter(c, src, sorted, n_src, p, first && fl, false, kv ? vsrc : nullptr,
                                kv ? vsorted : nullptr));
        if (n_src == 0) HIP_TRY(c, hipMemsetAsync(d_tot, 0, kRadix * 8, c->stream));
        uint64_t *d_allt = reinterpret_cast<uint64_t *>(allh.p);
        ST_TRY(comm_try(c, c->comm->allgather(d_tot, d_allt, kRadix * 8, c->stream)));
        HIP_TRY(c, hipMemcpyAsync(hp.data(), d_allt, hp.size() * 8, hipMemcpyDeviceToHost,
                                  c->stream));
        HIP_TRY(c, hipStreamSynchronize(c->stream));

        size_t nseg = 0;
        ST_TRY(gsort_plan_radix_route(P, hp.data(), B, me, send.data(), recv.data(), seg.data(),
                                      &nseg));
        size_t so = 0, ro = 0;
        for (int q = 0; q < P; ++q) {
            sc[q] = send[q] * 4; sd[q] = so; so += sc[q];
            rc[q] = recv[q] * 4; rd[q] = ro; ro += rc[q];
            if (stats && q != me) {
                stats->bytes_sent += sc[q] * (kv ? 2 : 1);
                stats->max_pair_bytes = std::max<uint64_t>(stats->max_pair_bytes, sc[q]);
            }
        }
        uint32_t *rbuf = slot_ptr<uint32_t>(c, S_RECV);
        t = tic_rec(c);
        ST_TRY(comm_try(c, c->comm->alltoallv(sorted, sc.data(), sd.data(), rbuf, rc.data(),
                                              rd.data(), c->stream)));
        if (kv)
            ST_TRY(comm_try(c, c->comm->alltoallv(vsorted, sc.data(), sd.data(), vrecv,
                                                  rc.data(), rd.data(), c->stream)));
        toc_rec(c, PH_EXCH, t);
        if (stats) stats->exchanges++;
        // placement table: {offset in recv buffer, dest offset, length}
        uint64_t *h_seg = reinterpret_cast<uint64_t *>(c->h_small + OFF_PLAN);
        uint64_t *d_seg = reinterpret_cast<uint64_t *>(c->d_small + OFF_PLAN);
        if (nseg * 24 > kSmallBytes - OFF_PLAN) return set_err(c, GSORT_EINVAL, "segment table");
        HIP_TRY(c, hipStreamSynchronize(c->stream));  // h_seg may still feed an earlier copy
        for (size_t s = 0; s < nseg; ++s) {
            const uint64_t r = seg[4 * s];
            h_seg[3 * s + 0] = rd[r] / 4 + seg[4 * s + 1];
            h_seg[3 * s + 1] = seg[4 * s + 2];
            h_seg[3 * s + 2] = seg[4 * s + 3];
        }
        HIP_TRY(c, hipMemcpyAsync(d_seg, h_seg, nseg * 24, hipMemcpyHostToDevice, c->stream));
        uint32_t *dst = last && !kv ? slot_ptr<uint32_t>(c, S_OUT) : placed[i & 1];
        t = tic(c);
        if (!(kv && last))  // kv: the keys of the last pass are not needed
            HIP_TRY(c, launch_place(rbuf, dst, d_seg, (int)nseg, mine, nullptr, 0, last && fl,
                                    c->stream));
        if (kv) {
            uint32_t *vdst = last ? slot_ptr<uint32_t>(c, S_OUT) : vplaced;
            HIP_TRY(c, launch_place(vrecv, vdst, d_seg, (int)nseg, mine, nullptr, 0, false,
                                    c->stream));
            vsrc = vdst;
        }
        toc(c, PH_PLACE, t);
        src = dst;
        n_src = mine;
    }
    if (stats) stats->passes_run = k;
    *d_out = slot_ptr<int32_t>(c, S_OUT);
    *n_out = mine;
    return GSORT_OK;
}

// ---- reference-compat radix (gsort_set_ref_compat) -----------------------
// The reference's radix sort is a stable sort of the values by the base-P digits of |v| that
// number_digit_at extracts (mpi_radix_sort.c:54-58), loop = number_digits(max) of them (:100).
// K20 + an all-gather give the global min / max, gsort_plan_ref_digits the reference's digit
// plan, K19 the composite key of every value; then stable key-value LSD passes: locally, or
// through radix_dist's exchange (kv), so rank q ends with positions [qB, (q+1)B).
gsort_status radix_compat(gsort_ctx *c, const int32_t *d_keys, uint64_t n_in, int32_t **d_out,
                          uint64_t *n_out, gsort_stats *stats) {
    const int Pref = c->ref_compat > 0 ? c->ref_compat : c->nranks;
    std::vector<uint64_t> n_all;
    ST_TRY(allgather_u64(c, n_in, n_all));
    uint64_t N = 0;
    for (uint64_t v : n_all) N += v;
    const uint64_t Bref = (N + Pref - 1) / Pref;
    if (N > 0 && (int64_t)N - (int64_t)(Bref * (uint64_t)(Pref - 1)) <= 0)
        return set_err(c, GSORT_EINVAL, "ref compat: the reference's last block would be empty "
                                        "(N < (P-1)*ceil(N/P) + 1, quirk Q8)");
    const size_t cap = std::max<uint64_t>(n_in, 1) * 4;
    ST_TRY(ensure(c, c->m_cmm, 16));
    ST_TRY(ensure(c, c->m_ckey[0], cap));
    // global min / max (K20)
    int32_t *h_mm = reinterpret_cast<int32_t *>(c->h_small + OFF_PLAN);
    HIP_TRY(c, hipStreamSynchronize(c->stream));  // h_small may feed an earlier copy
    h_mm[0] = INT32_MAX;
    h_mm[1] = INT32_MIN;
    memset(h_mm + 2, 0, 8);  // K19's bad-key counter
    HIP_TRY(c, hipMemcpyAsync(c->m_cmm.p, h_mm, 16, hipMemcpyHostToDevice, c->stream));
    HIP_TRY(c, launch_minmax(d_keys, n_in, reinterpret_cast<int *>(c->m_cmm.p), c->stream));
    HIP_TRY(c, hipMemcpyAsync(h_mm, c->m_cmm.p, 8, hipMemcpyDeviceToHost, c->stream));
    HIP_TRY(c, hipStreamSynchronize(c->stream));
    std::vector<uint64_t> mm;
    ST_TRY(allgather_u64(c, (uint64_t)(uint32_t)h_mm[0] | ((uint64_t)(uint32_t)h_mm[1] << 32), mm));
    int32_t gmin = INT32_MAX, gmax = -1;  // the reference's max_element starts at -1 (:77)
    for (int r = 0; r < c->nranks; ++r) {
        if (!n_all[r]) continue;
        gmin = std::min(gmin, (int32_t)(uint32_t)mm[r]);
        gmax = std::max(gmax, (int32_t)(uint32_t)(mm[r] >> 32));
    }
    if (N > 0 && gmin == INT32_MIN)
        return set_err(c, GSORT_EINVAL, "ref compat: an INT_MIN key has no |v|; the reference "
                                        "indexes a negative bucket there (quirk Q5)");
    int loop = 0;
    int32_t mod[64];
    double scale[64];
    if (gsort_plan_ref_digits(Pref, gmax, &loop, mod, scale, 64) != GSORT_OK)
        return set_err(c, GSORT_EINVAL, "ref compat: digit plan");
    uint32_t *key = reinterpret_cast<uint32_t *>(c->m_ckey[0].p);
    if (loop < 1) {  // no pass (P = 1, Q1): the input order, only redistributed
        HIP_TRY(c, hipMemsetAsync(key, 0, cap, c->stream));
    } else {
        HIP_TRY(c, launch_compat_keys(d_keys, n_in, Pref, loop, mod, scale, key,
                                      reinterpret_cast<uint64_t *>(c->m_cmm.p) + 1, c->stream));
        uint64_t *h_bad = reinterpret_cast<uint64_t *>(c->h_small + OFF_PLAN);
        HIP_TRY(c, hipMemcpyAsync(h_bad, reinterpret_cast<uint64_t *>(c->m_cmm.p) + 1, 8,
                                  hipMemcpyDeviceToHost, c->stream));
        HIP_TRY(c, hipStreamSynchronize(c->stream));
        std::vector<uint64_t> bad;
        ST_TRY(allgather_u64(c, *h_bad, bad));
        for (uint64_t b : bad)
            if (b) return set_err(c, GSORT_EINVAL, "ref compat: a digit outside [0, P) (the "
                                                   "reference indexes outside its buckets)");
    }
    if (c->comm) return radix_dist(c, d_keys, n_in, d_out, n_out, stats, key);
    // one rank: the stable key-value LSD passes locally (K1 + four histograms, K2, K3 kv)
    ST_TRY(ensure(c, c->slot[S_OUT], cap));
    ST_TRY(ensure(c, c->m_ckey[1], cap));
    ST_TRY(ensure(c, c->m_vtmp[0], cap));
    ST_TRY(ensure(c, c->m_vtmp[1], cap));
    ST_TRY(ensure_pass_scratch(c, n_in));
    *d_out = slot_ptr<int32_t>(c, S_OUT);
    *n_out = n_in;
    if (n_in == 0) return GSORT_OK;
    uint64_t *d_hist = reinterpret_cast<uint64_t *>(c->d_small + OFF_HIST);
    uint64_t *h_hist = reinterpret_cast<uint64_t *>(c->h_small + OFF_HIST);
    HIP_TRY(c, hipMemsetAsync(d_hist, 0, 4 * kRadix * 8, c->stream));
    hipEvent_t t = tic(c);
    HIP_TRY(c, launch_tile_counts(key, n_in, 0, false, d_tcounts(c), d_hist, c->stream));
    toc(c, PH_COUNT, t);
    HIP_TRY(c, hipMemcpyAsync(h_hist, d_hist, 4 * kRadix * 8, hipMemcpyDeviceToHost, c->stream));
    HIP_TRY(c, hipStreamSynchronize(c->stream));
    std::vector<int> active;
    for (int p = 0; p < 4; ++p) {
        const uint64_t *h = h_hist + p * kRadix;
        if (*std::max_element(h, h + kRadix) < n_in) active.push_back(p);
    }
    if (active.empty()) {
        HIP_TRY(c, launch_copy(reinterpret_cast<const uint32_t *>(d_keys),
                               slot_ptr<uint32_t>(c, S_OUT), n_in, c->stream));
        return GSORT_OK;
    }
    uint32_t *kb[2] = {key, reinterpret_cast<uint32_t *>(c->m_ckey[1].p)};
    uint32_t *vb[2] = {reinterpret_cast<uint32_t *>(c->m_vtmp[0].p),
                       reinterpret_cast<uint32_t *>(c->m_vtmp[1].p)};
    const uint32_t *vsrc = reinterpret_cast<const uint32_t *>(d_keys);
    const int k = (int)active.size();
    for (int i = 0; i < k; ++i) {
        const bool last = i == k - 1;
        uint32_t *vdst = last ? slot_ptr<uint32_t>(c, S_OUT) : vb[i & 1];
        if (!(i == 0 && active[0] == 0)) ST_TRY(count_tiles(c, kb[i & 1], n_in, active[i], false));
        ST_TRY(scan_and_scatter(c, kb[i & 1], kb[(i & 1) ^ 1], n_in, active[i], false, false, vsrc,
                                vdst));
        vsrc = vdst;
    }
    if (stats) stats->passes_run = k;
    return GSORT_OK;
}

// ---- sample sort ------------------------------------------------------------------------
// The reference (mpi_sample_sort.c:85-174): local qsort, 2P-1 regular samples of the sorted
// block to the root, P-1 splitters from the sorted samples, each key to the first bucket whose
// splitter is >= it, all-to-all, final qsort.

// The int32 form (the LSD local algorithm, a rank past 2^32 keys, or -- rarely -- below): a
// full local sort, K4 samples, K5 + broadcast, K6 bounds on the sorted block, an int32
// exchange and the receive sort of the P sorted runs.
gsort_status sample_dist_sorted(gsort_ctx *c, const int32_t *d_keys, uint64_t n_in,
                                const std::vector<uint64_t> &n_all, int32_t **d_out,
                                uint64_t *n_out, gsort_stats *stats) {
    const int P = c->nranks, me = c->rank;
    uint64_t N = 0;
    for (uint64_t v : n_all) N += v;
    const uint64_t B = (N + P - 1) / P;
    const int k = 2 * P - 1;
    const uint64_t interval = B / k;
    ST_TRY(check_send_limit(c, n_all, 4, "sample"));
    const uint64_t cap = std::max<uint64_t>(n_in, 1);
    ST_TRY(ensure(c, c->slot[S_SORTED], cap * 4));
    int32_t *sorted = slot_ptr<int32_t>(c, S_SORTED);
    int pr = 0;
    ST_TRY(local_sort(c, reinterpret_cast<const uint32_t *>(d_keys), n_in,
                      reinterpret_cast<uint32_t *>(sorted), nullptr, &pr, nullptr, true));

    // K4 samples -> root (grouped send/recv), K5 on root, broadcast splitters
    hipEvent_t t = tic_rec(c);
    int32_t *d_samp = reinterpret_cast<int32_t *>(c->d_small + OFF_PLAN);
    int32_t *d_all = d_samp + 64;
    int32_t *d_spl = d_all + 1024 + 64;
    uint64_t *d_bounds = reinterpret_cast<uint64_t *>(d_spl + 64);
    HIP_TRY(c, launch_regular_sample(sorted, interval, k, d_samp, c->stream));
    std::vector<size_t> sc(P, 0), sd(P, 0), rc(P, 0), rd(P, 0);
    sc[0] = (size_t)k * 4;
    if (me == 0)
        for (int r = 0; r < P; ++r) { rc[r] = (size_t)k * 4; rd[r] = (size_t)r * k * 4; }
    ST_TRY(comm_try(c, c->comm->alltoallv(d_samp, sc.data(), sd.data(), d_all, rc.data(),
                                          rd.data(), c->stream)));
    if (me == 0) HIP_TRY(c, launch_select_splitters(d_all, P * k, k, P - 1, d_spl, c->stream));
    ST_TRY(comm_try(c, c->comm->bcast(d_spl, (size_t)(P - 1) * 4, 0, c->stream)));
    HIP_TRY(c, launch_bucket_bounds(sorted, n_in, d_spl, P - 1, d_bounds, c->stream));
    toc_rec(c, PH_SAMPLE, t);
    int32_t *h_spl = reinterpret_cast<int32_t *>(c->h_small + OFF_PLAN);
    uint64_t *h_bounds = reinterpret_cast<uint64_t *>(c->h_small + OFF_PLAN + 1024);
    HIP_TRY(c, hipMemcpyAsync(h_spl, d_spl, (size_t)(P - 1) * 4, hipMemcpyDeviceToHost, c->stream));
    HIP_TRY(c, hipMemcpyAsync(h_bounds, d_bounds, (size_t)(P - 1) * 8, hipMemcpyDeviceToHost,
                              c->stream));
    HIP_TRY(c, hipStreamSynchronize(c->stream));
    c->splitters.assign(h_spl, h_spl + P - 1);
    c->bucket_counts.assign(P, 0);
    uint64_t prev = 0;
    for (int j = 0; j < P; ++j) {
        const uint64_t end = j < P - 1 ? h_bounds[j] : n_in;
        c->bucket_counts[j] = end - prev;
        prev = end;
    }
    // bucket-count matrix: allgather P counts per rank (mpi_sample_sort.c:161,:168 sends the
    // length in the MPI tag of a fixed-size message; here exact lengths size the messages)
    uint64_t *d_cnt = reinterpret_cast<uint64_t *>(c->d_small + OFF_PLAN + 16384);
    uint64_t *d_mat = d_cnt + 64;
    uint64_t *h_cnt = reinterpret_cast<uint64_t *>(c->h_small + OFF_PLAN + 16384);
    std::vector<uint64_t> M((size_t)P * P);
    if (!c->sample_balanced) {
        memcpy(h_cnt, c->bucket_counts.data(), (size_t)P * 8);
        HIP_TRY(c, hipMemcpyAsync(d_cnt, h_cnt, (size_t)P * 8, hipMemcpyHostToDevice, c->stream));
        ST_TRY(comm_try(c, c->comm->allgather(d_cnt, d_mat, (size_t)P * 8, c->stream)));
        HIP_TRY(c, hipMemcpyAsync(M.data(), d_mat, M.size() * 8, hipMemcpyDeviceToHost, c->stream));
        HIP_TRY(c, hipStreamSynchronize(c->stream));
    } else {
        // duplicate-aware buckets: keys < s_j (strict K6) and <= s_j of every rank, then the
        // same cut rule as the distributed radix with the boundary clamped into s_j's copies
        const int S = P - 1;
        uint64_t *d_lt = d_bounds + 64;
        HIP_TRY(c, launch_bucket_bounds(sorted, n_in, d_spl, S, d_lt, c->stream, true));
        uint64_t *d_ll = d_cnt;  // this rank: [lt x S | le x S]
        HIP_TRY(c, hipMemcpyAsync(d_ll, d_lt, (size_t)S * 8, hipMemcpyDeviceToDevice, c->stream));
        HIP_TRY(c, hipMemcpyAsync(d_ll + S, d_bounds, (size_t)S * 8, hipMemcpyDeviceToDevice,
                                  c->stream));
        uint64_t *d_all2 = d_cnt + 64;
        ST_TRY(comm_try(c, c->comm->allgather(d_ll, d_all2, (size_t)2 * S * 8, c->stream)));
        std::vector<uint64_t> A((size_t)P * 2 * S), lt((size_t)P * S), le((size_t)P * S);
        HIP_TRY(c, hipMemcpyAsync(A.data(), d_all2, A.size() * 8, hipMemcpyDeviceToHost, c->stream));
        HIP_TRY(c, hipStreamSynchronize(c->stream));
        for (int p = 0; p < P; ++p)
            for (int j = 0; j < S; ++j) {
                lt[(size_t)p * S + j] = A[(size_t)p * 2 * S + j];
                le[(size_t)p * S + j] = A[(size_t)p * 2 * S + S + j];
            }
        // every rank plans every rank's row (host, identical inputs) -> the full matrix
        std::vector<uint64_t> snd(P), rcv(P);
        for (int p = 0; p < P; ++p) {
            const gsort_status st =
                gsort_plan_split_balanced(P, n_all.data(), lt.data(), le.data(), p, snd.data(),
                                          rcv.data());
            if (st != GSORT_OK) return set_err(c, st, "inconsistent sample bucket bounds");
            for (int q = 0; q < P; ++q) M[(size_t)p * P + q] = snd[q];
        }
        for (int q = 0; q < P; ++q) c->bucket_counts[q] = M[(size_t)me * P + q];
    }
    uint64_t total = 0;
    size_t so = 0, ro = 0;
    for (int q = 0; q < P; ++q) {
        sc[q] = c->bucket_counts[q] * 4; sd[q] = so; so += sc[q];
        rc[q] = M[(size_t)q * P + me] * 4; rd[q] = ro; ro += rc[q];
        total += M[(size_t)q * P + me];
        if (stats && q != me) {
            stats->bytes_sent += sc[q];
            stats->max_pair_bytes = std::max<uint64_t>(stats->max_pair_bytes, sc[q]);
        }
    }
    const uint64_t cap2 = std::max<uint64_t>(total, 1);
    ST_TRY(ensure(c, c->slot[S_RECV], cap2 * 4));
    ST_TRY(ensure(c, c->slot[S_OUT], cap2 * 4));
    ST_TRY(ensure(c, c->slot[S_TMP], cap2 * 4));
    int32_t *rbuf = slot_ptr<int32_t>(c, S_RECV);
    // the rank's own bucket stays where it is (recv_sort reads it in place)
    const size_t self_off = sd[me];
    sc[me] = 0;
    rc[me] = 0;
    t = tic_rec(c);
    ST_TRY(comm_try(c, c->comm->alltoallv(sorted, sc.data(), sd.data(), rbuf, rc.data(),
                                          rd.data(), c->stream)));
    toc_rec(c, PH_EXCH, t);
    if (stats) stats->exchanges = 1;
    // final local order of the received bucket (mpi_sample_sort.c:174): the P received runs
    // are sorted slices of the senders' sorted blocks -> recv_sort
    std::vector<uint64_t> rlen(P);
    for (int q = 0; q < P; ++q) rlen[q] = M[(size_t)q * P + me];
    t = tic(c);
    ST_TRY(recv_sort(c, rbuf, false, rlen, total, slot_ptr<uint32_t>(c, S_OUT),
                     slot_ptr<uint32_t>(c, S_TMP), stats, me, sorted + self_off / 4));
    toc(c, PH_MERGE, t);
    if (stats) stats->passes_run = pr;
    *d_out = slot_ptr<int32_t>(c, S_OUT);
    *n_out = total;
    return GSORT_OK;
}

// The packed form (default, round 6): no local sort.  The block is grouped
// by its top 16 bits exactly as the distributed radix's sender groups it (group_block16), and
// the reference's quantities are read off the grouped block:
//   * regular sample i = sorted[i * interval] (mpi_sample_sort.c:94-104) is the
//     (i * interval - gb[h])-th smallest key of the group h holding that position: K4g finds
//     the k = 2P-1 groups, K13g sorts them in place (the only keys sorted before the exchange),
//     K4r reads the samples;
//   * the splitters: the root's K5 over the gathered samples + ncclBroadcast, as before
//     (:107-133);
//   * bucket bounds #keys <= s_j (:148-155): K6g + K13g sort the splitters' groups, K13
//     binary-searches them (count_below16), and #keys < s_j for the duplicate-aware rule;
//   * the bucket matrix (the lengths the reference sends in its MPI tags, :161-168) by one
//     all-gather of those counts, read on the host with the K13g flags: the ONE host wait;
//   * the exchange of 2 B per key and the receive sort of the radix path (packed_exchange_sort).
// A group past K13g's 32 768 keys (skewed keys: Zipf) is flagged; every rank sees the flags in
// the gathered rows and all of them redo the select with those groups sorted on the host path
// (sort_groups16_host: K11 or the LSD passes), waiting on the host between the steps.
gsort_status sample_dist(gsort_ctx *c, const int32_t *d_keys, uint64_t n_in, int32_t **d_out,
                         uint64_t *n_out, gsort_stats *stats) {
    const int P = c->nranks, me = c->rank;
    std::vector<uint64_t> n_all;
    ST_TRY(allgather_u64(c, n_in, n_all));
    uint64_t N = 0;
    for (uint64_t v : n_all) N += v;
    // mpi_sample_sort.c:72 size_bucket = ceil(N/P); :89-90 k = 2P-1, interval = B / k
    const uint64_t B = (N + P - 1) / P;
    const int k = 2 * P - 1, S = P - 1;
    const uint64_t interval = B / k;
    if (P * k > 1024) return set_err(c, GSORT_EINVAL, "too many ranks for sample sort");
    for (int r = 0; r < P; ++r)  // :94-99, decided identically on every rank
        if ((uint64_t)(k - 1) * interval >= n_all[r])
            return set_err(c, GSORT_ENOSAMPLE,
                           "no enough sample: rank " + std::to_string(r) + " holds " +
                               std::to_string(n_all[r]) + " keys, needs index " +
                               std::to_string((uint64_t)(k - 1) * interval));
    // GSORT_SAMPLE_INT32=1: the int32 form whatever the block (A/B and test hook)
    const char *fi = getenv("GSORT_SAMPLE_INT32");  // (read per call: tests flip it)
    const bool force_int32 = fi && fi[0] == '1';
    bool packed = c->local_algo != GSORT_LOCAL_LSD && !force_int32;
    for (int r = 0; r < P; ++r) packed &= n_all[r] < (1ull << 32);  // u32 bucket counts
    if (!packed) return sample_dist_sorted(c, d_keys, n_in, n_all, d_out, n_out, stats);
    ST_TRY(check_send_limit(c, n_all, 2, "sample"));
    uint16_t *pack = nullptr;
    uint64_t *gb = nullptr;
    ST_TRY(group_block16(c, d_keys, n_in, stats, &pack, &gb));
    const int pr = stats ? stats->passes_run : 0;

    // count row per rank: le (S) | lt (S) | K13g flags of the sample groups (k) and of the
    // splitter groups (S)
    const int W = 3 * S + k;
    const size_t nw = (size_t)2 * (k + S) + 2 * S + W;  // u64 words of m_split, then int32s
    ST_TRY(ensure(c, c->m_split, nw * 8 + ((size_t)k + (size_t)P * k + S + 64) * 4));
    ST_TRY(ensure(c, c->slot[S_STAGE], (size_t)P * W * 8));
    uint64_t *d_pref = reinterpret_cast<uint64_t *>(c->m_split.p);  // k sample + S splitter groups
    uint64_t *d_g = d_pref + k + S;                                  // (zeros: K13g's "g < N")
    uint64_t *d_xs = d_g + k + S;                                    // 2S thresholds
    uint64_t *d_row = d_xs + 2 * S;
    int32_t *d_samp = reinterpret_cast<int32_t *>(d_row + W);
    int32_t *d_sall = d_samp + k;
    int32_t *d_spl = d_sall + (size_t)P * k;
    const uint64_t *d_all = reinterpret_cast<const uint64_t *>(c->slot[S_STAGE].p);
    std::vector<uint64_t> all((size_t)P * W);
    std::vector<int32_t> spl(S);
    std::vector<size_t> sc(P, 0), sd(P, 0), rc(P, 0), rd(P, 0);
    sc[0] = (size_t)k * 4;
    if (me == 0)
        for (int r = 0; r < P; ++r) { rc[r] = (size_t)k * 4; rd[r] = (size_t)r * k * 4; }
    // host == false: the common path, no host wait until the gathered rows.  host == true: the
    // groups holding samples and splitters sorted on the host path (after a K13g flag), each
    // group once (a Zipf block's giant group holds samples and splitters alike)
    std::set<uint64_t> host_sorted;
    auto host_sort = [&](std::vector<uint64_t> hs) -> gsort_status {
        std::vector<uint64_t> todo;
        for (uint64_t g : hs)
            if (host_sorted.insert(g).second) todo.push_back(g);
        return sort_groups16_host(c, pack, gb, todo);
    };
    auto select = [&](bool host) -> gsort_status {
        HIP_TRY(c, launch_sample_groups(gb, interval, k, d_pref, d_g, c->stream));
        if (!host) {
            HIP_TRY(c, launch_boundary_sort16(pack, gb, d_pref, d_g, 1, k, c->atomic_rank,
                                              d_row + 2 * S, c->stream));
        } else {
            std::vector<uint64_t> pf(k), hs;
            HIP_TRY(c, hipMemcpyAsync(pf.data(), d_pref, (size_t)k * 8, hipMemcpyDeviceToHost,
                                      c->stream));
            HIP_TRY(c, hipStreamSynchronize(c->stream));
            for (uint64_t v : pf) hs.push_back(v >> 16);
            ST_TRY(host_sort(hs));
        }
        HIP_TRY(c, launch_read_samples16(pack, d_pref, interval, k, d_samp, c->stream));
        ST_TRY(comm_try(c, c->comm->alltoallv(d_samp, sc.data(), sd.data(), d_sall, rc.data(),
                                              rd.data(), c->stream)));
        if (me == 0) HIP_TRY(c, launch_select_splitters(d_sall, P * k, k, S, d_spl, c->stream));
        ST_TRY(comm_try(c, c->comm->bcast(d_spl, (size_t)S * 4, 0, c->stream)));
        HIP_TRY(c, launch_splitter_groups(d_spl, S, d_pref + k, d_g + k, d_xs, c->stream));
        if (!host) {
            HIP_TRY(c, launch_boundary_sort16(pack, gb, d_pref + k, d_g + k, 1, S,
                                              c->atomic_rank, d_row + 2 * S + k, c->stream));
        } else {
            HIP_TRY(c, hipMemcpyAsync(spl.data(), d_spl, (size_t)S * 4, hipMemcpyDeviceToHost,
                                      c->stream));
            HIP_TRY(c, hipStreamSynchronize(c->stream));
            std::vector<uint64_t> hs;
            for (int32_t v : spl) hs.push_back(((uint32_t)v ^ 0x80000000u) >> 16);
            ST_TRY(host_sort(hs));
            HIP_TRY(c, hipMemsetAsync(d_row + 2 * S, 0, (size_t)(k + S) * 8, c->stream));
        }
        HIP_TRY(c, launch_count_below16(pack, gb, d_xs, 2 * S, d_row, c->stream));
        ST_TRY(comm_try(c, c->comm->allgather(d_row, c->slot[S_STAGE].p, (size_t)W * 8,
                                              c->stream)));
        HIP_TRY(c, hipMemcpyAsync(all.data(), d_all, all.size() * 8, hipMemcpyDeviceToHost,
                                  c->stream));
        if (S)
            HIP_TRY(c, hipMemcpyAsync(spl.data(), d_spl, (size_t)S * 4, hipMemcpyDeviceToHost,
                                      c->stream));
        HIP_TRY(c, hipStreamSynchronize(c->stream));
        return GSORT_OK;
    };
    hipEvent_t t = tic_rec(c);
    if (P > 1) {  // (one rank: one bucket, nothing to split -- as the radix path skips its select)
        ST_TRY(select(false));
        bool big = false;
        for (int p = 0; p < P; ++p)
            for (int i = 2 * S; i < W; ++i) big |= all[(size_t)p * W + i] != 0;
        if (c->plan_trace && big) fprintf(stderr, "gsort sample: a group past K13g, host path\n");
        if (big) ST_TRY(select(true));
    }
    toc_rec(c, PH_SAMPLE, t);
    // (3) the bucket matrix M[p][q] (rank p's keys for bucket q) and this rank's cut
    c->splitters.assign(spl.begin(), spl.end());
    std::vector<uint64_t> M((size_t)P * P), lt((size_t)P * S), le((size_t)P * S);
    for (int p = 0; p < P; ++p)
        for (int j = 0; j < S; ++j) {
            le[(size_t)p * S + j] = all[(size_t)p * W + j];
            lt[(size_t)p * S + j] = all[(size_t)p * W + S + j];
        }
    for (int p = 0; p < P; ++p) {
        if (!c->sample_balanced) {
            uint64_t prev = 0;
            for (int q = 0; q < P; ++q) {
                const uint64_t end = q < S ? le[(size_t)p * S + q] : n_all[p];
                if (end < prev || end > n_all[p])
                    return set_err(c, GSORT_EINVAL, "inconsistent sample bucket bounds");
                M[(size_t)p * P + q] = end - prev;
                prev = end;
            }
        } else {
            // duplicate-aware buckets: the distributed radix's cut rule with the boundary
            // clamped into s_j's copies; every rank plans every rank's row (identical inputs)
            std::vector<uint64_t> snd(P), rcv(P);
            const gsort_status st = gsort_plan_split_balanced(P, n_all.data(), lt.data(),
                                                              le.data(), p, snd.data(), rcv.data());
            if (st != GSORT_OK) return set_err(c, st, "inconsistent sample bucket bounds");
            for (int q = 0; q < P; ++q) M[(size_t)p * P + q] = snd[q];
        }
    }
    c->bucket_counts.assign(P, 0);
    std::vector<uint64_t> cut(P + 1, 0), recv(P), hlo(P), nh(P);
    for (int q = 0; q < P; ++q) {
        c->bucket_counts[q] = M[(size_t)me * P + q];
        cut[q + 1] = cut[q] + M[(size_t)me * P + q];
        recv[q] = M[(size_t)q * P + me];
        // bucket q holds keys in [s_{q-1}, s_q] (the reference's (s_{q-1}, s_q]; the balanced
        // rule may also give it copies of s_{q-1}): 16-bit buckets from s_{q-1}'s to s_q's
        const uint64_t lo = q == 0 ? 0 : ((uint32_t)spl[q - 1] ^ 0x80000000u);
        const uint64_t hi = q == S ? 0xFFFFFFFFull : ((uint32_t)spl[q] ^ 0x80000000u);
        hlo[q] = lo >> 16;
        nh[q] = (hi >> 16) - hlo[q] + 1;
    }
    if (cut[P] != n_in) return set_err(c, GSORT_EINVAL, "sample cut does not cover the block");
    ST_TRY(packed_exchange_sort(c, pack, gb, cut, recv, hlo, nh, stats, d_out, n_out));
    if (stats) stats->passes_run = pr;
    return GSORT_OK;
}


// The sort writes its scratch slots; an input living in one of them would be overwritten.
}  // namespace rt
}  // namespace gsort
