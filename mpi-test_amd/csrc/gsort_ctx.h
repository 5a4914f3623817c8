// gsort_ctx.h -- internal to libgsort: the context, its scratch layout and the helpers the
// runtime's translation units share:
//   gsort_runtime.cpp  contexts, device memory, timing, diagnostics, the C-ABI, drop-in staging
//   gsort_local.cpp    the one-rank sorts (LSD passes, MSD levels, two-level / sampled plans,
//                      the counted dominant child) -- mpi_radix_sort.c:144-147, mpi_sample_sort.c:85
//   gsort_dist.cpp     the distributed sorts (receive side, radix select + one exchange, LSD
//                      passes, reference-compat order, sample sort) -- mpi_radix_sort.c:150-192,
//                      mpi_sample_sort.c:89-174
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <cmath>
#include <atomic>
#include <chrono>
#include <map>
#include <mutex>
#include <set>
#include <string>
#include <thread>
#include <vector>

#include "gsort.h"
#include "gsort_comm.h"
#include "gsort_debug.h"
#include "gsort_kernels.h"

using namespace gsort;

struct gsort_group {
    GroupState *st;
};

namespace gsort {
namespace rt {

enum Slot { S_TMP, S_OUT, S_CUR, S_SORTED, S_RECV, S_IN, S_STAGE, S_NSLOTS };
enum Phase { PH_COUNT, PH_PASS0, PH_PASS1, PH_PASS2, PH_PASS3, PH_EXCH, PH_PLACE, PH_SAMPLE,
             PH_MERGE, PH_TOTAL, PH_LEVEL3, PH_LEVEL2, PH_LEVEL1, PH_LEVEL0, PH_BUCKET, PH_N };

constexpr size_t kSmallBytes = 256 * 1024;  // device + pinned scratch for counts, plans
constexpr size_t kMailBytes = 4096;          // K12p mailbox: flag, then the counters (u64)

struct DevBuf {
    void *p = nullptr;     // what the kernels use
    size_t cap = 0;        // usable bytes at p
    void *base = nullptr;  // the allocation (p - kGuardBytes with GSORT_CANARY)
    // GSORT_EFENCE: the reserved VA range [base, base + va_bytes) and its physical handle
    size_t va_bytes = 0, map_bytes = 0;
    hipMemGenericAllocationHandle_t handle{};
};

}  // namespace rt
}  // namespace gsort

using namespace gsort::rt;

struct gsort_ctx {
    int rank = 0, nranks = 1, device = 0;
    hipStream_t stream = nullptr;
    // the distributed sorts' receive plan runs on stream2 behind the count exchange (ev_meta)
    // while the payload moves on stream; stream then waits for it (ev_plan)
    hipStream_t stream2 = nullptr;
    hipEvent_t ev_meta = nullptr, ev_plan = nullptr;
    Comm *comm = nullptr;
    std::string err;
    DevBuf slot[S_NSLOTS];
    DevBuf tcounts;  // K1/K2: per-tile digit counts -> in-group offsets (u32 [tiles][256])
    DevBuf gsum;     // K2: per-group digit prefixes (u64 [groups][256])
    int local_algo = GSORT_LOCAL_MSD;
    bool sample_balanced = false;  // gsort_set_sample_balanced
    int ref_compat = 0;            // gsort_set_ref_compat: 0 off, -1 P = nranks, else P
    // reference-compat radix: composite keys (two), values in flight, min/max + bad counter
    DevBuf m_ckey[2], m_vtmp[3], m_cmm;
    bool atomic_rank = false;  // LDS lane-order property verified on this device (create)
    // MSD scratch: segment plan/maps, child starts, work lists (u64 {start, len} pairs)
    DevBuf m_tpfx, m_gpfx, m_segmap, m_groupmap, m_cstart, m_next[2], m_local[kLocalClasses];
    uint64_t group16_nseg = 0;  // msd_sort(group16): level-2 segments (list m_next[0])
    // two-level plan front end (K1h / K12h / K3a): 16-bit histogram partials, wrap repairs,
    // level-2 cursors, K11 lists of the level-3 buckets; counters read while levels 3/2 run
    bool plan16 = true;
    DevBuf m_part, m_fix, m_cur, m_local3[kLocalClasses];
    DevBuf m_ccount, m_t3, m_cur3;  // K12a child counts, per-shard level-3 counts + totals, K3r cursors
    DevBuf m_tdesc;                 // K12c: K3a tile descriptors
    // sampled plan (K1e .. K11e): level-3 / level-2 region buffers, sample partials, plan
    // arrays, K3a tile descriptors, overflow scratch tile
    bool plan_est = true;   // GSORT_EST (default 1)
    bool plan_giant = true; // GSORT_GIANT (default 1): the one-dominant-child path
    double est_slack = 1.0; // GSORT_EST_SLACK (test hook: the sampling-error margin's scale)
    // GSORT_RECV_CX: receive buckets of K11g class >= recv_cx (1..4) and list 0 are counted by
    // K18c (default 4: buckets past 16 384 keys -- per 2^28 keys, 16 384-key buckets K11g
    // 0.72 / K18c 0.85 ms, 32 768-key K11g 1.01 / K18c 0.58 ms, tools/recv_probe.py); 5 = list
    // 0 only; -1 = the round-2 kernels (K11g classes, two-read K18)
    int recv_cx = 4;
    // GSORT_RECV_CB: K18c's bin width on the receive side, 8 (default since round 5: 64 KiB of
    // bins, two workgroups per CU; a bucket with >= 256 copies of one key redone with 16-bit
    // bins) or 16
    int recv_cb = 8;
    DevBuf m_fb;  // K18c (u8): the wrapped buckets' {h, len} entries
    // the previous packed receive sort's list counts (list 0, classes 1..4): the shape of the
    // next call's receive launches, queued before its counts are read (spec_recv_launch)
    uint32_t recv_hint[kLocalClasses + 1] = {};
    bool recv_hint_ok = false;
    // K15s (the receive plan's single-pass lookback scan): the allocation whose status words and
    // ticket were zeroed, and the per-call epoch its status words carry
    void *scan_clean = nullptr;
    uint32_t scan_epoch = 0;
    int ncu = 256;
    int last_plan = 0;      // gsort_last_plan: 0 exact, 1 sampled, 2 sampled then exact
    bool plan_trace = false; // GSORT_PLAN_TRACE: one stderr line per plan decision
    DevBuf m_ex, m_ey, m_epart, m_eplan, m_edesc, m_edump;
    DevBuf m_gplan;  // one dominant child: counts (65536 u64), starts (65537 u64), chunk bins
    bool est_busy = false;   // msd_sort_est is using m_ex / m_ey (not reclaimable)
    size_t scratch_bytes = 0;  // device bytes held by ensure()-managed scratch
    // K12p mailbox: pinned host memory the GPU writes the work-list counters into, then a
    // sequence number (polled by the host: no copy or event on the stream)
    uint64_t *h_mail = nullptr, *d_mail = nullptr;
    uint64_t mail_seq = 0;
    void *fix_clean = nullptr;  // m_fix.p when it is known to be zero (K12a clears it after use)
    DevBuf m_split;  // radix select thresholds + counts of the distributed radix
    DevBuf m_rpos, m_bsize;  // receive side: run bucket bounds (P x 65537), bucket size/start
    DevBuf m_bseg, m_blist;  // boundary groups of the distributed radix: scratch, K11 list
    DevBuf m_gb, m_pack, m_meta, m_g16;  // packed exchange: bucket bounds, low 16 bits, counts
    // device small area: [0, 8K) hist4 (4x256 u64) | [8K, 10K) pass digit totals (256 u64) |
    // [10K, 12K) pass digit bases (256 u64) | [20K, 256K) plans / samples / routing tables
    DevBuf small;               // kSmallBytes; d_small aliases small.p
    char *d_small = nullptr;
    char *h_small = nullptr;  // pinned mirror
    std::map<void *, DevBuf> user_bufs;  // gsort_device_alloc (guarded with GSORT_CANARY)
    std::vector<int32_t> splitters;
    std::vector<uint64_t> bucket_counts;
    // timing
    bool timing = false;
    std::vector<hipEvent_t> ev_pool;
    size_t ev_used = 0;
    struct Span { int phase; hipEvent_t a, b; };
    std::vector<Span> spans;
    LaunchTimer timer;  // kernel-attached timing events (tic / toc)
    // host staging of the drop-in path (gsort_scatter_from_root / gsort_gather_to_root):
    // kStageBufs pinned chunks, allocated on first use
    char *h_stage[4] = {nullptr, nullptr, nullptr, nullptr};
    hipEvent_t ev_stage[4] = {nullptr, nullptr, nullptr, nullptr};
};

namespace gsort {
namespace rt {

// [12K, 12K+96): MSD work-list counters, {entries, keys, longest} for the next-level list and
// the K11 class lists; [12K+128, 12K+144): a one-entry list for a single-bucket sort;
// [12K+256, 12K+352): the counters of the level-3 K11 lists of the two-level plan
constexpr size_t OFF_HIST = 0, OFF_TOT = 8192, OFF_BASES = 10240, OFF_CTR = 12288,
                 OFF_ONE = 12416, OFF_CTR3 = 12544, OFF_PLAN = 20480;
constexpr size_t OFF_FLAGS = 12408;  // K12b's trivial-level word, inside the published range
constexpr size_t OFF_MINMAX = 12480;  // the offset retry's exact min / max (2 int32)
constexpr size_t OFF_FBCTR = 12800;   // K18c (u8): the count of wrapped buckets (u32)
// K1m result (3 u64, word 3 spare), then K1g's counters from word 4: ctr[0] (cold keys of all
// workgroups) + one per K1g workgroup (1 + kH16Blocks u64; static_assert in giant_sort)
constexpr size_t OFF_GIANT = 16384;

constexpr size_t kCtrBytes = 3 * 8 * (kLocalClasses + 1);
static_assert(OFF_CTR + kCtrBytes <= OFF_FLAGS && OFF_FLAGS + 4 <= OFF_ONE, "counter area");

// ---- shared helpers (gsort_runtime.cpp) ----
gsort_status check_all_guards(gsort_ctx *c, const char *where);
void fault_info(gsort_ctx *c, const std::string &what);
gsort_status set_err(gsort_ctx *c, gsort_status st, const std::string &msg);
gsort_status comm_try(gsort_ctx *c, gsort_status st);
bool reclaim_regions(gsort_ctx *c, const DevBuf &asking);
gsort_status ensure(gsort_ctx *c, DevBuf &b, size_t bytes);
hipEvent_t tic(gsort_ctx *c);
void toc(gsort_ctx *c, int phase, hipEvent_t a);
hipEvent_t tic_rec(gsort_ctx *c);
void toc_rec(gsort_ctx *c, int phase, hipEvent_t a);
gsort_status ensure_pass_scratch(gsort_ctx *c, uint64_t n);
uint32_t *d_tcounts(gsort_ctx *c);
uint64_t *d_gsum(gsort_ctx *c);
gsort_status count_tiles(gsort_ctx *c, const uint32_t *src, uint64_t n, int digit, bool flip);
gsort_status scan_and_scatter(gsort_ctx *c, const uint32_t *src, uint32_t *dst, uint64_t n,
    int digit, bool flip_in, bool flip_out, const uint32_t *vin = nullptr,
    uint32_t *vout = nullptr);
gsort_status ensure_list(gsort_ctx *c, DevBuf &b, uint64_t entries);
bool check_mode();
gsort_status check_bounds(gsort_ctx *c, const uint64_t *d, size_t m, uint64_t last,
    const char *what);
gsort_status read_counters(gsort_ctx *c, uint64_t *h);
// K12p's mailbox: wait for sequence number seq (the counters behind it are then visible); a
// stream `s` (default: the context's) that goes idle without it, or fails, is an error
gsort_status wait_mail(gsort_ctx *c, uint64_t seq, hipStream_t s = nullptr);
WorkLists work_lists(gsort_ctx *c, int next);
gsort_status check_ctx(gsort_ctx *c);
template <class T>
T *slot_ptr(gsort_ctx *c, Slot s) { return reinterpret_cast<T *>(c->slot[s].p); }

// ---- the one-rank sorts (gsort_local.cpp) ----
gsort_status lsd_sort(gsort_ctx *c, const uint32_t *in, uint64_t n, uint32_t *out, uint32_t *tmp,
    int *passes_run);
gsort_status msd_levels(gsort_ctx *c, int L, uint32_t *cur, uint32_t *out, uint32_t *tmp,
    int cur_list, uint64_t *h, gsort_stats *stats, int *levels, int last_level = 0,
    uint16_t *out16 = nullptr, bool flip_first = false);
gsort_status msd_sort(gsort_ctx *c, const uint32_t *in, uint64_t n, uint32_t *out, uint32_t *tmp,
    gsort_stats *stats, bool group16 = false, uint16_t *out16 = nullptr, uint64_t *gb = nullptr,
    bool allow_est = false, bool allow_giant = true);
gsort_status local_sort(gsort_ctx *c, const uint32_t *in, uint64_t n, uint32_t *out, uint32_t *tmp,
    int *passes_run, gsort_stats *stats = nullptr, bool allow_est = false);
gsort_status giant_sort(gsort_ctx *c, const uint32_t *in, uint64_t n, uint32_t *out,
    uint32_t child, gsort_stats *stats, bool *ok);

// ---- the distributed sorts (gsort_dist.cpp) ----
gsort_status allgather_u64(gsort_ctx *c, uint64_t v, std::vector<uint64_t> &out);
void block_of(uint64_t N, int P, int r, uint64_t *B, uint64_t *len);
gsort_status radix_dist_exact(gsort_ctx *c, const int32_t *d_keys, uint64_t n_in, int32_t **d_out,
    uint64_t *n_out, gsort_stats *stats);
gsort_status radix_dist(gsort_ctx *c, const int32_t *d_keys, uint64_t n_in, int32_t **d_out,
    uint64_t *n_out, gsort_stats *stats, const uint32_t *sort_keys = nullptr);
gsort_status radix_compat(gsort_ctx *c, const int32_t *d_keys, uint64_t n_in, int32_t **d_out,
    uint64_t *n_out, gsort_stats *stats);
gsort_status sample_dist(gsort_ctx *c, const int32_t *d_keys, uint64_t n_in, int32_t **d_out,
    uint64_t *n_out, gsort_stats *stats);

}  // namespace rt
}  // namespace gsort

// Every HIP call of the runtime goes through hip_op (GSORT_SERIAL: serialized + device-synced,
// then with GSORT_CANARY the guards of all contexts are checked after the call).
#define HIP_TRY(ctx, expr)                                                                   \
    do {                                                                                     \
        if (trace_mode()) trace_op((ctx)->rank, #expr);                                      \
        hipError_t e_ = hip_op([&]() -> hipError_t { return (expr); });                      \
        if (e_ != hipSuccess && trace_mode()) trace_dump(#expr);                             \
        if (e_ != hipSuccess) fault_info(ctx, #expr);                                        \
        if (e_ != hipSuccess)                                                                \
            return set_err(ctx, GSORT_EHIP, std::string(#expr) + ": " +                      \
                                                hipGetErrorString(e_) + " (rank " +          \
                                                std::to_string((ctx)->rank) + ")");         \
        if (serial_mode() && canary_mode()) {                                                \
            gsort_status g_ = check_all_guards(ctx, #expr);                                  \
            if (g_ != GSORT_OK) return g_;                                                   \
        }                                                                                    \
    } while (0)

#define ST_TRY(expr)                         \
    do {                                     \
        gsort_status s_ = (expr);            \
        if (s_ != GSORT_OK) return s_;       \
    } while (0)

