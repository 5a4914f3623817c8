// gsort_runtime.cpp -- the C-ABI of libgsort (include/gsort.h): contexts, device memory,
// timing, diagnostics and drop-in staging; the sorts themselves are in gsort_local.cpp (one
// rank) and gsort_dist.cpp (P ranks), sharing the context through gsort_ctx.h.
//
// Reference being replaced: sort() of mpi_radix_sort.c:60-205 and mpi_sample_sort.c:28-218.
// Data stays resident on each rank's GPU for the whole sort; the host only moves per-pass
// digit counts (a few KB) to size the RCCL messages, which need host-side counts.
#include "gsort_ctx.h"

namespace gsort {
namespace rt {

gsort_status set_err(gsort_ctx *c, gsort_status st, const std::string &msg) {
    if (c) c->err = msg;
    return st;
}

// Diagnostic modes (gsort_debug.h).  GSORT_CANARY checks every live context's guards, so the
// contexts register themselves here.
std::mutex g_ctx_mu;
std::set<gsort_ctx *> g_ctxs;
gsort_status check_all_guards(gsort_ctx *c, const char *where);

gsort_status comm_try(gsort_ctx *c, gsort_status st) {
    if (st != GSORT_OK) c->err = c->comm->err + " (rank " + std::to_string(c->rank) + ")";
    return st;
}

// GSORT_ALLOC_LIMIT=bytes (diagnostics): refuse any larger scratch allocation, naming the buffer;
// GSORT_ALLOC_TOTAL=bytes: refuse a scratch allocation that would take the context's scratch
// past that many bytes (a device with less free memory, for tests)
std::string buf_name(gsort_ctx *c, const DevBuf &b);

// Device allocation of `want` usable bytes (+ guards with GSORT_CANARY).  Returns the HIP error.
// Allocation granularity: 4 KiB (256 B with GSORT_EFENCE, so buffers end at the unmapped page).
bool efence_mode();
size_t alloc_align() { return efence_mode() ? 256 : 4096; }

// GSORT_EFENCE=1 (diagnostics): every buffer ends flush against an unmapped VA page (HIP VMM:
// reserve a range with a free granule on each side, map physical memory only in the middle,
// place the buffer at the end of the mapping), so any read or write past a buffer's end faults
// at once; with GSORT_SERIAL the failing operation is then named.
bool efence_mode() {
    static const bool on = getenv("GSORT_EFENCE") && atoi(getenv("GSORT_EFENCE"));
    return on;
}

hipError_t efence_malloc(DevBuf &b, size_t want) {
    int dev = 0;
    hipError_t e = hipGetDevice(&dev);
    if (e != hipSuccess) return e;
    hipMemAllocationProp prop{};
    prop.type = hipMemAllocationTypePinned;
    prop.location.type = hipMemLocationTypeDevice;
    prop.location.id = dev;
    size_t gran = 0;
    e = hipMemGetAllocationGranularity(&gran, &prop, hipMemAllocationGranularityMinimum);
    if (e != hipSuccess) return e;
    static bool said = false;
    if (!said) { said = true; fprintf(stderr, "GSORT_EFENCE: granularity %zu\n", gran); }
    static const size_t slack = getenv("GSORT_EFENCE_SLACK")
                                    ? (size_t)strtoull(getenv("GSORT_EFENCE_SLACK"), nullptr, 0)
                                    : 0;
    const size_t msize = (want + slack + gran - 1) / gran * gran, va_bytes = msize + 2 * gran;
    void *va = nullptr;
    e = hipMemAddressReserve(&va, va_bytes, gran, nullptr, 0);
    if (e != hipSuccess) return e;
    hipMemGenericAllocationHandle_t h{};
    e = hipMemCreate(&h, msize, &prop, 0);
    if (e != hipSuccess) { (void)hipMemAddressFree(va, va_bytes); return e; }
    char *m = static_cast<char *>(va) + gran;
    e = hipMemMap(m, msize, 0, h, 0);
    if (e == hipSuccess) {
        hipMemAccessDesc acc{};
        acc.location.type = hipMemLocationTypeDevice;
        acc.location.id = dev;
        acc.flags = hipMemAccessFlagsProtReadWrite;
        e = hipMemSetAccess(m, msize, &acc, 1);
        if (e != hipSuccess) (void)hipMemUnmap(m, msize);
    }
    if (e != hipSuccess) {
        (void)hipMemRelease(h);
        (void)hipMemAddressFree(va, va_bytes);
        return e;
    }
    b.base = va;
    b.va_bytes = va_bytes;
    b.map_bytes = msize;
    b.handle = h;
    b.p = m + msize - want - slack;  // the buffer ends at the unmapped granule (- slack)
    b.cap = want;
    return hipSuccess;
}

// The freed VA range stays reserved (never handed out again): re-mapping a just-unmapped range
// to new physical pages gave wrong results on MI355X (a buffer grown mid-sort read stale
// contents), an artifact of this diagnostic mode, not of the sort.  VA space is plentiful.
hipError_t efence_free(DevBuf &b) {
    char *m = static_cast<char *>(b.base) + (b.va_bytes - b.map_bytes) / 2;
    hipError_t e = hipDeviceSynchronize();
    if (e == hipSuccess) e = hipMemUnmap(m, b.map_bytes);
    if (e == hipSuccess) e = hipMemRelease(b.handle);
    return e;
}

// With GSORT_CANARY every change of a buffer happens under serial_mutex, so the guard checks
// of other threads never see a half-updated DevBuf.
// GSORT_EFENCE_ONLY=name,name,...: fence only the named buffers (bisecting a fault)
bool efence_for(const std::string &name) {
    const char *only = getenv("GSORT_EFENCE_ONLY");
    if (!only || !*only) return true;
    const std::string list = std::string(",") + only + ",";
    return list.find("," + name + ",") != std::string::npos;
}

hipError_t dev_malloc(DevBuf &b, size_t want, const std::string &name = "") {
    if (efence_mode() && efence_for(name)) {
        std::lock_guard<std::mutex> lk(serial_mutex());
        b.p = b.base = nullptr;
        b.cap = 0;
        return efence_malloc(b, want);
    }
    if (!canary_mode()) {
        b.p = b.base = nullptr;
        b.cap = 0;
        hipError_t e = hip_op([&] { return hipMalloc(&b.base, want); });
        if (e != hipSuccess) { b.base = nullptr; return e; }
        b.p = b.base;
        b.cap = want;
        return hipSuccess;
    }
    std::lock_guard<std::mutex> lk(serial_mutex());
    void *base = nullptr;
    hipError_t e = hipMalloc(&base, want + 2 * kGuardBytes);
    if (e != hipSuccess) return e;
    char *g = static_cast<char *>(base);
    e = hipMemset(g, kGuardByte, kGuardBytes);
    if (e == hipSuccess) e = hipMemset(g + kGuardBytes + want, kGuardByte, kGuardBytes);
    if (e == hipSuccess) e = hipDeviceSynchronize();
    if (e != hipSuccess) { (void)hipFree(base); return e; }
    b.base = base;
    b.p = g + kGuardBytes;
    b.cap = want;
    return hipSuccess;
}

// GSORT_FAULTINFO=1: the last kFreedRing freed device ranges, printed with every live buffer
// when the first HIP error is seen (where a faulting address lands: past a live buffer, in a
// freed one, or elsewhere)
constexpr size_t kFreedRing = 512;
std::mutex g_freed_mu;
std::vector<std::pair<uintptr_t, size_t>> g_freed(kFreedRing);
size_t g_freed_n = 0;
bool faultinfo_mode() {
    static const bool on = getenv("GSORT_FAULTINFO") && atoi(getenv("GSORT_FAULTINFO"));
    return on;
}

hipError_t dev_free(DevBuf &b) {
    if (faultinfo_mode() && b.base) {
        std::lock_guard<std::mutex> lk(g_freed_mu);
        g_freed[g_freed_n++ % kFreedRing] = {(uintptr_t)b.p, b.cap};
    }
    hipError_t e = hipSuccess;
    if (efence_mode() && b.va_bytes) {
        std::lock_guard<std::mutex> lk(serial_mutex());
        if (b.base) e = efence_free(b);
        b.p = b.base = nullptr;
        b.cap = b.va_bytes = b.map_bytes = 0;
        return e;
    }
    if (canary_mode()) {
        std::lock_guard<std::mutex> lk(serial_mutex());
        if (b.base) e = hipFree(b.base);
        b.p = b.base = nullptr;
        b.cap = 0;
        return e;
    }
    if (b.base) e = hip_op([&] { return hipFree(b.base); });
    b.p = b.base = nullptr;
    b.cap = 0;
    return e;
}

void for_each_buf_fwd(gsort_ctx *c, void (*f)(void *, const std::string &, DevBuf &), void *u);

// GSORT_FAULTINFO: print every live buffer of every context and the recently freed ranges
void fault_info(gsort_ctx *c, const std::string &what) {
    if (!faultinfo_mode()) return;
    static std::atomic<bool> done{false};
    if (done.exchange(true)) return;
    fprintf(stderr, "GSORT_FAULTINFO: first HIP error (rank %d): %s\n", c->rank, what.c_str());
    std::lock_guard<std::mutex> lk(g_ctx_mu);
    for (gsort_ctx *o : g_ctxs)
        for_each_buf_fwd(o, [](void *u, const std::string &nm, DevBuf &b) {
            if (b.p)
                fprintf(stderr, "  live r%d %-10s [%#zx, %#zx) %zu B\n",
                        static_cast<gsort_ctx *>(u)->rank, nm.c_str(), (size_t)(uintptr_t)b.p,
                        (size_t)((uintptr_t)b.p + b.cap), b.cap);
        }, o);
    std::lock_guard<std::mutex> lk2(g_freed_mu);
    const size_t m = std::min(g_freed_n, kFreedRing);
    for (size_t i = g_freed_n - m; i < g_freed_n; ++i) {
        const auto &f = g_freed[i % kFreedRing];
        fprintf(stderr, "  freed #%zu [%#zx, %#zx) %zu B\n", i, (size_t)f.first,
                (size_t)(f.first + f.second), f.second);
    }
    fflush(stderr);
}

// An allocation failure is GSORT_ENOMEM only when HIP says out-of-memory: after an earlier
// asynchronous kernel fault every hipMalloc fails with that sticky error, which must surface
// as what it is (GSORT_EHIP + the HIP message), not as a bogus out-of-memory.
gsort_status alloc_err(gsort_ctx *c, hipError_t e, size_t want, const std::string &what) {
    (void)hipGetLastError();
    if (trace_mode()) trace_dump("hipMalloc failed");
    const std::string msg = "hipMalloc of " + std::to_string(want) + " bytes for " + what +
                            " (rank " + std::to_string(c->rank) + "): " + hipGetErrorString(e);
    if (e != hipErrorOutOfMemory) fault_info(c, msg);
    return set_err(c, e == hipErrorOutOfMemory ? GSORT_ENOMEM : GSORT_EHIP, msg);
}

// The sampled plan's region buffers (~2.9x the block) stay allocated between sorts; when some
// other scratch allocation finds no room they are dropped (and re-made by the next sampled
// sort), unless the plan is using them right now.
bool reclaim_regions(gsort_ctx *c, const DevBuf &asking) {
    if (c->est_busy) return false;
    bool freed = false;
    for (DevBuf *r : {&c->m_ex, &c->m_ey}) {
        if (r == &asking || !r->p) continue;
        c->scratch_bytes -= std::min(c->scratch_bytes, r->cap);
        (void)dev_free(*r);
        freed = true;
    }
    return freed;
}

gsort_status ensure(gsort_ctx *c, DevBuf &b, size_t bytes) {
    if (bytes <= b.cap) return GSORT_OK;
    static const unsigned long long limit =
        getenv("GSORT_ALLOC_LIMIT") ? strtoull(getenv("GSORT_ALLOC_LIMIT"), nullptr, 0) : 0ull;
    static const unsigned long long total =
        getenv("GSORT_ALLOC_TOTAL") ? strtoull(getenv("GSORT_ALLOC_TOTAL"), nullptr, 0) : 0ull;
    if (limit && bytes > limit)
        return set_err(c, GSORT_ENOMEM, "allocation of " + std::to_string(bytes) +
                                            " bytes for " + buf_name(c, b) +
                                            " over GSORT_ALLOC_LIMIT (rank " +
                                            std::to_string(c->rank) + ")");
    c->scratch_bytes -= std::min(c->scratch_bytes, b.cap);
    // buffers known to hold zeros (K12a's fix[], K15s's status words and ticket) are no longer
    // known to once replaced: a new allocation may come back at the same address
    if (b.p && c->fix_clean == b.p) c->fix_clean = nullptr;
    if (b.p && c->scan_clean == b.p) c->scan_clean = nullptr;
    hipError_t e = dev_free(b);
    if (e != hipSuccess)
        return set_err(c, GSORT_EHIP, "hipFree of " + buf_name(c, b) + " (rank " +
                                          std::to_string(c->rank) + "): " + hipGetErrorString(e));
    const size_t want = (bytes + alloc_align() - 1) & ~(alloc_align() - 1);
    for (int attempt = 0;; ++attempt) {
        const bool refused = total && c->scratch_bytes + want > total;
        if (!refused) {
            e = dev_malloc(b, want, buf_name(c, b));
            if (e == hipSuccess) {
                c->scratch_bytes += want;
                return GSORT_OK;
            }
        }
        if ((refused || e == hipErrorOutOfMemory) && attempt == 0 && reclaim_regions(c, b)) {
            (void)hipGetLastError();
            continue;
        }
        if (refused)
            return set_err(c, GSORT_ENOMEM, "allocation of " + std::to_string(want) +
                                                " bytes for " + buf_name(c, b) +
                                                " over GSORT_ALLOC_TOTAL (rank " +
                                                std::to_string(c->rank) + ")");
        return alloc_err(c, e, want, buf_name(c, b));
    }
}


// ---- timing ---------------------------------------------------------------------------
// Timing events release at device scope (hipEventDisableSystemFence): they only feed
// hipEventElapsedTime, and a default event's system-scope release at the end of every timed
// dispatch cost a 2^28-key sort 12 us (1.339 -> 1.351 ms, tools/event_cost.py).  A runtime that
// refuses the flag gets default events.
hipEvent_t next_event(gsort_ctx *c) {
    if (c->ev_used == c->ev_pool.size()) {
        hipEvent_t e;
        if (hipEventCreateWithFlags(&e, hipEventDisableSystemFence) != hipSuccess &&
            hipEventCreateWithFlags(&e, 0u) != hipSuccess)
            return nullptr;
        c->ev_pool.push_back(e);
    }
    return c->ev_pool[c->ev_used++];
}
// Phase spans of gsort_stats.  tic/toc time the kernels launched between them with the stop
// events the kernels' own dispatches carry (LaunchTimer, gsort_kernels.h): a span runs from
// the stop of the kernel before it (or, first in a call, an event recorded while the stream
// is idle) to the stop of its last kernel, so it includes one launch gap (~1 us) and the
// stream carries no marker packets between kernels; a span without a kernel is dropped.
// (A hipEventRecord between two kernels left ~5-8 us of idle, an attached start event ~5 us:
// tools/experiments/launch_gap.hip.)  Spans whose work is not a library kernel (RCCL
// collectives, copies) use tic_rec / toc_rec, which record both events on the stream.
hipEvent_t timer_make(void *u) { return next_event(static_cast<gsort_ctx *>(u)); }
hipEvent_t tic(gsort_ctx *c) {
    if (!c->timing) return nullptr;
    if (!c->timer.last_stop) {
        hipEvent_t e = next_event(c);
        if (!e || hipEventRecord(e, c->stream) != hipSuccess) return nullptr;
        c->timer.last_stop = e;
    }
    return c->timer.last_stop;
}
void toc(gsort_ctx *c, int phase, hipEvent_t a) {
    if (!c->timing || !a || c->timer.last_stop == a) return;
    c->spans.push_back({phase, a, c->timer.last_stop});
}
hipEvent_t tic_rec(gsort_ctx *c) {
    if (!c->timing) return nullptr;
    hipEvent_t e = next_event(c);
    if (e && hipEventRecord(e, c->stream) != hipSuccess) e = nullptr;
    return e;
}
void toc_rec(gsort_ctx *c, int phase, hipEvent_t a) {
    if (!c->timing || !a) return;
    hipEvent_t b = next_event(c);
    if (!b || hipEventRecord(b, c->stream) != hipSuccess) return;
    c->spans.push_back({phase, a, b});
    c->timer.last_stop = b;  // the next kernel span starts here
}
void timing_begin(gsort_ctx *c, gsort_stats *st) {
    c->timing = st != nullptr;
    c->ev_used = 0;
    c->spans.clear();
    c->timer.last_stop = nullptr;
    c->timer.make = timer_make;
    c->timer.u = c;
    set_launch_timer(st ? &c->timer : nullptr);
    if (st) memset(st, 0, sizeof(*st));
}
// Clears this thread's launch timer when a timed call returns (on every path).
struct TimerScope {
    ~TimerScope() { set_launch_timer(nullptr); }
};
void timing_finish(gsort_ctx *c, gsort_stats *st) {
    if (!st) return;
    for (auto &sp : c->spans) {
        float ms = 0.f;
        if (hipEventElapsedTime(&ms, sp.a, sp.b) != hipSuccess) continue;
        switch (sp.phase) {
            case PH_COUNT: st->ms_hist += ms; st->ms_local_sort += ms; break;
            case PH_PASS0: case PH_PASS1: case PH_PASS2: case PH_PASS3:
                st->ms_pass[sp.phase - PH_PASS0] += ms; st->ms_local_sort += ms; break;
            case PH_EXCH: st->ms_exchange += ms; break;
            case PH_PLACE: st->ms_place += ms; break;
            case PH_SAMPLE: st->ms_sample += ms; break;
            case PH_MERGE: st->ms_merge += ms; break;
            case PH_TOTAL: st->ms_total += ms; break;
            case PH_LEVEL3: case PH_LEVEL2: case PH_LEVEL1: case PH_LEVEL0:
                st->ms_level[sp.phase - PH_LEVEL3] += ms; st->ms_local_sort += ms; break;
            case PH_BUCKET: st->ms_bucket_sort += ms; st->ms_local_sort += ms; break;
        }
    }
    c->timing = false;
}

gsort_status ensure_pass_scratch(gsort_ctx *c, uint64_t n) {
    ST_TRY(ensure(c, c->tcounts, (size_t)std::max<uint64_t>(sweep_tiles(n), 1) * kRadix * 4));
    ST_TRY(ensure(c, c->gsum, (size_t)std::max<uint64_t>(scan_groups(n), 1) * kRadix * 8));
    return GSORT_OK;
}

uint32_t *d_tcounts(gsort_ctx *c) { return reinterpret_cast<uint32_t *>(c->tcounts.p); }
uint64_t *d_gsum(gsort_ctx *c) { return reinterpret_cast<uint64_t *>(c->gsum.p); }

// K1 (digit counts per tile) for digit p of src; skipped when the caller already has them.
gsort_status count_tiles(gsort_ctx *c, const uint32_t *src, uint64_t n, int digit, bool flip) {
    hipEvent_t t = tic(c);
    HIP_TRY(c, launch_tile_counts(src, n, 8 * digit, flip, d_tcounts(c), nullptr, c->stream));
    toc(c, PH_COUNT, t);
    return GSORT_OK;
}

// K2 + K3: one stable LSD pass src -> dst over `digit`, tile counts already in tcounts.
// The pass's 256 digit counts are left in the small area at OFF_TOT (used for routing).
gsort_status scan_and_scatter(gsort_ctx *c, const uint32_t *src, uint32_t *dst, uint64_t n,
                              int digit, bool flip_in, bool flip_out,
                              const uint32_t *vin, uint32_t *vout) {
    uint64_t *totals = reinterpret_cast<uint64_t *>(c->d_small + OFF_TOT);
    uint64_t *bases = reinterpret_cast<uint64_t *>(c->d_small + OFF_BASES);
    hipEvent_t t = tic(c);
    HIP_TRY(c, launch_scan_tiles(d_tcounts(c), n, d_gsum(c), totals, bases, c->stream));
    toc(c, PH_COUNT, t);
    t = tic(c);
    HIP_TRY(c, launch_scatter(src, dst, n, 8 * digit, d_tcounts(c), d_gsum(c), bases, flip_in,
                              flip_out, c->stream, vin, vout));
    toc(c, PH_PASS0 + digit, t);
    return GSORT_OK;
}

gsort_status reset_call(gsort_ctx *c) {
    HIP_TRY(c, hipSetDevice(c->device));
    return GSORT_OK;
}

// ---- MSD local sort (gsort_kernels.hip, "MSD partition sort") --------------------------
// Level 3 partitions the whole input by its top digit (K1 + K2 + K3u, in -> tmp); every later
// level partitions the buckets still larger than kLocalMax by the next digit (alternating
// tmp -> out -> tmp -> out, same positions); every bucket of <= kLocalMax keys is finished by
// K11 in LDS and stored to out as int32.  The host reads two counters per level (a few us) to
// size the next launches.  Same reference hot loops as lsd_sort.

gsort_status ensure_list(gsort_ctx *c, DevBuf &b, uint64_t entries) {
    return ensure(c, b, (size_t)std::max<uint64_t>(entries, 1) * 16);
}

// Every device buffer a context owns, with its name (teardown, diagnostics).
template <class F>
void for_each_buf(gsort_ctx *c, F &&f) {
    const std::pair<const char *, DevBuf *> named[] = {
        {"tcounts", &c->tcounts}, {"gsum", &c->gsum}, {"m_tpfx", &c->m_tpfx},
        {"m_gpfx", &c->m_gpfx}, {"m_segmap", &c->m_segmap}, {"m_groupmap", &c->m_groupmap},
        {"m_cstart", &c->m_cstart}, {"m_next0", &c->m_next[0]}, {"m_next1", &c->m_next[1]},
        {"m_part", &c->m_part}, {"m_fix", &c->m_fix}, {"m_cur", &c->m_cur},
        {"m_ccount", &c->m_ccount}, {"m_t3", &c->m_t3}, {"m_cur3", &c->m_cur3},
        {"m_tdesc", &c->m_tdesc}, {"m_ex", &c->m_ex}, {"m_ey", &c->m_ey},
        {"m_epart", &c->m_epart}, {"m_eplan", &c->m_eplan}, {"m_edesc", &c->m_edesc},
        {"m_edump", &c->m_edump}, {"m_gplan", &c->m_gplan}, {"m_fb", &c->m_fb},
        {"m_split", &c->m_split}, {"m_rpos", &c->m_rpos}, {"m_bsize", &c->m_bsize},
        {"m_bseg", &c->m_bseg}, {"m_blist", &c->m_blist}, {"m_gb", &c->m_gb},
        {"m_pack", &c->m_pack}, {"m_meta", &c->m_meta}, {"m_g16", &c->m_g16},
        {"m_ckey0", &c->m_ckey[0]}, {"m_ckey1", &c->m_ckey[1]}, {"m_vtmp0", &c->m_vtmp[0]},
        {"m_vtmp1", &c->m_vtmp[1]}, {"m_vtmp2", &c->m_vtmp[2]}, {"m_cmm", &c->m_cmm},
        {"small", &c->small}};
    for (const auto &nb : named) f(std::string(nb.first), *nb.second);
    static const char *slot_names[S_NSLOTS] = {"S_TMP",  "S_OUT", "S_CUR",  "S_SORTED",
                                               "S_RECV", "S_IN",  "S_STAGE"};
    for (int i = 0; i < S_NSLOTS; ++i) f(std::string(slot_names[i]), c->slot[i]);
    for (int k = 0; k < kLocalClasses; ++k) {
        f("m_local" + std::to_string(k), c->m_local[k]);
        f("m_local3_" + std::to_string(k), c->m_local3[k]);
    }
    for (auto &ub : c->user_bufs) f(std::string("user"), ub.second);
}

void for_each_buf_fwd(gsort_ctx *c, void (*f)(void *, const std::string &, DevBuf &), void *u) {
    for_each_buf(c, [&](const std::string &nm, DevBuf &b) { f(u, nm, b); });
}

std::string buf_name(gsort_ctx *c, const DevBuf &b) {
    std::string name = "?";
    for_each_buf(c, [&](const std::string &nm, DevBuf &x) { if (&x == &b) name = nm; });
    return name;
}

// GSORT_CANARY: read back both guards of every buffer of every live context; the first
// overwritten byte fails the call with the buffer, the offset and the operation just run.
gsort_status check_ctx_guards(gsort_ctx *owner, gsort_ctx *c, const char *where) {
    std::vector<unsigned char> h(kGuardBytes);
    gsort_status st = GSORT_OK;
    for_each_buf(c, [&](const std::string &nm, DevBuf &b) {
        if (st != GSORT_OK || !b.base) return;
        for (int side = 0; side < 2 && st == GSORT_OK; ++side) {
            const char *g = static_cast<const char *>(b.base) +
                            (side ? kGuardBytes + b.cap : 0);
            if (hipMemcpy(h.data(), g, kGuardBytes, hipMemcpyDeviceToHost) != hipSuccess) {
                st = set_err(owner, GSORT_EHIP, "GSORT_CANARY: guard read failed");
                return;
            }
            for (size_t i = 0; i < kGuardBytes; ++i)
                if (h[i] != kGuardByte) {
                    const long long off = side ? (long long)(b.cap + i)
                                               : -(long long)(kGuardBytes - i);
                    st = set_err(owner, GSORT_EINVAL,
                                 "GSORT_CANARY: rank " + std::to_string(c->rank) + " buffer " + nm +
                                     " (" + std::to_string(b.cap) + " bytes) overwritten at byte " +
                                     std::to_string(off) + " after " + where + " (called by rank " +
                                     std::to_string(owner->rank) + ")");
                    return;
                }
        }
    });
    return st;
}

gsort_status check_all_guards(gsort_ctx *c, const char *where) {
    if (!canary_mode()) return GSORT_OK;
    std::lock_guard<std::mutex> lk(serial_mutex());
    if (hipDeviceSynchronize() != hipSuccess)
        return set_err(c, GSORT_EHIP, std::string("GSORT_CANARY: device fault before ") + where);
    std::lock_guard<std::mutex> lk2(g_ctx_mu);
    for (gsort_ctx *o : g_ctxs) ST_TRY(check_ctx_guards(c, o, where));
    return GSORT_OK;
}

// GSORT_CHECK=1 (diagnostics): host-side invariant checks between the distributed phases, so
// a broken count fails the call with a message instead of sizing buffers or launches from it
bool check_mode() {
    static const bool on = getenv("GSORT_CHECK") && atoi(getenv("GSORT_CHECK"));
    return on;
}

gsort_status check_bounds(gsort_ctx *c, const uint64_t *d, size_t m, uint64_t last,
                          const char *what) {
    std::vector<uint64_t> v(m);
    HIP_TRY(c, hipStreamSynchronize(c->stream));
    HIP_TRY(c, hipMemcpy(v.data(), d, m * 8, hipMemcpyDeviceToHost));
    for (size_t i = 1; i < m; ++i)
        if (v[i] < v[i - 1])
            return set_err(c, GSORT_EINVAL, std::string("GSORT_CHECK ") + what + ": decreases at " +
                                                std::to_string(i) + " (rank " +
                                                std::to_string(c->rank) + ")");
    if (v[0] != 0 || v[m - 1] != last)
        return set_err(c, GSORT_EINVAL, std::string("GSORT_CHECK ") + what + ": ends " +
                                            std::to_string(v[0]) + ".." +
                                            std::to_string(v[m - 1]) + ", want 0.." +
                                            std::to_string(last) + " (rank " +
                                            std::to_string(c->rank) + ")");
    return GSORT_OK;
}

gsort_status read_counters(gsort_ctx *c, uint64_t *h) {
    HIP_TRY(c, hipMemcpyAsync(c->h_small + OFF_CTR, c->d_small + OFF_CTR, kCtrBytes,
                              hipMemcpyDeviceToHost, c->stream));
    HIP_TRY(c, hipStreamSynchronize(c->stream));
    memcpy(h, c->h_small + OFF_CTR, kCtrBytes);
    return GSORT_OK;
}

WorkLists work_lists(gsort_ctx *c, int next) {
    WorkLists wl;
    wl.list[0] = reinterpret_cast<uint64_t *>(c->m_next[next].p);
    for (int k = 0; k < kLocalClasses; ++k)
        wl.list[k + 1] = reinterpret_cast<uint64_t *>(c->m_local[k].p);
    wl.ctr = reinterpret_cast<uint64_t *>(c->d_small + OFF_CTR);
    wl.force_next = false;
    return wl;
}

gsort_status check_ctx(gsort_ctx *c) { return c ? GSORT_OK : GSORT_EINVAL; }

gsort_status check_input(gsort_ctx *c, const int32_t *d_keys) {
    for (int s = 0; s < S_NSLOTS; ++s)
        if (s != S_IN && c->slot[s].p && (const void *)d_keys == c->slot[s].p)
            return set_err(c, GSORT_EINVAL, "d_keys aliases a context-owned scratch buffer");
    return GSORT_OK;
}

// The stable ranks of K11 (and K3) may come from LDS atomics only if the device serializes
// same-address lanes of one ds_add_rtn in lane order.  Checked once per process
// and device (the first context on it; VERDICT r3: not on every gsort_create) on xorshift
// digits at four densities; on any violation the ballot ranks are used instead.
std::mutex g_lds_order_mu;
int g_lds_order[64];  // per device: 0 unknown, 1 lane order holds, 2 violated

gsort_status check_lds_order(gsort_ctx *c) {
    std::lock_guard<std::mutex> lk(g_lds_order_mu);
    int *known = c->device >= 0 && c->device < 64 ? &g_lds_order[c->device] : nullptr;
    if (!known || !*known) {
        constexpr uint32_t kBlocks = 64, kN = kBlocks * 512 * 16;
        std::vector<uint32_t> h(kN);
        uint64_t x = 0x9E3779B97F4A7C15ull;
        for (auto &v : h) { x ^= x << 13; x ^= x >> 7; x ^= x << 17; v = (uint32_t)(x >> 32); }
        uint32_t *d = nullptr;
        HIP_TRY(c, hipMalloc(&d, kN * 4));
        uint64_t *bad = reinterpret_cast<uint64_t *>(c->d_small + OFF_PLAN);
        hipError_t e = hipMemcpyAsync(d, h.data(), kN * 4, hipMemcpyHostToDevice, c->stream);
        if (e == hipSuccess) e = hipMemsetAsync(bad, 0, 8, c->stream);
        for (uint32_t bins : {1u, 3u, 17u, 256u})
            if (e == hipSuccess) e = launch_lds_order_check(d, kBlocks, bins, bad, c->stream);
        uint64_t nbad = 1;
        if (e == hipSuccess) e = hipMemcpyAsync(&nbad, bad, 8, hipMemcpyDeviceToHost, c->stream);
        if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
        (void)hipFree(d);
        if (e != hipSuccess) return set_err(c, GSORT_EHIP, std::string("lds order check: ") +
                                                               hipGetErrorString(e));
        if (!known) {
            c->atomic_rank = nbad == 0 && !getenv("GSORT_BALLOT_RANK");
            return GSORT_OK;
        }
        *known = nbad == 0 ? 1 : 2;
    }
    c->atomic_rank = *known == 1 && !getenv("GSORT_BALLOT_RANK");
    return GSORT_OK;
}

gsort_status create_common(gsort_ctx *c, int hip_device) {
    if (hip_device < 0) {  // -1 - local_rank: pick the local rank's GPU
        int count = 0;
        HIP_TRY(c, hipGetDeviceCount(&count));
        if (count < 1) return set_err(c, GSORT_EHIP, "no HIP device visible");
        hip_device = (-1 - hip_device) % count;
    }
    c->device = hip_device;
    HIP_TRY(c, hipSetDevice(hip_device));
    HIP_TRY(c, hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking));
    // the receive plan's side stream and its two ordering events (packed_exchange_sort)
    HIP_TRY(c, hipStreamCreateWithFlags(&c->stream2, hipStreamNonBlocking));
    HIP_TRY(c, hipEventCreateWithFlags(&c->ev_meta, hipEventDisableTiming));
    HIP_TRY(c, hipEventCreateWithFlags(&c->ev_plan, hipEventDisableTiming));
    ST_TRY(ensure(c, c->small, kSmallBytes));
    c->d_small = static_cast<char *>(c->small.p);
    HIP_TRY(c, hipHostMalloc(&c->h_small, kSmallBytes, hipHostMallocDefault));
    HIP_TRY(c, hipHostMalloc(reinterpret_cast<void **>(&c->h_mail), kMailBytes,
                             hipHostMallocDefault));
    memset(c->h_mail, 0, kMailBytes);
    HIP_TRY(c, hipHostGetDevicePointer(reinterpret_cast<void **>(&c->d_mail), c->h_mail, 0));
    HIP_TRY(c, hipMemsetAsync(c->d_small, 0, kSmallBytes, c->stream));
    HIP_TRY(c, hipStreamSynchronize(c->stream));
    if (const char *e = getenv("GSORT_PLAN16")) c->plan16 = atoi(e) != 0;
    if (const char *e = getenv("GSORT_EST")) c->plan_est = atoi(e) != 0;
    if (const char *e = getenv("GSORT_GIANT")) c->plan_giant = atoi(e) != 0;
    if (const char *e = getenv("GSORT_RECV_CX")) c->recv_cx = atoi(e);
    if (const char *e = getenv("GSORT_RECV_CB")) c->recv_cb = atoi(e) == 16 ? 16 : 8;
    if (const char *e = getenv("GSORT_EST_SLACK")) c->est_slack = atof(e);
    if (const char *e = getenv("GSORT_PLAN_TRACE")) c->plan_trace = atoi(e) != 0;
    HIP_TRY(c, hipDeviceGetAttribute(&c->ncu, hipDeviceAttributeMultiprocessorCount, hip_device));
    {
        std::lock_guard<std::mutex> lk(g_ctx_mu);
        g_ctxs.insert(c);
    }
    return check_lds_order(c);
}

}  // namespace rt
}  // namespace gsort

// =========================================================================================
// C-ABI
// =========================================================================================
extern "C" {

const char *gsort_strerror(gsort_status st) {
    switch (st) {
        case GSORT_OK: return "ok";
        case GSORT_EINVAL: return "invalid argument";
        case GSORT_ENOMEM: return "out of memory";
        case GSORT_EHIP: return "HIP error";
        case GSORT_ERCCL: return "RCCL error";
        case GSORT_ENOSAMPLE: return "not enough keys for regular sampling";
        case GSORT_ECOMM: return "rank group error";
    }
    return "unknown status";
}

const char *gsort_last_error(const gsort_ctx *ctx) { return ctx ? ctx->err.c_str() : ""; }
int gsort_rank(const gsort_ctx *ctx) { return ctx ? ctx->rank : -1; }
int gsort_nranks(const gsort_ctx *ctx) { return ctx ? ctx->nranks : -1; }
size_t gsort_onesweep_tile(void) { return kSweepTile; }

// GSORT_FORCE_DIST=1: a one-rank context created with a uid (or in a group) still gets a
// communicator and runs the distributed algorithms -- the only way to drive the RCCL calls
// (init, all-gather, grouped send/recv to self, broadcast) on a one-GPU machine, since RCCL
// refuses two ranks on one device.  Test hook; the drop-in never sets it.
static bool force_dist() {
    const char *v = getenv("GSORT_FORCE_DIST");
    return v && v[0] == '1';
}

gsort_status gsort_get_uid(gsort_uid *out) {
    if (!out) return GSORT_EINVAL;
    return rccl_get_uid(out);
}

gsort_status gsort_get_uid_ipc(int nranks, gsort_uid *out) {
    if (!out) return GSORT_EINVAL;
    return ipc_get_uid(nranks, out);
}

gsort_status gsort_runtime_info(gsort_runtime_info_t *out) {
    if (!out) return GSORT_EINVAL;
    return runtime_info(out);
}

int gsort_visible_devices(void) {
    int count = 0;
    if (hipGetDeviceCount(&count) != hipSuccess) {
        (void)hipGetLastError();
        return 0;
    }
    return count;
}

gsort_status gsort_create(gsort_ctx **ctx, int rank, int nranks, int hip_device,
                          const gsort_uid *uid) {
    if (!ctx || nranks < 1 || rank < 0 || rank >= nranks || (nranks > 1 && !uid))
        return GSORT_EINVAL;
    *ctx = nullptr;
    gsort_ctx *c = new gsort_ctx();
    c->rank = rank;
    c->nranks = nranks;
    gsort_status st = create_common(c, hip_device);
    if (st == GSORT_OK && (nranks > 1 || (force_dist() && uid))) {
        std::string e;
        const bool ipc = is_ipc_uid(uid);
        c->comm = ipc ? make_ipc_comm(rank, nranks, uid, &e) : make_rccl_comm(rank, nranks, uid, &e);
        if (!c->comm) st = set_err(c, ipc ? GSORT_ECOMM : GSORT_ERCCL, e);
    }
    if (st != GSORT_OK) {
        fprintf(stderr, "gsort_create: %s\n", c->err.c_str());
        gsort_destroy(c);
        return st;
    }
    *ctx = c;
    return GSORT_OK;
}

gsort_status gsort_group_create(gsort_group **grp, int nranks) {
    if (!grp || nranks < 1) return GSORT_EINVAL;
    *grp = new gsort_group{group_state_create(nranks)};
    return GSORT_OK;
}

gsort_status gsort_group_destroy(gsort_group *grp) {
    if (!grp) return GSORT_EINVAL;
    group_state_destroy(grp->st);
    delete grp;
    return GSORT_OK;
}

gsort_status gsort_create_in_group(gsort_ctx **ctx, gsort_group *grp, int rank, int hip_device) {
    if (!ctx || !grp || rank < 0 || rank >= group_state_size(grp->st)) return GSORT_EINVAL;
    *ctx = nullptr;
    // one device per group: its collectives are ordered by device-scope events (ranks on
    // several GPUs are RCCL's job, one process per GPU)
    if (!group_state_join(grp->st, hip_device)) return GSORT_EINVAL;
    gsort_ctx *c = new gsort_ctx();
    c->rank = rank;
    c->nranks = group_state_size(grp->st);
    gsort_status st = create_common(c, hip_device);
    if (st != GSORT_OK) { gsort_destroy(c); return st; }
    if (c->nranks > 1 || force_dist()) c->comm = make_group_comm(grp->st, rank);
    *ctx = c;
    return GSORT_OK;
}

gsort_status gsort_destroy(gsort_ctx *c) {
    if (!c) return GSORT_EINVAL;
    // teardown: errors are not actionable here, so every status is deliberately dropped
    {
        std::lock_guard<std::mutex> lk(g_ctx_mu);
        g_ctxs.erase(c);
    }
    (void)hipSetDevice(c->device);
    if (c->stream) (void)hipStreamSynchronize(c->stream);
    delete c->comm;
    for_each_buf(c, [](const std::string &, DevBuf &b) { (void)dev_free(b); });
    c->d_small = nullptr;
    for (int b = 0; b < 4; ++b) {
        if (c->h_stage[b]) (void)hipHostFree(c->h_stage[b]);
        if (c->ev_stage[b]) (void)hipEventDestroy(c->ev_stage[b]);
    }
    if (c->h_small) (void)hipHostFree(c->h_small);
    if (c->h_mail) (void)hipHostFree(c->h_mail);
    for (auto e : c->ev_pool) (void)hipEventDestroy(e);
    if (c->stream) (void)hipStreamDestroy(c->stream);
    if (c->stream2) (void)hipStreamDestroy(c->stream2);
    if (c->ev_meta) (void)hipEventDestroy(c->ev_meta);
    if (c->ev_plan) (void)hipEventDestroy(c->ev_plan);
    delete c;
    return GSORT_OK;
}

gsort_status gsort_reserve(gsort_ctx *c, size_t n) {
    ST_TRY(check_ctx(c));
    HIP_TRY(c, hipSetDevice(c->device));
    const size_t cap = std::max<size_t>(n, 1) * 4;
    for (Slot s : {S_TMP, S_OUT}) ST_TRY(ensure(c, c->slot[s], cap));
    if (c->nranks > 1)
        for (Slot s : {S_CUR, S_SORTED, S_RECV}) ST_TRY(ensure(c, c->slot[s], cap));
    ST_TRY(ensure_pass_scratch(c, n));
    HIP_TRY(c, hipStreamSynchronize(c->stream));
    return GSORT_OK;
}

gsort_status gsort_set_local_algo(gsort_ctx *c, int algo) {
    ST_TRY(check_ctx(c));
    if (algo != GSORT_LOCAL_MSD && algo != GSORT_LOCAL_LSD)
        return set_err(c, GSORT_EINVAL, "unknown local sort algorithm");
    c->local_algo = algo;
    return GSORT_OK;
}

gsort_status gsort_set_sample_balanced(gsort_ctx *c, int on) {
    ST_TRY(check_ctx(c));
    c->sample_balanced = on != 0;
    return GSORT_OK;
}

gsort_status gsort_set_ref_compat(gsort_ctx *c, int radix_p) {
    ST_TRY(check_ctx(c));
    if (radix_p < -1) return set_err(c, GSORT_EINVAL, "ref compat: radix_p must be >= -1");
    c->ref_compat = radix_p;
    return GSORT_OK;
}

gsort_status gsort_radix(gsort_ctx *c, const int32_t *d_keys, size_t n_local, int32_t **d_out,
                         size_t *n_out, gsort_stats *stats) {
    ST_TRY(check_ctx(c));
    if (!d_out || !n_out || (n_local && !d_keys)) return set_err(c, GSORT_EINVAL, "null argument");
    ST_TRY(check_input(c, d_keys));
    ST_TRY(reset_call(c));
    timing_begin(c, stats);
    TimerScope timer_scope;
    hipEvent_t t0 = c->comm ? tic_rec(c) : tic(c);
    gsort_status st;
    uint64_t nout = 0;
    if (c->ref_compat) {
        st = radix_compat(c, d_keys, n_local, d_out, &nout, stats);
    } else if (!c->comm) {
        ST_TRY(ensure(c, c->slot[S_OUT], std::max<size_t>(n_local, 1) * 4));
        int pr = 0;
        st = local_sort(c, reinterpret_cast<const uint32_t *>(d_keys), n_local,
                        slot_ptr<uint32_t>(c, S_OUT), nullptr, &pr, stats, true);
        if (stats) stats->passes_run = pr;
        *d_out = slot_ptr<int32_t>(c, S_OUT);
        nout = n_local;
    } else if (c->local_algo == GSORT_LOCAL_LSD) {
        st = radix_dist(c, d_keys, n_local, d_out, &nout, stats);
    } else {
        st = radix_dist_exact(c, d_keys, n_local, d_out, &nout, stats);
    }
    if (st != GSORT_OK) return st;
    if (c->comm) toc_rec(c, PH_TOTAL, t0);
    else toc(c, PH_TOTAL, t0);
    HIP_TRY(c, hipStreamSynchronize(c->stream));
    *n_out = nout;
    if (stats) { stats->keys_local_in = n_local; stats->keys_local_out = nout; }
    timing_finish(c, stats);
    if (canary_mode()) ST_TRY(check_all_guards(c, __func__));
    return GSORT_OK;
}

gsort_status gsort_sample(gsort_ctx *c, const int32_t *d_keys, size_t n_local, int32_t **d_out,
                          size_t *n_out, gsort_stats *stats) {
    ST_TRY(check_ctx(c));
    if (!d_out || !n_out || (n_local && !d_keys)) return set_err(c, GSORT_EINVAL, "null argument");
    ST_TRY(check_input(c, d_keys));
    ST_TRY(reset_call(c));
    timing_begin(c, stats);
    TimerScope timer_scope;
    hipEvent_t t0 = c->comm ? tic_rec(c) : tic(c);
    uint64_t nout = 0;
    if (!c->comm) {
        // one rank: no splitters, one bucket (the reference reads splitters[-1] here, Q10)
        ST_TRY(ensure(c, c->slot[S_OUT], std::max<size_t>(n_local, 1) * 4));
        int pr = 0;
        ST_TRY(local_sort(c, reinterpret_cast<const uint32_t *>(d_keys), n_local,
                          slot_ptr<uint32_t>(c, S_OUT), nullptr, &pr, stats, true));
        if (stats) stats->passes_run = pr;
        c->splitters.clear();
        c->bucket_counts.assign(1, n_local);
        *d_out = slot_ptr<int32_t>(c, S_OUT);
        nout = n_local;
    } else {
        ST_TRY(sample_dist(c, d_keys, n_local, d_out, &nout, stats));
    }
    if (c->comm) toc_rec(c, PH_TOTAL, t0);
    else toc(c, PH_TOTAL, t0);
    HIP_TRY(c, hipStreamSynchronize(c->stream));
    *n_out = nout;
    if (stats) { stats->keys_local_in = n_local; stats->keys_local_out = nout; }
    timing_finish(c, stats);
    if (canary_mode()) ST_TRY(check_all_guards(c, __func__));
    return GSORT_OK;
}

int gsort_last_plan(const gsort_ctx *c) { return c ? c->last_plan : -1; }

gsort_status gsort_sample_info(const gsort_ctx *c, int32_t *splitters, uint64_t *bucket_counts) {
    if (!c) return GSORT_EINVAL;
    if (splitters) std::copy(c->splitters.begin(), c->splitters.end(), splitters);
    if (bucket_counts) std::copy(c->bucket_counts.begin(), c->bucket_counts.end(), bucket_counts);
    return GSORT_OK;
}

namespace {

// Pageable host <-> device copies of the drop-in path (the reference's rank-0 int_buf,
// radix:139,192 / sample:82,195) through kStageBufs pinned chunks: kStageThreads host threads
// copy chunk i between the caller's pageable array and a pinned buffer while the DMA engine
// moves chunk i-1 over PCIe, instead of the runtime's own pageable path.  Small copies go
// directly.
constexpr int kStageBufs = 4, kStageThreads = 16;  // 16: the GPU box's CPU share
constexpr size_t kStageChunk = 32u << 20, kStageMin = 16u << 20;

gsort_status stage_init(gsort_ctx *c) {
    for (int b = 0; b < kStageBufs; ++b) {
        if (!c->h_stage[b] &&
            hipHostMalloc(reinterpret_cast<void **>(&c->h_stage[b]), kStageChunk) != hipSuccess) {
            (void)hipGetLastError();
            c->h_stage[b] = nullptr;
            return set_err(c, GSORT_ENOMEM, "hipHostMalloc of a staging chunk failed");
        }
        if (!c->ev_stage[b])
            HIP_TRY(c, hipEventCreateWithFlags(&c->ev_stage[b], hipEventDisableTiming));
    }
    return GSORT_OK;
}

// host memcpy of len bytes split over kStageThreads threads (the calling thread takes a share;
// GSORT_STAGE_THREADS overrides the count)
void par_memcpy(char *dst, const char *src, size_t len) {
    static const int nt = getenv("GSORT_STAGE_THREADS")
                              ? std::max(1, std::min(64, atoi(getenv("GSORT_STAGE_THREADS"))))
                              : kStageThreads;
    const size_t share = ((len + nt - 1) / nt + 4095) & ~(size_t)4095;
    std::vector<std::thread> th;
    for (int t = 1; t < nt; ++t) {
        const size_t a = (size_t)t * share;
        if (a >= len) break;
        th.emplace_back([=] { memcpy(dst + a, src + a, std::min(share, len - a)); });
    }
    memcpy(dst, src, std::min(share, len));
    for (auto &x : th) x.join();
}

gsort_status staged_h2d(gsort_ctx *c, void *d_dst, const void *h_src, size_t bytes) {
    if (bytes < kStageMin) {
        HIP_TRY(c, hipMemcpyAsync(d_dst, h_src, bytes, hipMemcpyHostToDevice, c->stream));
        return GSORT_OK;
    }
    ST_TRY(stage_init(c));
    const size_t nch = (bytes + kStageChunk - 1) / kStageChunk;
    for (size_t i = 0; i < nch; ++i) {
        const int b = (int)(i % kStageBufs);
        const size_t off = i * kStageChunk, len = std::min(kStageChunk, bytes - off);
        if (i >= (size_t)kStageBufs) HIP_TRY(c, hipEventSynchronize(c->ev_stage[b]));
        par_memcpy(c->h_stage[b], static_cast<const char *>(h_src) + off, len);
        HIP_TRY(c, hipMemcpyAsync(static_cast<char *>(d_dst) + off, c->h_stage[b], len,
                                  hipMemcpyHostToDevice, c->stream));
        HIP_TRY(c, hipEventRecord(c->ev_stage[b], c->stream));
    }
    return GSORT_OK;
}

gsort_status staged_d2h(gsort_ctx *c, void *h_dst, const void *d_src, size_t bytes) {
    if (bytes < kStageMin) {
        HIP_TRY(c, hipMemcpyAsync(h_dst, d_src, bytes, hipMemcpyDeviceToHost, c->stream));
        HIP_TRY(c, hipStreamSynchronize(c->stream));
        return GSORT_OK;
    }
    ST_TRY(stage_init(c));
    const size_t nch = (bytes + kStageChunk - 1) / kStageChunk;
    auto issue = [&](size_t i) -> gsort_status {
        const int b = (int)(i % kStageBufs);
        const size_t off = i * kStageChunk, len = std::min(kStageChunk, bytes - off);
        HIP_TRY(c, hipMemcpyAsync(c->h_stage[b], static_cast<const char *>(d_src) + off, len,
                                  hipMemcpyDeviceToHost, c->stream));
        HIP_TRY(c, hipEventRecord(c->ev_stage[b], c->stream));
        return GSORT_OK;
    };
    for (size_t i = 0; i < nch && i < (size_t)kStageBufs; ++i) ST_TRY(issue(i));
    for (size_t i = 0; i < nch; ++i) {
        const int b = (int)(i % kStageBufs);
        const size_t off = i * kStageChunk, len = std::min(kStageChunk, bytes - off);
        HIP_TRY(c, hipEventSynchronize(c->ev_stage[b]));
        par_memcpy(static_cast<char *>(h_dst) + off, c->h_stage[b], len);
        if (i + kStageBufs < nch) ST_TRY(issue(i + kStageBufs));
    }
    return GSORT_OK;
}

}  // namespace

gsort_status gsort_scatter_from_root(gsort_ctx *c, const int32_t *h_root, size_t n_total,
                                     int32_t **d_keys, size_t *n_local) {
    ST_TRY(check_ctx(c));
    if (!d_keys || !n_local || (c->rank == 0 && n_total && !h_root)) return GSORT_EINVAL;
    ST_TRY(reset_call(c));
    const int P = c->nranks;
    uint64_t B, mine;
    block_of(n_total, P, c->rank, &B, &mine);
    ST_TRY(ensure(c, c->slot[S_IN], std::max<uint64_t>(mine, 1) * 4));
    int32_t *d_in = slot_ptr<int32_t>(c, S_IN);
    if (P == 1) {
        if (n_total)
            ST_TRY(staged_h2d(c, d_in, h_root, n_total * 4));
    } else {
        std::vector<size_t> sc(P, 0), sd(P, 0), rc(P, 0), rd(P, 0);
        const void *src = nullptr;
        if (c->rank == 0) {
            ST_TRY(ensure(c, c->slot[S_STAGE], std::max<size_t>(n_total, 1) * 4));
            if (n_total)
                ST_TRY(staged_h2d(c, c->slot[S_STAGE].p, h_root, n_total * 4));
            for (int q = 0; q < P; ++q) {
                uint64_t bq, lq;
                block_of(n_total, P, q, &bq, &lq);
                sc[q] = lq * 4;
                sd[q] = std::min<uint64_t>((uint64_t)q * B, n_total) * 4;
            }
            src = c->slot[S_STAGE].p;
        }
        rc[0] = mine * 4;
        ST_TRY(comm_try(c, c->comm->alltoallv(src, sc.data(), sd.data(), d_in, rc.data(),
                                              rd.data(), c->stream)));
    }
    HIP_TRY(c, hipStreamSynchronize(c->stream));
    *d_keys = d_in;
    *n_local = mine;
    return GSORT_OK;
}

gsort_status gsort_gather_to_root(gsort_ctx *c, const int32_t *d_out, size_t n_out,
                                  int32_t *h_root) {
    ST_TRY(check_ctx(c));
    if ((n_out && !d_out) || (c->rank == 0 && !h_root)) return GSORT_EINVAL;
    ST_TRY(reset_call(c));
    const int P = c->nranks;
    if (P == 1) {
        if (n_out) ST_TRY(staged_d2h(c, h_root, d_out, n_out * 4));
        HIP_TRY(c, hipStreamSynchronize(c->stream));
        return GSORT_OK;
    }
    std::vector<uint64_t> sizes;
    ST_TRY(allgather_u64(c, n_out, sizes));
    uint64_t total = 0;
    std::vector<size_t> sc(P, 0), sd(P, 0), rc(P, 0), rd(P, 0);
    for (int r = 0; r < P; ++r) {
        if (c->rank == 0) { rc[r] = sizes[r] * 4; rd[r] = total * 4; }
        total += sizes[r];
    }
    sc[0] = n_out * 4;
    void *dst = nullptr;
    if (c->rank == 0) {
        ST_TRY(ensure(c, c->slot[S_STAGE], std::max<uint64_t>(total, 1) * 4));
        dst = c->slot[S_STAGE].p;
    }
    ST_TRY(comm_try(c, c->comm->alltoallv(d_out, sc.data(), sd.data(), dst, rc.data(), rd.data(),
                                          c->stream)));
    if (c->rank == 0 && total) ST_TRY(staged_d2h(c, h_root, dst, total * 4));
    HIP_TRY(c, hipStreamSynchronize(c->stream));
    return GSORT_OK;
}

gsort_status gsort_generate(gsort_ctx *c, int dist, uint64_t seed, uint64_t start, size_t n,
                            int32_t *d_out) {
    ST_TRY(check_ctx(c));
    if ((dist != 0 && dist != 1) || (n && !d_out)) return GSORT_EINVAL;
    HIP_TRY(c, hipSetDevice(c->device));
    HIP_TRY(c, launch_generate(dist, seed, start, n, d_out, c->stream));
    HIP_TRY(c, hipStreamSynchronize(c->stream));
    return GSORT_OK;
}

gsort_status gsort_fingerprint(gsort_ctx *c, const int32_t *d_keys, size_t n, uint64_t *sum,
                               uint64_t *xr, int *sorted, int32_t *first, int32_t *last) {
    ST_TRY(check_ctx(c));
    if (n && !d_keys) return GSORT_EINVAL;
    HIP_TRY(c, hipSetDevice(c->device));
    unsigned long long *d_acc = reinterpret_cast<unsigned long long *>(c->d_small + OFF_PLAN);
    uint64_t *h = reinterpret_cast<uint64_t *>(c->h_small + OFF_PLAN);
    HIP_TRY(c, hipMemsetAsync(d_acc, 0, 24, c->stream));
    HIP_TRY(c, launch_fingerprint(d_keys, n, d_acc, c->stream));
    HIP_TRY(c, hipMemcpyAsync(h, d_acc, 24, hipMemcpyDeviceToHost, c->stream));
    int32_t *h_fl = reinterpret_cast<int32_t *>(h + 3);
    h_fl[0] = h_fl[1] = 0;
    if (n) {
        HIP_TRY(c, hipMemcpyAsync(h_fl, d_keys, 4, hipMemcpyDeviceToHost, c->stream));
        HIP_TRY(c, hipMemcpyAsync(h_fl + 1, d_keys + n - 1, 4, hipMemcpyDeviceToHost, c->stream));
    }
    HIP_TRY(c, hipStreamSynchronize(c->stream));
    if (sum) *sum = h[0];
    if (xr) *xr = h[1];
    if (sorted) *sorted = h[2] == 0;
    if (first) *first = h_fl[0];
    if (last) *last = h_fl[1];
    return GSORT_OK;
}

gsort_status gsort_device_alloc(gsort_ctx *c, size_t bytes, void **d_ptr) {
    ST_TRY(check_ctx(c));
    if (!d_ptr) return GSORT_EINVAL;
    HIP_TRY(c, hipSetDevice(c->device));
    DevBuf b;
    const size_t want = (std::max<size_t>(bytes, 4) + alloc_align() - 1) & ~(alloc_align() - 1);
    hipError_t e = dev_malloc(b, want, "user");
    if (e != hipSuccess) return alloc_err(c, e, want, "gsort_device_alloc");
    {
        std::unique_lock<std::mutex> lk(serial_mutex(), std::defer_lock);
        if (canary_mode()) lk.lock();
        c->user_bufs[b.p] = b;
    }
    *d_ptr = b.p;
    return GSORT_OK;
}

gsort_status gsort_device_free(gsort_ctx *c, void *d_ptr) {
    ST_TRY(check_ctx(c));
    HIP_TRY(c, hipSetDevice(c->device));
    if (!d_ptr) return GSORT_OK;
    auto it = c->user_bufs.find(d_ptr);
    if (it == c->user_bufs.end())
        return set_err(c, GSORT_EINVAL, "gsort_device_free: not a gsort_device_alloc pointer");
    DevBuf b = it->second;
    {
        std::unique_lock<std::mutex> lk(serial_mutex(), std::defer_lock);
        if (canary_mode()) lk.lock();
        c->user_bufs.erase(it);
    }
    hipError_t e = dev_free(b);
    if (e != hipSuccess)
        return set_err(c, GSORT_EHIP, std::string("hipFree: ") + hipGetErrorString(e));
    return GSORT_OK;
}

gsort_status gsort_copy_ceiling(gsort_ctx *c, size_t bytes, int reps, double *ms,
                                double *gbps) {
    ST_TRY(check_ctx(c));
    if (!ms || !gbps || reps < 1 || bytes < 16) return GSORT_EINVAL;
    HIP_TRY(c, hipSetDevice(c->device));
    bytes &= ~size_t(15);
    DevBuf a, b;
    hipError_t e = dev_malloc(a, bytes, "ceiling_src");
    if (e != hipSuccess) return alloc_err(c, e, bytes, "gsort_copy_ceiling");
    e = dev_malloc(b, bytes, "ceiling_dst");
    if (e != hipSuccess) { (void)dev_free(a); return alloc_err(c, e, bytes, "gsort_copy_ceiling"); }
    hipEvent_t e0 = next_event(c), e1 = nullptr;
    if (e0) e1 = next_event(c);
    gsort_status st = (e0 && e1) ? GSORT_OK : set_err(c, GSORT_EHIP, "hipEventCreate failed");
    double best = 0.0;
    auto run = [&]() -> gsort_status {
        HIP_TRY(c, hipMemsetAsync(a.p, 0x5a, bytes, c->stream));
        std::vector<float> t;
        for (int r = 0; r <= reps; ++r) {  // r == 0: warm-up
            HIP_TRY(c, hipEventRecord(e0, c->stream));
            HIP_TRY(c, launch_stream_copy(a.p, b.p, bytes, c->stream));
            HIP_TRY(c, hipEventRecord(e1, c->stream));
            HIP_TRY(c, hipEventSynchronize(e1));
            float x = 0.f;
            HIP_TRY(c, hipEventElapsedTime(&x, e0, e1));
            if (r) t.push_back(x);
        }
        std::sort(t.begin(), t.end());
        best = t[t.size() / 2];
        return GSORT_OK;
    };
    if (st == GSORT_OK) st = run();
    c->ev_used = 0;
    (void)dev_free(a);
    (void)dev_free(b);
    if (st != GSORT_OK) return st;
    *ms = best;
    *gbps = 2.0 * (double)bytes / (best * 1e-3) / 1e9;
    return GSORT_OK;
}

gsort_status gsort_copy_to_host(gsort_ctx *c, void *h_dst, const void *d_src, size_t bytes) {
    ST_TRY(check_ctx(c));
    HIP_TRY(c, hipSetDevice(c->device));
    if (bytes) HIP_TRY(c, hipMemcpyAsync(h_dst, d_src, bytes, hipMemcpyDeviceToHost, c->stream));
    HIP_TRY(c, hipStreamSynchronize(c->stream));
    return GSORT_OK;
}

gsort_status gsort_copy_to_device(gsort_ctx *c, void *d_dst, const void *h_src, size_t bytes) {
    ST_TRY(check_ctx(c));
    HIP_TRY(c, hipSetDevice(c->device));
    if (bytes) HIP_TRY(c, hipMemcpyAsync(d_dst, h_src, bytes, hipMemcpyHostToDevice, c->stream));
    HIP_TRY(c, hipStreamSynchronize(c->stream));
    return GSORT_OK;
}

}  // extern "C"
