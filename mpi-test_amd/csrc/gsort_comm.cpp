// gsort_comm.cpp -- RCCL and in-process transports (see gsort_comm.h).
#include "gsort_comm.h"

#include "gsort_debug.h"

#include <dlfcn.h>
#include <errno.h>
#include <fcntl.h>
#include <rccl/rccl.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <time.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <mutex>
#include <vector>

namespace gsort {

bool serial_mode() {
    static const bool on = getenv("GSORT_SERIAL") && atoi(getenv("GSORT_SERIAL"));
    return on;
}
bool canary_mode() {
    static const bool on = getenv("GSORT_CANARY") && atoi(getenv("GSORT_CANARY"));
    return on;
}
std::mutex &serial_mutex() {
    static std::mutex m;
    return m;
}
bool trace_mode() {
    static const bool on = getenv("GSORT_TRACE") && atoi(getenv("GSORT_TRACE"));
    return on;
}

namespace {
struct TraceRec {
    double t_us;
    int rank;
    const char *what;
};
constexpr size_t kTraceRing = 1 << 16, kTraceDump = 400;
std::mutex g_trace_mu;
std::vector<TraceRec> g_trace(kTraceRing);
size_t g_trace_n = 0;
bool g_trace_dumped = false;
const auto g_t0 = std::chrono::steady_clock::now();
}  // namespace

void trace_op(int rank, const char *what) {
    const double t = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() -
                                                               g_t0).count();
    std::lock_guard<std::mutex> lk(g_trace_mu);
    g_trace[g_trace_n++ % kTraceRing] = {t, rank, what};
}

void trace_dump(const char *why) {
    std::lock_guard<std::mutex> lk(g_trace_mu);
    if (g_trace_dumped) return;
    g_trace_dumped = true;
    const size_t n = std::min(g_trace_n, kTraceDump);
    fprintf(stderr, "GSORT_TRACE: %s; last %zu of %zu HIP ops (time us, rank, op):\n", why, n,
            g_trace_n);
    for (size_t i = g_trace_n - n; i < g_trace_n; ++i) {
        const TraceRec &r = g_trace[i % kTraceRing];
        fprintf(stderr, "  %12.1f r%-2d %.160s\n", r.t_us, r.rank, r.what);
    }
    fflush(stderr);
}

// ---------------------------------------------------------------------------------------
// RCCL over xGMI
// ---------------------------------------------------------------------------------------
class RcclComm : public Comm {
  public:
    RcclComm(ncclComm_t c, int rank, int n) : comm_(c) { rank_ = rank; size_ = n; }
    ~RcclComm() override { ncclCommDestroy(comm_); }

    gsort_status check(ncclResult_t r, const char *what) {
        if (r == ncclSuccess) return GSORT_OK;
        err = std::string(what) + ": " + ncclGetErrorString(r);
        return GSORT_ERCCL;
    }
    gsort_status allgather(const void *send, void *recv, size_t bytes, hipStream_t s) override {
        return check(ncclAllGather(send, recv, bytes, ncclChar, comm_, s), "ncclAllGather");
    }
    // One grouped send/recv round: every (src, dst) pair with a non-zero count is one
    // message of exactly that many bytes (the reference sends fixed 1.5B-int messages with
    // the real length in the tag, mpi_sample_sort.c:161,168).
    gsort_status alltoallv(const void *send, const size_t *scount, const size_t *sdispl,
                           void *recv, const size_t *rcount, const size_t *rdispl,
                           hipStream_t s) override {
        // the rank's own piece is a device copy on its stream, not an RCCL self send/recv:
        // RCCL's copy moved a 512 MiB self-message at ~2.2 TB/s of HBM traffic (0.49 ms at
        // 2^28 keys, forced-distributed P = 1), hipMemcpyAsync at the copy ceiling (~5.8 TB/s).
        // GSORT_RCCL_SELF=1 keeps it in RCCL (tests/test_gpu_rccl.py pins RCCL's own limits)
        const bool self_rccl = rccl_self();
        if (!self_rccl && scount[rank_]) {
            if (scount[rank_] != rcount[rank_]) {
                err = "alltoallv: self send / receive counts differ";
                return GSORT_EINVAL;
            }
            const hipError_t e = hipMemcpyAsync((char *)recv + rdispl[rank_],
                                                (const char *)send + sdispl[rank_],
                                                scount[rank_], hipMemcpyDeviceToDevice, s);
            if (e != hipSuccess) {
                err = std::string("hipMemcpyAsync (self piece): ") + hipGetErrorString(e);
                return GSORT_EHIP;
            }
        }
        // nothing for RCCL (one rank; a rank that neither sends nor receives): no group at all
        // -- an empty ncclGroupStart / End still left ~20 us of idle on the stream
        // (forced-distributed P = 1 trace, round 3)
        bool any = false;
        for (int q = 0; q < size_ && !any; ++q)
            if (q != rank_ || self_rccl) any = scount[q] || rcount[q];
        if (!any) return GSORT_OK;
        gsort_status st = check(ncclGroupStart(), "ncclGroupStart");
        if (st != GSORT_OK) return st;
        // messages go in pieces of at most max_msg_ = 2^30 bytes (matched in order on both
        // sides): measured on MI355X with RCCL of ROCm 7.2, a self ncclSend/ncclRecv of
        // 2^30 + 256 bytes or more comes back wrong (keys missing) while 2^30-byte pieces are
        // exact (tests/test_gpu_rccl.py pins both sides of the boundary;
        // GSORT_RCCL_MAX_MSG overrides the piece size for that test)
        for (int q = 0; q < size_ && st == GSORT_OK; ++q) {
            if (q == rank_ && !self_rccl) continue;
            for (size_t o = 0; o < scount[q] && st == GSORT_OK; o += max_msg_)
                st = check(ncclSend((const char *)send + sdispl[q] + o,
                                    std::min(max_msg_, scount[q] - o), ncclChar, q, comm_, s),
                           "ncclSend");
            for (size_t o = 0; o < rcount[q] && st == GSORT_OK; o += max_msg_)
                st = check(ncclRecv((char *)recv + rdispl[q] + o,
                                    std::min(max_msg_, rcount[q] - o), ncclChar, q, comm_, s),
                           "ncclRecv");
        }
        gsort_status st2 = check(ncclGroupEnd(), "ncclGroupEnd");
        return st != GSORT_OK ? st : st2;
    }
    gsort_status bcast(void *buf, size_t bytes, int root, hipStream_t s) override {
        return check(ncclBroadcast(buf, buf, bytes, ncclChar, root, comm_, s), "ncclBroadcast");
    }

  private:
    static bool rccl_self() {
        const char *e = getenv("GSORT_RCCL_SELF");
        return e && e[0] == '1';
    }
    static size_t max_msg() {
        const char *e = getenv("GSORT_RCCL_MAX_MSG");
        const size_t v = e ? (size_t)strtoull(e, nullptr, 0) : 0;
        return v ? v : size_t(1) << 30;
    }
    const size_t max_msg_ = max_msg();
    ncclComm_t comm_;
};

// RCCL's bootstrap (the uid's listening socket and the ranks' connections to it) runs over
// TCP on an interface RCCL picks itself; on these single-node boxes the picked interface
// refused the connection (measured: ncclCommInitRank "remote process exited or there was a
// network error" after 35 retries).  Every rank of a gsort job is on one node, so the
// bootstrap goes over loopback unless the caller chose an interface.  The key exchange itself
// is GPU-to-GPU (xGMI), not sockets.
static void bootstrap_on_loopback() { setenv("NCCL_SOCKET_IFNAME", "lo", 0); }

gsort_status rccl_get_uid(gsort_uid *out) {
    static_assert(sizeof(ncclUniqueId) == sizeof(gsort_uid), "uid size");
    bootstrap_on_loopback();
    ncclUniqueId id;
    if (ncclGetUniqueId(&id) != ncclSuccess) return GSORT_ERCCL;
    memcpy(out, &id, sizeof(id));
    return GSORT_OK;
}

gsort_status runtime_info(gsort_runtime_info_t *out) {
    memset(out, 0, sizeof(*out));
    if (hipRuntimeGetVersion(&out->hip_runtime) != hipSuccess) out->hip_runtime = -1;
    if (ncclGetVersion(&out->rccl) != ncclSuccess) out->rccl = -1;
    Dl_info di;
    if (dladdr(reinterpret_cast<void *>(&hipRuntimeGetVersion), &di) && di.dli_fname)
        snprintf(out->hip_path, sizeof(out->hip_path), "%s", di.dli_fname);
    if (dladdr(reinterpret_cast<void *>(&ncclGetVersion), &di) && di.dli_fname)
        snprintf(out->rccl_path, sizeof(out->rccl_path), "%s", di.dli_fname);
    return GSORT_OK;
}

Comm *make_rccl_comm(int rank, int nranks, const gsort_uid *uid, std::string *err) {
    bootstrap_on_loopback();
    ncclUniqueId id;
    memcpy(&id, uid, sizeof(id));
    ncclComm_t c;
    ncclResult_t r = ncclCommInitRank(&c, nranks, id, rank);
    if (r != ncclSuccess) {
        *err = std::string("ncclCommInitRank: ") + ncclGetErrorString(r);
        return nullptr;
    }
    return new RcclComm(c, rank, nranks);
}

// ---------------------------------------------------------------------------------------
// In-process rank group, stream-ordered like RCCL (no host wait on the GPU inside a
// collective).  Each collective: every rank records a "ready" event on its stream (its send
// data is complete once the stream reaches it), publishes pointers and events, meets the others
// at a host barrier, makes its stream wait for the peers' ready events and pulls what it needs
// with hipMemcpyAsync, records a "done" event, meets them again, and makes its stream wait for
// the peers' done events (so no rank reuses a buffer a peer is still reading).  The two
// barriers order every event's record before the waits on it and before its next record.
// (Round 4 and before synchronised both streams in every collective: the P-rank emulation then
// paid host round trips that the RCCL path does not.)
// ---------------------------------------------------------------------------------------
struct GroupState {
    int n;
    std::mutex m;
    std::condition_variable cv;
    int arrived = 0;
    uint64_t generation = 0;
    bool broken = false;
    std::vector<const void *> ptr;
    std::vector<const size_t *> count, displ;
    std::vector<hipEvent_t> ready, done;  // per rank, created by the rank on first use
    int device = -1;                      // every rank's HIP device (group_state_join)
    explicit GroupState(int n_)
        : n(n_), ptr(n_), count(n_), displ(n_), ready(n_, nullptr), done(n_, nullptr) {}
    ~GroupState() {
        for (auto e : ready)
            if (e) (void)hipEventDestroy(e);
        for (auto e : done)
            if (e) (void)hipEventDestroy(e);
    }
};

GroupState *group_state_create(int nranks) { return new GroupState(nranks); }
void group_state_destroy(GroupState *g) { delete g; }
int group_state_size(const GroupState *g) { return g->n; }
bool group_state_join(GroupState *g, int device) {
    std::lock_guard<std::mutex> lk(g->m);
    if (g->device < 0) g->device = device;
    return g->device == device;
}

class GroupComm : public Comm {
  public:
    GroupComm(GroupState *g, int rank) : g_(g) { rank_ = rank; size_ = g->n; }

    // generation barrier with a timeout so a dead peer cannot hang the process (60 s: far above
    // any collective here, short enough that a failed rank surfaces as an error, not a hang)
    bool barrier() {
        std::unique_lock<std::mutex> lk(g_->m);
        if (g_->broken) return false;
        const uint64_t gen = g_->generation;
        if (++g_->arrived == g_->n) {
            g_->arrived = 0;
            ++g_->generation;
            g_->cv.notify_all();
            return true;
        }
        const bool ok = g_->cv.wait_for(lk, std::chrono::seconds(60),
                                        [&] { return g_->generation != gen || g_->broken; });
        if (!ok || g_->broken) {
            g_->broken = true;
            g_->cv.notify_all();
            return false;
        }
        return true;
    }
    gsort_status fail(const char *what) {
        err = std::string("in-process group: ") + what;
        return GSORT_ECOMM;
    }
    void break_group() {
        std::lock_guard<std::mutex> lk(g_->m);
        g_->broken = true;
        g_->cv.notify_all();
    }
    // every HIP call goes through hip_op (GSORT_SERIAL: serialized with all other contexts)
    template <class F>
    gsort_status hip(F &&f, const char *what) {
        if (trace_mode()) trace_op(rank_, what);
        const hipError_t e = hip_op(f);
        if (e == hipSuccess) return GSORT_OK;
        if (trace_mode()) trace_dump(what);
        err = std::string(what) + ": " + hipGetErrorString(e);
        return GSORT_EHIP;
    }

    // the collective's first half: this rank's ready event recorded and published, the
    // barrier, the stream made to wait for every peer's ready event
    gsort_status open(hipStream_t s) {
        gsort_status st = GSORT_OK;
        // (the ranks share one device -- group_state_join refuses any other -- so a device-scope
        // release orders a rank's writes before a peer stream's copies; default flags if the
        // runtime refuses that one)
        for (hipEvent_t *e : {&g_->ready[rank_], &g_->done[rank_]})
            if (!*e && st == GSORT_OK)
                st = hip([&] {
                    const hipError_t r = hipEventCreateWithFlags(
                        e, hipEventDisableTiming | hipEventDisableSystemFence);
                    return r == hipSuccess ? r : hipEventCreateWithFlags(e, hipEventDisableTiming);
                }, "hipEventCreateWithFlags");
        if (st == GSORT_OK)
            st = hip([&] { return hipEventRecord(g_->ready[rank_], s); }, "hipEventRecord");
        // a local failure breaks the group before the barrier: the peers must neither wait for
        // this rank in vain nor copy its buffers behind a stale ready event
        if (st != GSORT_OK) { break_group(); return st; }
        if (!barrier()) return fail("barrier timeout");
        for (int r = 0; r < size_ && st == GSORT_OK; ++r)
            if (r != rank_)
                st = hip([&] { return hipStreamWaitEvent(s, g_->ready[r], 0); },
                         "hipStreamWaitEvent");
        return st;
    }
    // the second half: done event recorded, the barrier, the stream made to wait for the peers'
    // done events (their reads of this rank's buffers)
    gsort_status close(hipStream_t s, gsort_status st) {
        if (st == GSORT_OK)
            st = hip([&] { return hipEventRecord(g_->done[rank_], s); }, "hipEventRecord");
        if (st != GSORT_OK) { break_group(); return st; }  // every rank fails this collective
        if (!barrier()) return fail("barrier timeout");
        for (int r = 0; r < size_ && st == GSORT_OK; ++r)
            if (r != rank_)
                st = hip([&] { return hipStreamWaitEvent(s, g_->done[r], 0); },
                         "hipStreamWaitEvent");
        return st;
    }
    gsort_status allgather(const void *send, void *recv, size_t bytes, hipStream_t s) override {
        g_->ptr[rank_] = send;
        gsort_status st = open(s);
        for (int r = 0; r < size_ && st == GSORT_OK; ++r)
            if (bytes)
                st = hip([&] {
                    return hipMemcpyAsync((char *)recv + (size_t)r * bytes, g_->ptr[r], bytes,
                                          hipMemcpyDeviceToDevice, s);
                }, "hipMemcpyAsync");
        return close(s, st);
    }
    gsort_status alltoallv(const void *send, const size_t *scount, const size_t *sdispl,
                           void *recv, const size_t *rcount, const size_t *rdispl,
                           hipStream_t s) override {
        g_->ptr[rank_] = send;
        g_->count[rank_] = scount;
        g_->displ[rank_] = sdispl;
        gsort_status st = open(s);
        for (int r = 0; r < size_ && st == GSORT_OK; ++r) {
            const size_t c = g_->count[r][rank_];
            if (c != rcount[r]) { st = fail("send/recv count mismatch"); break; }
            if (c)
                st = hip([&] {
                    return hipMemcpyAsync((char *)recv + rdispl[r],
                                          (const char *)g_->ptr[r] + g_->displ[r][rank_], c,
                                          hipMemcpyDeviceToDevice, s);
                }, "hipMemcpyAsync");
        }
        return close(s, st);
    }
    gsort_status bcast(void *buf, size_t bytes, int root, hipStream_t s) override {
        g_->ptr[rank_] = buf;
        gsort_status st = open(s);
        if (st == GSORT_OK && rank_ != root && bytes)
            st = hip([&] {
                return hipMemcpyAsync(buf, g_->ptr[root], bytes, hipMemcpyDeviceToDevice, s);
            }, "hipMemcpyAsync");
        return close(s, st);
    }

  private:
    GroupState *g_;
};

Comm *make_group_comm(GroupState *g, int rank) { return new GroupComm(g, rank); }

}  // namespace gsort

// ---------------------------------------------------------------------------------------
// Same-node process group over HIP IPC (one process per rank, any number of ranks per GPU).
// RCCL refuses two ranks on one device, so this is how `mpirun -np P radix_sort` runs the
// distributed algorithm on a node with fewer GPUs than ranks (a one-GPU box in particular),
// each rank its own process and context as with RCCL.  Keys move GPU to GPU: every rank owns
// one exported staging buffer; a collective copies the rank's send range into it, publishes its
// counts in a POSIX shared-memory control block, meets the others at a barrier, pulls what it
// needs from the peers' staging buffers (opened once through their IPC handles, again only when
// a peer grew its buffer), synchronises and meets them again (so no rank overwrites a staging
// buffer a peer is still reading) -- GroupComm's protocol across processes.  (Exporting and
// opening every send buffer per collective instead failed intermittently on MI355X / ROCm 7.2:
// hipIpcOpenMemHandle "invalid device pointer".  The cause, isolated with
// tools/experiments/ipc_group.hip (profiles/r04_ipc_export_patterns.txt): an exported
// allocation that is FREED and replaced by a new one (the context's scratch buffers grow by
// free + malloc) -- importers of the replacement then read wrong bytes (P = 4: 225 of 768
// reads) or the runtime prints "IPC Attach: Invalid IPC handle!" and the group hangs, while
// re-exporting / re-opening one live allocation every round (P = 4, 8: 13 600 reads) and
// growing into new allocations that are never freed (768 reads) are exact.  So a staging
// buffer, once exported, is never freed while the group lives -- a grown one is kept in stages_
// until the destructor, whatever it costs in memory.)  The uid carries
// the control block's name; rank 0 creates it (gsort_get_uid_ipc) and unlinks it once every
// rank has attached.
// ---------------------------------------------------------------------------------------
namespace gsort {
namespace {

constexpr char kIpcMagic[8] = {'G', 'S', 'I', 'P', 'C', 0, 0, 2};
constexpr int kIpcMaxRanks = 64;
// A staging buffer past 2^30 bytes is exported as chunks of 2^30, each its own allocation and
// handle: with one exported 2^31-byte buffer (2^30 keys per rank at P = 2, packed) both ranks
// logged "pull: opening peer" and never "pull: opened" (GSORT_IPC_LOG,
// profiles/r05_ipc_2gib_hang.txt): they hung inside hipIpcOpenMemHandle of the peer's 2^31-byte
// export, before any copy, while every run with buffers of at most 2^30 bytes passed.  16
// chunks = 16 GiB of staging per rank: 2^32 keys of 4 B, 2^33 packed keys of 2 B.  The
// distributed radix caps a rank below 2^32 keys; the int32 send paths (sample sort's fallback,
// the LSD passes) check their largest send range against kIpcStageMax up front.
constexpr size_t kIpcChunk = size_t(1) << 30;
constexpr int kIpcChunks = 16;
constexpr size_t kIpcNameOff = 8, kIpcNameMax = 88, kIpcRanksOff = 96;

struct IpcSlot {
    hipIpcMemHandle_t handle[kIpcChunks];  // the rank's staging buffer, chunk by chunk
    uint64_t gen;                          // bumped whenever the staging buffer grows
    uint64_t chunk;                        // bytes per chunk
    uint32_t nchunk;
    uint64_t count[kIpcMaxRanks], displ[kIpcMaxRanks];  // bytes to / offsets for each rank
};
struct IpcShared {
    std::atomic<uint32_t> arrived, generation, broken, attached;
    int32_t n;
    IpcSlot slot[kIpcMaxRanks];
};
static_assert(std::atomic<uint32_t>::is_always_lock_free, "shared-memory atomics");

std::mutex g_shm_mu;
std::vector<std::string> g_shm_pending;  // created here, not yet unlinked (unlinked at exit)

void unlink_pending() {
    std::lock_guard<std::mutex> lk(g_shm_mu);
    for (const auto &n : g_shm_pending) shm_unlink(n.c_str());
    g_shm_pending.clear();
}

void forget_pending(const std::string &name) {
    std::lock_guard<std::mutex> lk(g_shm_mu);
    g_shm_pending.erase(std::remove(g_shm_pending.begin(), g_shm_pending.end(), name),
                        g_shm_pending.end());
}

IpcShared *map_shared(const char *name, bool create, std::string *err) {
    const int fd = shm_open(name, create ? O_RDWR | O_CREAT | O_EXCL : O_RDWR, 0600);
    if (fd < 0) {
        *err = std::string("shm_open ") + name + ": " + strerror(errno);
        return nullptr;
    }
    if (create && ftruncate(fd, sizeof(IpcShared)) != 0) {
        *err = std::string("ftruncate: ") + strerror(errno);
        close(fd);
        return nullptr;
    }
    void *p = mmap(nullptr, sizeof(IpcShared), PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
    close(fd);
    if (p == MAP_FAILED) {
        *err = std::string("mmap: ") + strerror(errno);
        return nullptr;
    }
    return static_cast<IpcShared *>(p);
}

// GSORT_IPC_LOG=1 (diagnostics): every step of every IPC collective to stderr
static bool ipc_log_on() {
    static const bool on = getenv("GSORT_IPC_LOG") && getenv("GSORT_IPC_LOG")[0] == '1';
    return on;
}

class IpcComm : public Comm {
    void log(const char *what, size_t a = 0, size_t b = 0) const {
        if (!ipc_log_on()) return;
        const double t = std::chrono::duration<double>(std::chrono::steady_clock::now() -
                                                       std::chrono::steady_clock::time_point{}).count();
        fprintf(stderr, "[ipc r%d %.6f] %s %zu %zu\n", rank_, t, what, a, b);
        fflush(stderr);
    }

  public:
    IpcComm(IpcShared *sh, int rank, int n)
        : sh_(sh), peer_(n), peer_chunk_(n, 0), peer_gen_(n, 0) { rank_ = rank; size_ = n; }
    ~IpcComm() override {
        for (auto &v : peer_)
            for (void *p : v) (void)hipIpcCloseMemHandle(p);
        // peers may still hold this rank's staging buffers open; the memory goes with the
        // process (or with their close), so the buffers are freed last
        for (void *p : stages_) (void)hipFree(p);
        munmap(sh_, sizeof(IpcShared));
    }

    // generation barrier in shared memory; a peer that does not arrive within 120 s breaks the
    // group (every later collective fails instead of hanging)
    bool barrier() {
        if (sh_->broken.load()) return false;
        const uint32_t gen = sh_->generation.load(std::memory_order_acquire);
        if (sh_->arrived.fetch_add(1, std::memory_order_acq_rel) + 1 == (uint32_t)size_) {
            sh_->arrived.store(0, std::memory_order_relaxed);
            sh_->generation.fetch_add(1, std::memory_order_acq_rel);
            return true;
        }
        const auto t0 = std::chrono::steady_clock::now();
        for (uint64_t spin = 0; sh_->generation.load(std::memory_order_acquire) == gen; ++spin) {
            if (sh_->broken.load()) return false;
            if (spin < 2000) continue;
            struct timespec ts = {0, 20000};
            nanosleep(&ts, nullptr);
            if ((spin & 1023) == 0 &&
                std::chrono::steady_clock::now() - t0 > std::chrono::seconds(120)) {
                sh_->broken.store(1);
                return false;
            }
        }
        return true;
    }
    gsort_status fail(const std::string &what) {
        err = "ipc group: " + what;
        return GSORT_ECOMM;
    }
    gsort_status hip(hipError_t e, const char *what) {
        if (e == hipSuccess) return GSORT_OK;
        err = std::string("ipc group: ") + what + ": " + hipGetErrorString(e);
        return GSORT_EHIP;
    }
    gsort_status copy(void *dst, const void *src, size_t bytes, hipStream_t s, const char *what) {
        return hip(hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToDevice, s), what);
    }
    // chunk size of a staging buffer for `span` bytes (GSORT_IPC_CHUNK: a smaller one, the test
    // hook that runs the chunked path on small inputs)
    static size_t chunk_limit() {
        static const size_t v = [] {
            const char *e = getenv("GSORT_IPC_CHUNK");
            const size_t c = e ? (size_t)strtoull(e, nullptr, 0) : 0;
            return c ? c : kIpcChunk;
        }();
        return v;
    }
    // the send range [0, span) into this rank's staging buffer (grown and re-exported as
    // needed), the counts into the control block
    gsort_status publish(const void *send, size_t span, const size_t *count, const size_t *displ,
                         hipStream_t s) {
        log("publish", span, chunk_ * chunks_.size());
        IpcSlot &me = sh_->slot[rank_];
        for (int q = 0; q < size_ && count; ++q) {
            me.count[q] = count[q];
            me.displ[q] = displ[q];
        }
        if (span > chunk_ * chunks_.size()) {
            // up to the chunk limit one power-of-two chunk, past it whole chunks (the ones
            // already at the limit are kept, a smaller one is replaced)
            const size_t lim = chunk_limit();
            size_t chunk = size_t(1) << 20;
            while (chunk < span && chunk < lim) chunk <<= 1;
            chunk = std::min(chunk, lim);
            const size_t n = (span + chunk - 1) / chunk;
            if (n > (size_t)kIpcChunks) {
                sh_->broken.store(1);  // the peers must not read this rank's stale staging
                return fail("send range over the staging limit");
            }
            if (chunk != chunk_) chunks_.clear();
            while (chunks_.size() < n) {
                void *p = nullptr;
                gsort_status st = hip(hipMalloc(&p, chunk), "hipMalloc (staging)");
                if (st == GSORT_OK)
                    st = hip(hipIpcGetMemHandle(&me.handle[chunks_.size()], p), "hipIpcGetMemHandle");
                if (st != GSORT_OK) {
                    if (p) (void)hipFree(p);
                    sh_->broken.store(1);
                    return st;
                }
                // never freed while the group lives: freeing an exported allocation and
                // exporting its replacement is what broke the peers' imports (header comment)
                stages_.push_back(p);
                chunks_.push_back(p);
            }
            chunk_ = chunk;
            me.chunk = chunk;
            me.nchunk = (uint32_t)n;
            me.gen = ++gen_;
        }
        gsort_status st = GSORT_OK;
        for (size_t o = 0; o < span && st == GSORT_OK; o += chunk_)
            st = copy(chunks_[o / chunk_], static_cast<const char *>(send) + o,
                      std::min(chunk_, span - o), s, "hipMemcpyAsync (stage)");
        log("publish: staged, synchronising");
        if (st == GSORT_OK) st = hip(hipStreamSynchronize(s), "hipStreamSynchronize");
        log("publish: done");
        return st;
    }
    // bytes [a, a + len) of rank r's send range into dst
    gsort_status pull(int r, const void *own, uint64_t a, size_t len, void *dst, hipStream_t s) {
        if (!len) return GSORT_OK;
        if (r == rank_) return copy(dst, static_cast<const char *>(own) + a, len, s, "hipMemcpyAsync");
        const IpcSlot &ps = sh_->slot[r];
        if (!ps.chunk || !ps.nchunk) return fail("pull from a peer without a staging buffer");
        std::vector<void *> &pv = peer_[r];
        if (peer_gen_[r] != ps.gen) {
            log("pull: opening peer", (size_t)r, (size_t)ps.gen);
            // chunks of an unchanged size are the same allocations: only the new ones open
            if (peer_chunk_[r] != ps.chunk) {
                for (void *p : pv) (void)hipIpcCloseMemHandle(p);
                pv.clear();
                peer_chunk_[r] = ps.chunk;
            }
            while (pv.size() < ps.nchunk) {
                void *p = nullptr;
                gsort_status st = hip(hipIpcOpenMemHandle(&p, ps.handle[pv.size()],
                                                          hipIpcMemLazyEnablePeerAccess),
                                      "hipIpcOpenMemHandle");
                if (st != GSORT_OK) return st;
                pv.push_back(p);
            }
            peer_gen_[r] = ps.gen;
            log("pull: opened", (size_t)r, pv.size());
        }
        const size_t c = peer_chunk_[r];
        gsort_status st = GSORT_OK;
        for (size_t end = a + len; a < end && st == GSORT_OK;) {
            const size_t i = a / c, off = a % c, l = std::min(end - a, c - off);
            if (i >= pv.size()) return fail("pull past the peer's staging buffer");
            st = copy(dst, static_cast<const char *>(pv[i]) + off, l, s, "hipMemcpyAsync");
            dst = static_cast<char *>(dst) + l;
            a += l;
        }
        log("pull: queued", (size_t)r, len);
        return st;
    }
    uint64_t max_send_bytes() const override { return (uint64_t)kIpcChunks * chunk_limit(); }
    gsort_status finish(hipStream_t s, gsort_status st) {
        log("finish: synchronising");
        gsort_status st2 = hip(hipStreamSynchronize(s), "hipStreamSynchronize");
        log("finish: barrier");
        if (!barrier()) return fail("barrier timeout");
        log("finish: done");
        return st != GSORT_OK ? st : st2;
    }

    gsort_status allgather(const void *send, void *recv, size_t bytes, hipStream_t s) override {
        gsort_status st = publish(send, bytes, nullptr, nullptr, s);
        if (!barrier()) return st != GSORT_OK ? st : fail("barrier timeout or a peer failed");
        for (int r = 0; r < size_ && st == GSORT_OK; ++r)
            st = pull(r, send, 0, bytes, (char *)recv + (size_t)r * bytes, s);
        return finish(s, st);
    }
    gsort_status alltoallv(const void *send, const size_t *scount, const size_t *sdispl,
                           void *recv, const size_t *rcount, const size_t *rdispl,
                           hipStream_t s) override {
        if (size_ > kIpcMaxRanks) return fail("too many ranks");
        size_t span = 0;  // what the peers read of this rank's send buffer
        for (int q = 0; q < size_; ++q)
            if (q != rank_ && scount[q]) span = std::max(span, sdispl[q] + scount[q]);
        gsort_status st = publish(send, span, scount, sdispl, s);
        if (!barrier()) return st != GSORT_OK ? st : fail("barrier timeout or a peer failed");
        for (int r = 0; r < size_ && st == GSORT_OK; ++r) {
            const IpcSlot &ps = sh_->slot[r];
            if (ps.count[rank_] != rcount[r]) { st = fail("send/recv count mismatch"); break; }
            st = pull(r, send, ps.displ[rank_], rcount[r], (char *)recv + rdispl[r], s);
        }
        return finish(s, st);
    }
    gsort_status bcast(void *buf, size_t bytes, int root, hipStream_t s) override {
        gsort_status st = publish(buf, rank_ == root ? bytes : 0, nullptr, nullptr, s);
        if (!barrier()) return st != GSORT_OK ? st : fail("barrier timeout or a peer failed");
        if (st == GSORT_OK && rank_ != root) st = pull(root, buf, 0, bytes, buf, s);
        return finish(s, st);
    }
    // every rank has mapped the control block: its name can go
    gsort_status attach(const std::string &name) {
        sh_->attached.fetch_add(1);
        if (!barrier()) return fail("not every rank attached within 120 s");
        if (rank_ == 0) {
            shm_unlink(name.c_str());
            forget_pending(name);
        }
        return GSORT_OK;
    }

  private:
    IpcShared *sh_;
    std::vector<void *> chunks_;               // this rank's staging buffer, chunk by chunk
    size_t chunk_ = 0;                         // ... of this many bytes each
    uint64_t gen_ = 0;
    std::vector<void *> stages_;               // every staging chunk this rank made
    std::vector<std::vector<void *>> peer_;    // the peers' staging chunks, opened
    std::vector<size_t> peer_chunk_;           // ... of this size
    std::vector<uint64_t> peer_gen_;           // ... at these generations
};

}  // namespace

bool is_ipc_uid(const gsort_uid *uid) {
    return uid && memcmp(uid->internal, kIpcMagic, sizeof kIpcMagic) == 0;
}

gsort_status ipc_get_uid(int nranks, gsort_uid *out) {
    if (nranks < 1 || nranks > kIpcMaxRanks) return GSORT_EINVAL;
    static std::atomic<int> seq{0};
    char name[kIpcNameMax];
    const unsigned long long t =
        (unsigned long long)std::chrono::steady_clock::now().time_since_epoch().count();
    snprintf(name, sizeof name, "/gsort_ipc_%d_%d_%llx", (int)getpid(), seq++, t & 0xffffffffull);
    std::string err;
    IpcShared *sh = map_shared(name, true, &err);
    if (!sh) return GSORT_ECOMM;
    {
        std::lock_guard<std::mutex> lk(g_shm_mu);
        if (g_shm_pending.empty()) atexit(unlink_pending);
        g_shm_pending.push_back(name);
    }
    memset(static_cast<void *>(sh), 0, sizeof(IpcShared));
    sh->n = nranks;
    munmap(sh, sizeof(IpcShared));
    memset(out, 0, sizeof(*out));
    memcpy(out->internal, kIpcMagic, sizeof kIpcMagic);
    memcpy(out->internal + kIpcNameOff, name, strlen(name) + 1);
    memcpy(out->internal + kIpcRanksOff, &nranks, sizeof nranks);
    return GSORT_OK;
}

Comm *make_ipc_comm(int rank, int nranks, const gsort_uid *uid, std::string *err) {
    int n = 0;
    memcpy(&n, uid->internal + kIpcRanksOff, sizeof n);
    if (n != nranks) {
        *err = "ipc uid made for " + std::to_string(n) + " ranks, not " + std::to_string(nranks);
        return nullptr;
    }
    char name[kIpcNameMax];
    memcpy(name, uid->internal + kIpcNameOff, kIpcNameMax);
    name[kIpcNameMax - 1] = 0;
    IpcShared *sh = map_shared(name, false, err);
    if (!sh) return nullptr;
    IpcComm *c = new IpcComm(sh, rank, nranks);
    if (c->attach(name) != GSORT_OK) {
        *err = c->err;
        delete c;
        return nullptr;
    }
    return c;
}

}  // namespace gsort
