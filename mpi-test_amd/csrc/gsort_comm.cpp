// gsort_comm.cpp -- RCCL and in-process transports (see gsort_comm.h).
#include "gsort_comm.h"

#include "gsort_debug.h"

#include <rccl/rccl.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
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
        gsort_status st = check(ncclGroupStart(), "ncclGroupStart");
        if (st != GSORT_OK) return st;
        // messages go in pieces of at most max_msg_ = 2^30 bytes (matched in order on both
        // sides): measured on MI355X with RCCL of ROCm 7.2, a self ncclSend/ncclRecv of
        // 2^30 + 256 bytes or more comes back wrong (keys missing) while 2^30-byte pieces are
        // exact (tests/test_gpu_rccl.py pins both sides of the boundary;
        // GSORT_RCCL_MAX_MSG overrides the piece size for that test)
        for (int q = 0; q < size_ && st == GSORT_OK; ++q) {
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
// In-process rank group.  Each collective: every rank synchronises its stream (its send data
// is complete), publishes pointers, meets the others at a barrier, pulls what it needs with
// hipMemcpyAsync on its own stream, synchronises, and meets them again (so no sender reuses a
// buffer a peer is still reading).
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
    explicit GroupState(int n_) : n(n_), ptr(n_), count(n_), displ(n_) {}
};

GroupState *group_state_create(int nranks) { return new GroupState(nranks); }
void group_state_destroy(GroupState *g) { delete g; }
int group_state_size(const GroupState *g) { return g->n; }

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

    gsort_status allgather(const void *send, void *recv, size_t bytes, hipStream_t s) override {
        gsort_status st = hip([&] { return hipStreamSynchronize(s); }, "hipStreamSynchronize");
        if (st != GSORT_OK) return st;
        g_->ptr[rank_] = send;
        if (!barrier()) return fail("barrier timeout");
        for (int r = 0; r < size_ && st == GSORT_OK; ++r)
            if (bytes)
                st = hip([&] {
                    return hipMemcpyAsync((char *)recv + (size_t)r * bytes, g_->ptr[r], bytes,
                                          hipMemcpyDeviceToDevice, s);
                }, "hipMemcpyAsync");
        if (st == GSORT_OK) st = hip([&] { return hipStreamSynchronize(s); }, "hipStreamSynchronize");
        if (!barrier()) return fail("barrier timeout");
        return st;
    }
    gsort_status alltoallv(const void *send, const size_t *scount, const size_t *sdispl,
                           void *recv, const size_t *rcount, const size_t *rdispl,
                           hipStream_t s) override {
        gsort_status st = hip([&] { return hipStreamSynchronize(s); }, "hipStreamSynchronize");
        if (st != GSORT_OK) return st;
        g_->ptr[rank_] = send;
        g_->count[rank_] = scount;
        g_->displ[rank_] = sdispl;
        if (!barrier()) return fail("barrier timeout");
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
        gsort_status st2 = hip([&] { return hipStreamSynchronize(s); }, "hipStreamSynchronize");
        if (!barrier()) return fail("barrier timeout");
        return st != GSORT_OK ? st : st2;
    }
    gsort_status bcast(void *buf, size_t bytes, int root, hipStream_t s) override {
        gsort_status st = hip([&] { return hipStreamSynchronize(s); }, "hipStreamSynchronize");
        if (st != GSORT_OK) return st;
        g_->ptr[rank_] = buf;
        if (!barrier()) return fail("barrier timeout");
        if (rank_ != root && bytes)
            st = hip([&] {
                return hipMemcpyAsync(buf, g_->ptr[root], bytes, hipMemcpyDeviceToDevice, s);
            }, "hipMemcpyAsync");
        gsort_status st2 = hip([&] { return hipStreamSynchronize(s); }, "hipStreamSynchronize");
        if (!barrier()) return fail("barrier timeout");
        return st != GSORT_OK ? st : st2;
    }

  private:
    GroupState *g_;
};

Comm *make_group_comm(GroupState *g, int rank) { return new GroupComm(g, rank); }

}  // namespace gsort
