// gsort_comm.h -- the rank-to-rank transport of libgsort (internal).
//
// Replaces the reference's MPI point-to-point loops (mpi_radix_sort.c:150-173,
// mpi_sample_sort.c:100-133, :160-170) and its rank-0 Scatter/Gather(v).  Three transports:
//   RcclComm   one process per GPU, RCCL over xGMI: grouped ncclSend/ncclRecv for the
//              all-to-all-v and the gather, ncclAllGather, ncclBroadcast.
//   GroupComm  P contexts driven by P threads of one process (in-process rank group),
//              moving bytes with device-to-device hipMemcpyAsync; lets the distributed
//              algorithm run with P ranks on a single GPU.
//   IpcComm    one process per rank on one node, any number of ranks per GPU: peers' buffers
//              opened through HIP IPC handles, a POSIX shared-memory control block; lets the
//              drop-in programs run under `mpirun -np P` with fewer GPUs than ranks.
// Every call is collective over the P ranks and blocking on return w.r.t. `stream` ordering
// (data is valid on `stream` when the call returns).  Byte counts are size_t.
#pragma once
#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

#include <string>

#include "gsort.h"

namespace gsort {

class Comm {
  public:
    virtual ~Comm() {}
    int rank() const { return rank_; }
    int size() const { return size_; }
    // recv[r*bytes .. ) = rank r's send (bytes each)
    virtual gsort_status allgather(const void *send, void *recv, size_t bytes,
                                   hipStream_t s) = 0;
    // rank r's send + sdispl[q] (scount[q] bytes) lands in rank q's recv + rdispl[r]
    virtual gsort_status alltoallv(const void *send, const size_t *scount, const size_t *sdispl,
                                   void *recv, const size_t *rcount, const size_t *rdispl,
                                   hipStream_t s) = 0;
    virtual gsort_status bcast(void *buf, size_t bytes, int root, hipStream_t s) = 0;
    // the largest send range (bytes of one rank's send buffer its peers read in one alltoallv)
    // the transport carries: the IPC group's staging limit, unbounded otherwise
    virtual uint64_t max_send_bytes() const { return ~0ull; }
    std::string err;

  protected:
    int rank_ = 0, size_ = 1;
};

Comm *make_rccl_comm(int rank, int nranks, const gsort_uid *uid, std::string *err);
gsort_status runtime_info(gsort_runtime_info_t *out);  // gsort_runtime_info
gsort_status rccl_get_uid(gsort_uid *out);
// Same-node process group over HIP IPC (gsort_get_uid_ipc): one process per rank, any number
// of ranks per GPU.
bool is_ipc_uid(const gsort_uid *uid);
gsort_status ipc_get_uid(int nranks, gsort_uid *out);
Comm *make_ipc_comm(int rank, int nranks, const gsort_uid *uid, std::string *err);

struct GroupState;  // opaque; gsort_group wraps it
Comm *make_group_comm(GroupState *g, int rank);
GroupState *group_state_create(int nranks);
void group_state_destroy(GroupState *g);
int group_state_size(const GroupState *g);
// The group's device: the first rank to join sets it, a rank on another device is refused (the
// group's ordering events are device-scope).  false: refused.
bool group_state_join(GroupState *g, int device);

}  // namespace gsort
