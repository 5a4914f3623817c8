// gsort_debug.h -- diagnostic modes of libgsort (internal; off unless the env var is set).
//
//   GSORT_SERIAL=1  every HIP operation of every context in the process (kernel launch, copy,
//                   memset, the in-process group's peer copies) runs under one process-wide
//                   mutex and is followed by hipDeviceSynchronize, so the first failing call
//                   names the operation (its source text) and rank that faulted, instead of a
//                   later, unrelated call in another thread seeing the sticky error.
//   GSORT_CANARY=1  every device buffer the library allocates gets kGuardBytes guard regions on
//                   both sides, filled with kGuardByte; after every HIP operation (with
//                   GSORT_SERIAL) or at the end of every sort call (without), the guards of all
//                   live contexts are read back and the first overwritten one is reported with
//                   the buffer name and offset.
//   GSORT_TRACE=1   every HIP operation is recorded (rank, source text, time) in a process-wide
//                   ring buffer before it is issued; the first HIP error dumps the last
//                   kTraceDump entries to stderr, i.e. the interleaving of all ranks' launches
//                   that led up to an asynchronous fault.
#pragma once
#include <hip/hip_runtime.h>

#include <mutex>

namespace gsort {

bool serial_mode();
bool canary_mode();
bool trace_mode();
std::mutex &serial_mutex();
void trace_op(int rank, const char *what);  // what: a string literal (kept by pointer)
void trace_dump(const char *why);

// Run one HIP operation; in GSORT_SERIAL mode under the process-wide mutex, then device-synced.
template <class F>
hipError_t hip_op(F &&f) {
    if (!serial_mode()) return f();
    std::lock_guard<std::mutex> lk(serial_mutex());
    hipError_t e = f();
    if (e == hipSuccess) e = hipDeviceSynchronize();
    return e;
}

constexpr size_t kGuardBytes = 16 * 1024;
constexpr unsigned char kGuardByte = 0xA5;

}  // namespace gsort
