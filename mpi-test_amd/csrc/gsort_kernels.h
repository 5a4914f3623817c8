// gsort_kernels.h -- launchers for the gfx950 kernels in gsort_kernels.hip (internal).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace gsort {

// Onesweep geometry (gsort_kernels.hip): 512 threads = 8 waves, 16 keys per thread.
constexpr int kSweepBlock = 512;
constexpr int kSweepItems = 16;
constexpr int kSweepTile = kSweepBlock * kSweepItems;  // 8192 keys per workgroup tile
constexpr int kRadix = 256;

// Status word of the decoupled lookback: [63:48] epoch, [47:46] flag, [45:0] count.
constexpr uint64_t kFlagAgg = 1, kFlagInc = 2;

inline uint64_t sweep_tiles(uint64_t n) { return (n + kSweepTile - 1) / kSweepTile; }

// K10 canonical generator.
hipError_t launch_generate(int dist, uint64_t seed, uint64_t start, uint64_t n, int32_t *out,
                           hipStream_t s);
// K1: all four 8-bit digit histograms of (key ^ 0x80000000) in one read; hist[4][256] u64
// must be zeroed by the caller.
hipError_t launch_hist4(const uint32_t *in, uint64_t n, uint64_t *hist, hipStream_t s);
// K3: one stable onesweep pass over digit `shift/8`.  base[256] = exclusive digit offsets
// for this pass (u64).  status: >= tiles*256 words, tile_ctr: one zeroed u32.  A lookback
// that spins past its bound sets *err (and the pass output is garbage) instead of hanging.
// flip_in / flip_out apply the int32 <-> ordered-u32 map on load / store.
hipError_t launch_onesweep(const uint32_t *in, uint32_t *out, uint64_t n, int shift,
                           const uint64_t *base, uint64_t *status, uint32_t *tile_ctr,
                           uint32_t *err, uint32_t epoch, bool flip_in, bool flip_out,
                           hipStream_t s);
// K8 receive-side placement: segs[k] = {src_off (in recv buffer), dst_off, len}; copies the
// segments into out and (if hist != nullptr) accumulates the 256-bin histogram of digit
// `next_shift/8` of the placed keys (ordered-u32 form); flip_out maps back to int32 on store.
hipError_t launch_place(const uint32_t *recv, uint32_t *out, const uint64_t *segs, int nseg,
                        uint64_t n_out, uint64_t *hist, int next_shift, bool flip_out,
                        hipStream_t s);
// K9 fingerprint: acc[0] += sum mix64(key), acc[1] ^= xor, acc[2] += #descents; acc zeroed.
hipError_t launch_fingerprint(const int32_t *keys, uint64_t n, unsigned long long *acc,
                              hipStream_t s);
// K4 regular sampling: out[i] = sorted[i * interval], i < k (caller checks bounds).
hipError_t launch_regular_sample(const int32_t *sorted, uint64_t interval, int k,
                                 int32_t *out, hipStream_t s);
// K5 splitter selection: sort m <= 1024 samples in LDS, splitters[i] = S[(i+1)*k].
hipError_t launch_select_splitters(const int32_t *samples, int m, int k, int nsplit,
                                   int32_t *splitters, hipStream_t s);
// K6 bucket bounds on a sorted block: bounds[j] = #keys <= splitters[j] (j < nsplit).
hipError_t launch_bucket_bounds(const int32_t *sorted, uint64_t n, const int32_t *splitters,
                                int nsplit, uint64_t *bounds, hipStream_t s);
// Plain device copy kernel (used when a sort has no non-trivial pass).
hipError_t launch_copy(const uint32_t *in, uint32_t *out, uint64_t n, hipStream_t s);

}  // namespace gsort
