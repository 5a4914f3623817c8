// gsort_kernels.h -- launchers for the gfx950 kernels in gsort_kernels.hip (internal).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace gsort {

// Pass geometry (gsort_kernels.hip): K3 tiles of 512 threads = 8 waves x 16 keys per thread.
constexpr int kSweepBlock = 512;
constexpr int kSweepItems = 16;
constexpr int kSweepTile = kSweepBlock * kSweepItems;  // 8192 keys per workgroup tile
constexpr int kScanGroup = 32;                           // tiles per K2a scan group
constexpr int kRadix = 256;

inline uint64_t sweep_tiles(uint64_t n) { return (n + kSweepTile - 1) / kSweepTile; }
inline uint64_t scan_groups(uint64_t n) { return (sweep_tiles(n) + kScanGroup - 1) / kScanGroup; }

// K10 canonical generator.
hipError_t launch_generate(int dist, uint64_t seed, uint64_t start, uint64_t n, int32_t *out,
                           hipStream_t s);
// K1: tcounts[tile][256] = digit (shift/8) counts of every kSweepTile-key tile (u32).  With
// hist4 != nullptr (shift must be 0) it also adds all four digit histograms of the keys into
// hist4[4][256] (u64, zeroed by the caller).  flip maps int32 input to ordered u32.
hipError_t launch_tile_counts(const uint32_t *in, uint64_t n, int shift, bool flip,
                              uint32_t *tcounts, uint64_t *hist4, hipStream_t s);
// K2: tcounts -> group-local exclusive tile offsets (in place); gsum[scan_groups(n)][256] ->
// per-group exclusive digit prefix; totals[256] = the pass's digit histogram; bases[256] =
// exclusive scan of totals.  totals and bases are device arrays of 256 u64 (required).
hipError_t launch_scan_tiles(uint32_t *tcounts, uint64_t n, uint64_t *gsum, uint64_t *totals,
                             uint64_t *bases, hipStream_t s);
// K3: one stable LSD pass over digit shift/8 using the K2 offsets; flip_in / flip_out apply
// the int32 <-> ordered-u32 map on load / store.
hipError_t launch_scatter(const uint32_t *in, uint32_t *out, uint64_t n, int shift,
                          const uint32_t *toff, const uint64_t *gpfx, const uint64_t *bases,
                          bool flip_in, bool flip_out, hipStream_t s);
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
