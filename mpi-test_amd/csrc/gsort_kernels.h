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
constexpr int kPartBlock = 1024;                         // K3u: 1024 threads x 8 keys per tile
constexpr int kRadix = 256;

// Kernel-attached timing (gsort_kernels.hip, launch_k): while a timer is set on a thread, every
// kernel that thread launches records its end into a fresh event from make(u) (last_stop).
struct LaunchTimer {
    hipEvent_t last_stop = nullptr;
    hipEvent_t (*make)(void *) = nullptr;
    void *u = nullptr;
};
void set_launch_timer(LaunchTimer *t);  // nullptr: untimed launches

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
// the int32 <-> ordered-u32 map on load / store.  vin != nullptr: a key-value pass (value
// vin[i] travels with key i into vout; no flips).
hipError_t launch_scatter(const uint32_t *in, uint32_t *out, uint64_t n, int shift,
                          const uint32_t *toff, const uint64_t *gpfx, const uint64_t *bases,
                          bool flip_in, bool flip_out, hipStream_t s,
                          const uint32_t *vin = nullptr, uint32_t *vout = nullptr);
// K8 receive-side placement: segs[k] = {src_off (in recv buffer), dst_off, len}; copies the
// segments into out and (if hist != nullptr) accumulates the 256-bin histogram of digit
// `next_shift/8` of the placed keys (ordered-u32 form); flip_out maps back to int32 on store.
hipError_t launch_place(const uint32_t *recv, uint32_t *out, const uint64_t *segs, int nseg,
                        uint64_t n_out, uint64_t *hist, int next_shift, bool flip_out,
                        hipStream_t s);
// K9 fingerprint: acc[0] += sum mix64(key), acc[1] ^= xor, acc[2] += #descents; acc zeroed.
hipError_t launch_fingerprint(const int32_t *keys, uint64_t n, unsigned long long *acc,
                              hipStream_t s);
// K13: out[i] = #keys of the sorted int32 block whose ordered-u32 form is < xs[i] (i < m).
hipError_t launch_count_below(const int32_t *sorted, uint64_t n, const uint64_t *xs, int m,
                              uint64_t *out, hipStream_t s);
// K4 regular sampling: out[i] = sorted[i * interval], i < k (caller checks bounds).
hipError_t launch_regular_sample(const int32_t *sorted, uint64_t interval, int k,
                                 int32_t *out, hipStream_t s);
// K5 splitter selection: sort m <= 1024 samples in LDS, splitters[i] = S[(i+1)*k].
hipError_t launch_select_splitters(const int32_t *samples, int m, int k, int nsplit,
                                   int32_t *splitters, hipStream_t s);
// K6 bucket bounds on a sorted block: bounds[j] = #keys <= splitters[j] (j < nsplit).
hipError_t launch_bucket_bounds(const int32_t *sorted, uint64_t n, const int32_t *splitters,
                                int nsplit, uint64_t *bounds, hipStream_t s,
                                bool strict = false);
// ---- MSD partition sort (gsort_kernels.hip, "MSD partition sort") -----------------------
// K11 geometry: one workgroup sorts a bucket entirely in LDS.  A stable pass costs a wave
// ~16 rounds of 64 keys best (measured, tools/kexp3.hip), so the workgroup size follows the
// bucket size: class 1 = 256 threads x 18 keys, class 2 = 512 x 18, class 3 = 512 x 32,
// class 4 = 1024 x 32 (one workgroup per CU: 144 KiB of LDS).  Class 4 keeps the children of a
// level-2 bucket in one pass when they outgrow 16 384 keys (2^29 31-bit keys, 2^28 30-bit
// keys): without it each went through a level-1 partition into ~64-key buckets (3.7x slower
// sort, tools/run_length_probe.py).
constexpr int kLocalClasses = 4;
constexpr uint64_t kLocalCap[kLocalClasses + 1] = {0, 256 * 18, 512 * 18, 512 * 33, 1024 * 32};
constexpr uint64_t kLocalMax = kLocalCap[kLocalClasses];
// Sampled-plan children past class 3 (16 897 .. 32 768 keys, e.g. 29-bit keys at 2^28) go to
// K18c (K12g's list 0) with the oversized ones, as the receive side's class 4 does
// (GSORT_RECV_CX): 2^28 29-bit keys K11 0.67 -> 0.56 ms (profiles/r04_ab_est_class4_k18c.txt).
// Not on a plan shifted by 8 or more bits (sb >= 8): K11e then sorts one digit in one pass,
// where K18c still walks 65 536 counters per child (Gaussian 2^28: K11 0.52 -> 1.05 ms).
constexpr int kEstCx = 4;
inline int local_class(uint64_t len) {
    for (int k = 1; k <= kLocalClasses; ++k)
        if (len <= kLocalCap[k]) return k;
    return 0;
}

// K1 without the all-digit histograms: one block per tile (tcounts as launch_tile_counts).
hipError_t launch_tile_counts1(const uint32_t *in, uint64_t n, int shift, bool flip,
                               uint32_t *tcounts, hipStream_t s);
// K3u, level 3: unstable partition of global tiles by digit shift/8 (offsets from K1/K2).
hipError_t launch_partition(const uint32_t *in, uint32_t *out, uint64_t n, int shift,
                            const uint32_t *toff, const uint64_t *gpfx, const uint64_t *bases,
                            bool flip_in, hipStream_t s);
// Work lists of child buckets: list[0] = next level (> kLocalMax keys), list[k] = K11 class k
// (kLocalCap[k-1] < len <= kLocalCap[k]).  Each list is u64 pairs {start, len};
// ctr[3*i .. 3*i+2] = {entries, keys, longest} of list i.  ctr == nullptr: no classification
// (the last level).
struct WorkLists {
    uint64_t *list[kLocalClasses + 1];
    uint64_t *ctr;
    bool force_next;  // every non-empty child to list[0]
};
// The 256 level-3 buckets {bases[d], totals[d]} -> work lists.
hipError_t launch_classify_buckets(const uint64_t *bases, const uint64_t *totals,
                                   const WorkLists &wl, hipStream_t s);
// One segmented level: partition every segment of `segs` by digit shift/8 (in -> out, same
// positions), children classified into `lists`.  Device scratch sized by the caller for
// max_tiles >= tiles of all segments and max_groups >= their scan groups.
struct SegPass {
    const uint32_t *in;
    uint32_t *out;
    const uint64_t *segs;
    uint32_t nseg;
    int shift;
    bool flip_out;
    bool flip_in = false;          // in is the int32 input (first level of a sort that starts there)
    uint32_t max_tiles, max_groups;
    uint32_t *tpfx, *gpfx;         // nseg + 1 each
    uint32_t *segmap, *groupmap;   // max_tiles / max_groups
    uint32_t *tcounts;             // max_tiles x 256
    uint64_t *gsum;                // max_groups x 256
    uint64_t *cstart;              // nseg x 256
    WorkLists lists;
    uint16_t *out16 = nullptr;     // set: K3u stores the low 16 bits of every key here
};
// K12 + K1s + K2s: plan the tiles, count them, scan, child starts + classification.
hipError_t launch_seg_count(const SegPass &sp, hipStream_t s);
// K3u over the planned segment tiles (after launch_seg_count).
hipError_t launch_seg_partition(const SegPass &sp, hipStream_t s);
// ---- two-level plan front end (gsort_kernels.hip, "Two-level plan") ----------------------
// K1h workgroups (at most; one per CU) and the size of their partial 16-bit histograms (u32).
constexpr uint32_t kH16Blocks = 256;
constexpr size_t kH16PartWords = 32768;
constexpr uint32_t kH16Shards = 8;  // level-3 cursors / wrap repairs per XCD shard
// K1h: per-workgroup packed histograms of the top 16 bits (ordered u32) into part (nblk x
// kH16PartWords u32), wrap repairs into fix (kH16Shards x 65536 u64, zeroed by the caller).
// Returns the workgroup count (a multiple of kH16Shards) in *nblk.
hipError_t launch_hist16(const uint32_t *in, uint64_t n, bool flip, uint32_t *part, uint64_t *fix,
                         uint32_t *nblk, hipStream_t s);
// K12a + K12b: from the K1h partials, ccount (65536 child counts), t3 (kH16Shards x 256 level-3
// counts per shard), tot (256), then bases / totals (256 u64 each: the level-3 buckets),
// cstart (65537 u64: the 16-bit bucket bounds, cstart[65536] = n), the level-2 child cursors
// cur (65536 u32, from their bucket's start), the level-3 cursors cur3 (kH16Shards x 256 u32,
// from their bucket's start), the K3a tile plan tpfx (257 u32) and the work lists (wl2:
// children of level-2 buckets; wl3: level-3 buckets finished by K11; ctr == nullptr: not
// filled).  force: every non-empty level-3 bucket is a level-2 bucket.
// K12a leaves fix zeroed for the next K1h and zeroes zero[0 .. nzero) (<= 256 u64: the
// work-list counters) before K12b counts into them.
hipError_t launch_plan16(const uint32_t *part, uint32_t nblk, uint64_t *fix, uint64_t n,
                         bool force, uint64_t *ccount, uint64_t *t3, uint64_t *tot,
                         uint64_t *bases, uint64_t *totals, uint64_t *cstart, uint32_t *cur,
                         uint32_t *cur3, uint32_t *tpfx, const WorkLists &wl2,
                         const WorkLists &wl3, uint64_t *zero, uint32_t nzero, uint32_t *flags,
                         hipStream_t s);
// K12p: dst[0 .. n) = src[0 .. n) in pinned host memory, then *flag = seq (system release).
hipError_t launch_publish(const uint64_t *src, uint32_t n, uint64_t *dst, uint64_t *flag,
                          uint64_t seq, hipStream_t s);
// K3r: level 3 of the int32 input by the top digit into out (ordered u32), runs reserved on cur3.
// flags (K12b's trivial-level word, or nullptr): see k_partition_res.
hipError_t launch_partition3r(const uint32_t *in, uint32_t *out, uint64_t n, uint32_t *cur3,
                              const uint64_t *bases, const uint32_t *flags, hipStream_t s);
// K12c + K3a: level 2 of every level-2 bucket (in = level 3's output, ordered u32) by digit 2
// into out (ordered u32), or with out16 != nullptr only the low 16 bits into out16.  tdesc:
// scratch for kTileDescBytes per level-2 tile (sweep_tiles(n) + 256 tiles).
constexpr size_t kTileDescBytes = 16;
hipError_t launch_partition2r(const uint32_t *in, uint32_t *out, uint16_t *out16, uint64_t n,
                              const uint32_t *tpfx, void *tdesc, const uint64_t *bases,
                              const uint64_t *totals, uint32_t *cur, const uint32_t *flags,
                              const uint32_t *raw, hipStream_t s);
// K11: sort each listed bucket (all of class cls: <= kLocalCap[cls] keys) on digits
// 0..ndigits-1 in LDS, store as int32 into out (same positions; in == out allowed).
// flip_in: the input is int32 (else ordered u32).  atomic_rank: stable ranks from LDS atomics
// (lane-order property, checked at context creation by launch_lds_order_check), else from
// wave64 ballots.
hipError_t launch_local_sort(const uint32_t *in, uint32_t *out, const uint64_t *list,
                             uint32_t nlist, int cls, int ndigits, bool flip_in,
                             bool atomic_rank, hipStream_t s);
// K18: receive buckets of kLocalMax < len <= kHxMax keys (list {h, len}), a counting sort of
// their low 16 bits written straight from the counts, int32 at out[bstart[h] ..).
constexpr uint64_t kHxMax = 1u << 20;
hipError_t launch_hist_expand(const void *recv, bool packed16, const uint64_t *pos,
                              const uint64_t *roff, int P, const uint64_t *bstart,
                              const uint64_t *list, uint32_t nlist, uint32_t *out,
                              hipStream_t s);
// K18c: the same buckets (any list of {h, len} entries with len <= kHxMax) in one read: packed
// u16 bin counters, wave-wise expansion by marked slots + max-scan, coalesced stores; one
// persistent workgroup per CU (ncu), the next bucket's keys loaded during this one's stores.
// fb_list != nullptr: u8 bins (64 KiB, two workgroups per CU); a bucket with >= 256 copies of
// one key (a byte wrapped) is appended to fb_list (count at fb_ctr, zeroed by the caller) and
// not written; the caller then runs the u16 form over fb_list with nlist_dev = fb_ctr (the
// list's length read on the device, nlist = its bound: the grid).
hipError_t launch_count_expand(const void *recv, bool packed16, const uint64_t *pos,
                               const uint64_t *roff, int P, const uint64_t *bstart,
                               const uint64_t *list, uint32_t nlist, int ncu, uint32_t *out,
                               hipStream_t s, uint64_t *fb_list = nullptr,
                               uint32_t *fb_ctr = nullptr, const uint32_t *nlist_dev = nullptr);
// K18c's work as several {h, len} lists walked as one index space (round 5: the class-4 list and
// list 0 in one persistent launch instead of two launches with a tail each).  List q holds n[q]
// entries or, with ndev[q] set, the count read on the device (n[q] is then only the grid's
// bound): the u8 kernel's wrapped buckets, redone by a u16 launch queued right behind it.
// skip: a list left out on the device when *skip_max > kHxMax (list 0, whose oversized buckets
// take the MSD levels), -1: none.
constexpr int kCxLists = 5;
struct CxLists {
    const uint64_t *list[kCxLists] = {};
    const uint32_t *ndev[kCxLists] = {};
    uint32_t n[kCxLists] = {};
    int nl = 0;
    int skip = -1;
    const uint64_t *skip_max = nullptr;
    void add(const uint64_t *l, uint32_t cnt, const uint32_t *dev = nullptr) {
        list[nl] = l; n[nl] = cnt; ndev[nl] = dev; ++nl;
    }
    uint32_t bound() const {
        uint32_t t = 0;
        for (int q = 0; q < nl; ++q) t += n[q];
        return t;
    }
};
hipError_t launch_count_expand_lists(const void *recv, bool packed16, const uint64_t *pos,
                                     const uint64_t *roff, int P, const uint64_t *bstart,
                                     const CxLists &cl, int ncu, uint32_t *out, hipStream_t s,
                                     uint64_t *fb_list = nullptr, uint32_t *fb_ctr = nullptr);
// {h, len} list entries -> {bstart[h], len}.
hipError_t launch_list_to_segments(uint64_t *list, uint32_t n, const uint64_t *bstart,
                                   hipStream_t s);
// ---- packed send buffer of the distributed radix (low 16 bits, grouped by the top 16) -----
// out[i] = int32 key of bucket h from its low 16 bits in[i].
hipError_t launch_unpack16(const uint16_t *in, uint64_t n, uint32_t h, int32_t *out,
                           hipStream_t s);
// gb[h] (65537 u64) = first position of 16-bit bucket h, from level 3's bases / totals and
// level 2's segments (list0) and child starts.
hipError_t launch_gb_from_plan(const uint64_t *bases, const uint64_t *totals,
                               const uint64_t *segs, uint32_t nseg, const uint64_t *cstart,
                               uint64_t n, uint64_t *gb, hipStream_t s);
// K13s: one radix-select round decided on the device (boundary q: prefix[q] += the largest
// digit d whose all-gathered count of keys below prefix[q] + (d << shift) stays <= g[q]; the
// next round's M thresholds prefix[q] + (d << (shift - 8)) written to xs).
// all: P rows of W u64 (boundary q's M counts at q * M); shift 0 (the last round) writes no xs.
hipError_t launch_select_digit(const uint64_t *all, int W, const uint64_t *g, uint64_t N, int P,
                               int nb, int M, int shift, uint64_t *prefix, uint64_t *xs,
                               hipStream_t s);
// K13g: block q sorts boundary q's 16-bit group (prefix[q] >> 16, known after the second select
// round) in place in the packed buffer (u16 low halves; gb = the block's 16-bit bucket bounds);
// big[q] = 1 if its group holds more than 32 768 keys (left unsorted: the caller's host path),
// else 0 (nb flags).
hipError_t launch_boundary_sort16(uint16_t *pack, const uint64_t *gb, const uint64_t *prefix,
                                  const uint64_t *g, uint64_t N, int nb, bool atomic_rank,
                                  uint64_t *big, hipStream_t s);
// Sample sort on the grouped block: K4g pref[i] = (16-bit group of position
// i * interval) << 16, g[i] = 0, i < k <= 128 (K13g's inputs: it then sorts those groups);
// K4r out[i] = the int32 key at position i * interval (its group sorted); K6g splitter j's
// group (pref, g) and count_below16 thresholds xs[j] = ord(s_j) + 1, xs[S + j] = ord(s_j).
hipError_t launch_sample_groups(const uint64_t *gb, uint64_t interval, int k, uint64_t *pref,
                                uint64_t *g, hipStream_t s);
hipError_t launch_read_samples16(const uint16_t *pack, const uint64_t *pref, uint64_t interval,
                                 int k, int32_t *out, hipStream_t s);
hipError_t launch_splitter_groups(const int32_t *spl, int S, uint64_t *pref, uint64_t *g,
                                  uint64_t *xs, hipStream_t s);
// K13 on the packed buffer (bucket bounds gb): out[i] = #keys < xs[i] (ordered u32).
hipError_t launch_count_below16(const uint16_t *a, const uint64_t *gb, const uint64_t *xs,
                                int m, uint64_t *out, hipStream_t s);
// ---- receive side of the distributed sorts: P sorted runs -> one sorted block -----------
constexpr uint32_t kBuckets16 = 65536;  // buckets by the top 16 bits (ordered u32)
// pos[p][h] (P x 65537 u64) = keys of run p (recv[roff[p] .. +rlen[p]), int32, grouped by
// the top 16 bits) below bucket h, by binary search.
hipError_t launch_run_bounds(const int32_t *recv, const uint64_t *roff, const uint64_t *rlen,
                             int P, uint64_t *pos, hipStream_t s);
// pos[p][h] from source p's counts of buckets [h_lo, h_lo + nh) at meta + moff[p]
// (moff[p] = ~0: nothing received from p) -- the packed exchange.
// scratch: 64 x P u64.
// pos (as launch_pos_from_meta) and bstart[0 .. 65536] (exclusive scan of every bucket's total
// over the sources) in ONE single-pass decoupled-lookback row scan of P + 1 rows (K15s); classify
// then takes bsize = nullptr (sizes from bstart).  scratch: kRecvScanStatusWords status words
// and a u32 ticket after them, both zero before a context's first scan; epoch: a number the
// caller changes every call.  zero[0 .. nzero) (<= 1024 u64) is cleared by the kernel (the
// work-list counters the classification adds into).
constexpr size_t kRecvScanStatusWords = 65 * 64;
hipError_t launch_recv_plan_from_meta(const uint32_t *meta, const uint64_t *moff, uint32_t h_lo,
                                     uint32_t nh, int P, uint64_t *pos, uint64_t *bstart,
                                     uint64_t *scratch, hipStream_t s, uint64_t *zero,
                                     uint32_t nzero, uint32_t epoch);
hipError_t launch_pos_from_meta(const uint32_t *meta, const uint64_t *moff, uint32_t h_lo,
                                uint32_t nh, int P, uint64_t *pos, uint64_t *scratch,
                                hipStream_t s);
// bsize / bstart (65536 u64) = bucket sizes and their exclusive scan; buckets classified into
// wl as {h | bstart[h] << 16, len} entries (the K11g classes and list 0; list_to_segments turns
// list 0 into {bstart, len} segments).
hipError_t launch_recv_classify(const uint64_t *pos, int P, uint64_t *bsize, uint64_t *bstart,
                                const WorkLists &wl, uint64_t *scratch, hipStream_t s);
// The two halves of launch_recv_classify (the distributed radix classifies only its own bucket
// range): bucket sizes + starts, then the work lists of the buckets [h0, h1) only.
hipError_t launch_recv_bounds(const uint64_t *pos, int P, uint64_t *bsize, uint64_t *bstart,
                              uint64_t *scratch, hipStream_t s);
hipError_t launch_classify_range(const uint64_t *bsize, const uint64_t *bstart,
                                 const WorkLists &wl, uint32_t h0, uint32_t h1, hipStream_t s);
// K11g: gather the P pieces of every listed bucket (int32 keys, or packed16: the low 16 bits),
// sort its low 16 bits in LDS, store int32 at out[bstart[h] ..).  Entries first .. first +
// nlist - 1; with ndev, only those below the count *ndev read on the device (nlist is then the
// grid: a guess made before the host knew the list's length).
hipError_t launch_gather_sort(const void *recv, bool packed16, const uint64_t *pos,
                              const uint64_t *roff, int P, const uint64_t *bstart,
                              const uint64_t *list, uint32_t nlist, int cls, bool atomic_rank,
                              uint32_t *out, hipStream_t s, const uint32_t *ndev = nullptr,
                              uint32_t first = 0);
// Copy the pieces of every bucket of more than min_len keys to out[bstart[h] ..) as ordered u32
// or, as_int32, int32 (one block per 64 Ki output positions; n_out = bstart[65536]).
hipError_t launch_gather_copy(const void *recv, bool packed16, const uint64_t *pos,
                              const uint64_t *roff, int P, const uint64_t *bstart, uint64_t n_out,
                              uint32_t *out, hipStream_t s, uint64_t min_len = kLocalMax,
                              bool as_int32 = false);
// Sender of the packed exchange: out[i] = low 16 bits of a[i]; meta counts per destination
// range (rng: nrng x {a, b, h_lo, nh, out_off}; gb = 65537 bucket bounds of the block).
hipError_t launch_pack16(const int32_t *a, uint64_t n, uint16_t *out, hipStream_t s);
hipError_t launch_meta_counts(const uint64_t *gb, const uint64_t *rng, int nrng, uint32_t *meta,
                              hipStream_t s);
// Lane-order self-check: nblocks x 512 threads x 16 digits from `digits` (mod nbins);
// bad[0] += violations (zeroed by the caller).
hipError_t launch_lds_order_check(const uint32_t *digits, uint32_t nblocks, uint32_t nbins,
                                  uint64_t *bad, hipStream_t s);
// Streaming copy of `bytes` (multiple of 16, 16-B aligned): one block per 16 KiB chunk, 16 B
// per lane, nontemporal stores -- the bench's read + write ceiling.
hipError_t launch_stream_copy(const void *in, void *out, uint64_t bytes, hipStream_t s);
// Reference-compat key map: K20 mm[0] = min(mm[0], keys), mm[1] = max(..)
// (mm preset by the caller); K19 key[i] = the mixed-radix number of the reference's base-P
// digits 1..loop of |a[i]| (mod[d] = the reference's (int)pow(P, d+1) as x86 converts it,
// scale[d] = pow(P, d)); bad[0] += keys the reference would put outside its buckets.
hipError_t launch_minmax(const int32_t *a, uint64_t n, int *mm, hipStream_t s);
hipError_t launch_compat_keys(const int32_t *a, uint64_t n, int P, int loop, const int *mod,
                              const double *scale, uint32_t *key, uint64_t *bad, hipStream_t s);
// ---- sampled plan (gsort_kernels.hip, "Sampled plan") -----------------------
// Levels 3 and 2 sized from a 1/64 sample instead of K1h's full histogram: in (int32) ->
// level 3 into the gapped regions of x -> level 2 into the gapped regions of y -> K11e into
// out (int32, exact positions).  eflag[0] bit 2: ineligible (nothing past the plan ran);
// eflag[1]: a region overflowed (the output is wrong).  Either way the caller re-sorts on the
// exact plan; both are known once K12g has run (the runtime reads them with the K11e list
// counts).  Sizes (u32 unless noted): part8 kEstWGs x 16384, part3 kEstWGs x 2048, msamp
// 4 x kEstWGs, capc / cur2 / lim2 / init2 65536, cap3 / cur3 / lim3 / init3 2048, r2 / r3 / bases3 /
// bases2 256 u64, tp 257, tdesc (est_max_tiles(n) + 2048) x kTileDescBytes (tile descriptors,
// then the 2048-entry level-3 piece table), dump kSweepTile keys;
// wl.list[1..4] 65536 entries each, wl.ctr the 15 counters (zeroed by the front).
#ifndef GSORT_EST_WGS
#define GSORT_EST_WGS 256
#endif
constexpr uint32_t kEstWGs = GSORT_EST_WGS;
constexpr uint32_t kEstBlockKeysHost = 512;  // one 8-key sample segment per block
constexpr uint64_t kEstMinKeys = 1ull << 22;   // below: too few samples per child
constexpr uint64_t kEstMaxKeys = 1ull << 31;   // level-3 regions stay below 2^32 keys
inline uint64_t est_max_tiles(uint64_t n) { return sweep_tiles(n) + 256; }
struct EstPlan {
    const uint32_t *in;
    uint64_t n;
    bool flip_in;
    uint32_t *x, *out;
    uint16_t *y;          // level 2's regions: the low 16 bits of every key
    uint64_t capx, capy;  // keys of x and y
    uint32_t *part8, *part3, *msamp;
    uint32_t *capc, *cap3;
    uint64_t *r2, *r3, *bases3, *bases2;
    uint32_t *cur2, *lim2, *init2, *cur3, *lim3, *init3;
    uint32_t *tp;
    void *tdesc;
    uint32_t *dump;
    uint32_t *eflag;
    WorkLists wl;
    double slack;
    bool atomic_rank;
    // pinned host mailbox (device pointer) and the sequence numbers K12e-b / K12g publish with:
    // mail[2] eligibility word, mail[4] the children with samples, mail[5] the key bits that
    // vary among the samples, mail[6] / mail[7] their min / max, mail[23] the samples of the
    // largest child, mail[3] = seq_elig;
    // mail[0] status {eflag, ovf}, mail[8 .. 23)
    // the K11e list counters, mail[1] = seq_done
    uint64_t *mail;
    uint64_t seq_elig, seq_done;
    int sb;         // 0 .. 16: the levels' digits start sb bits lower (a constant key prefix)
    uint32_t koff;  // keys taken as ordered u32 minus koff (the offset retry; 0 otherwise)
};
constexpr uint32_t kEstMailWords = 24;
hipError_t launch_est_front(const EstPlan &p, hipStream_t s);   // K1e + K12e
hipError_t launch_est_level3(const EstPlan &p, hipStream_t s);  // K3r
hipError_t launch_est_level2(const EstPlan &p, hipStream_t s);  // K12f + K3a
hipError_t launch_est_classify(const EstPlan &p, hipStream_t s);  // K12g
// K11e over entries [first, first + nlist) of class list cls (those at or past the count K12g
// made return at once); publish: its block 0 first hands K12g's counters and status to the
// host (mail, seq_done) -- exactly one launch behind K12g must, or launch_est_publish
hipError_t launch_local_sort_e(const EstPlan &p, int cls, uint32_t first, uint32_t nlist,
                               bool publish, hipStream_t s);
hipError_t launch_est_publish(const EstPlan &p, hipStream_t s);
// K18c over K12g's list 0: the children past kLocalMax keys (one-read counting sort from Y)
hipError_t launch_est_oversized(const EstPlan &p, uint32_t nlist, int ncu, hipStream_t s);
// ---- one dominant 16-bit child (gsort_kernels.hip, "giant child") -----------
// K1m: res[0] = the most frequent top-16-bit child (ordered u32) of min(n, 16384) evenly
// strided keys, res[1] = its sample count, res[2] = the samples (u64 each).
hipError_t launch_est_mode(const uint32_t *in, uint64_t n, uint64_t *res, hipStream_t s);
// K1g: child `child`'s keys (int32 input) into per-workgroup packed histograms of their low 16
// bits (part: g x kH16PartWords u32; fix: kH16Shards x 65536 u64, zero on entry, as K1h), every
// other key copied into its workgroup's segment cold + b * wg_cap; ctr[1 + b] = segment b's
// keys, ctr[0] = the cold keys below the child.  ctr (1 + g u64) zeroed by the caller; cold
// holds g * wg_cap keys (giant_wg_cap: g workgroups, a multiple of 8 up to kH16Blocks, each
// taking at most wg_cap keys).
inline uint64_t giant_wg_cap(uint64_t n, uint32_t *g) {
    const uint64_t pairs = (sweep_tiles(n) + 1) / 2;
    const uint64_t g8 = (pairs + kH16Shards - 1) / kH16Shards * kH16Shards;
    const uint64_t gg = g8 < kH16Blocks ? g8 : kH16Blocks;
    *g = (uint32_t)gg;
    return (pairs + gg - 1) / gg * 2 * kSweepTile;
}
hipError_t launch_giant_hist(const uint32_t *in, uint64_t n, uint32_t child, uint32_t *part,
                             uint64_t *fix, uint32_t *cold, uint64_t *ctr, hipStream_t s);
// K1g's segments gathered into out[0, sum ctr[1..g]) in workgroup order.
hipError_t launch_giant_gather(const uint32_t *cold, uint64_t n, const uint64_t *ctr,
                               uint32_t *out, hipStream_t s);
// K12m + K12s: counts (65536 u64) of the child's low 16 bits (fix zeroed again), starts (65537
// u64) = their exclusive scan + the cold keys below the child (output positions); the 64 u64
// after starts are K12s's scratch.
hipError_t launch_giant_plan(const uint32_t *part, uint32_t nblk, uint64_t *fix,
                             const uint64_t *ctr, uint64_t *counts, uint64_t *starts,
                             hipStream_t s);
// K12w + K18g: the child's n_child keys written sorted at out[starts[0] .. starts[65536]) from
// the counts; chunk_bin: scratch of ceil(n_child / 8192) u32.
hipError_t launch_giant_expand(const uint64_t *starts, uint64_t n_child, uint32_t child,
                               uint32_t *chunk_bin, uint32_t *out, hipStream_t s);
// Plain device copy kernel (used when a sort has no non-trivial pass).
hipError_t launch_copy(const uint32_t *in, uint32_t *out, uint64_t n, hipStream_t s);

}  // namespace gsort
