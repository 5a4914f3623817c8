/*
 * gsort.h -- C-ABI of libgsort, the MI355X-native distributed integer sorter.
 *
 * Drop-in boundary.  The reference (acgrid/mpi-test) has no library API: its boundary is the
 * program (argv + text file + stdout/stderr + exit status) and, inside it, one function
 *     void sort(const int rank, const int size, const char *file, const int debug)
 * (mpi_radix_sort/mpi_radix_sort.c:60, mpi_sample_sort/mpi_sample_sort.c:28), called from
 * main (mpi_radix_sort.c:224, mpi_sample_sort.c:237).  The host CLIs radix_sort / sample_sort
 * (mpi-test_amd/host/) keep that program contract and call the entry points below; each entry
 * point names the reference code it replaces.
 *
 * Conventions: plain pointers and sizes, no torch types.  One context per rank == one GPU;
 * not thread-safe (one thread per context).  Every call is blocking on return (its stream is
 * synchronised), matching the reference's blocking MPI semantics.  Counts are size_t (the
 * reference's int counts cap N at 2^31-1).  The library never aborts: it returns
 * a status and the host maps non-OK to the reference's stderr + MPI_Abort convention.
 * Keys are int32 and the output order is ascending signed order.
 */
#ifndef GSORT_H
#define GSORT_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct gsort_ctx gsort_ctx;
typedef struct gsort_group gsort_group;

typedef enum {
    GSORT_OK = 0,
    GSORT_EINVAL = 1,    /* bad argument / shape                                          */
    GSORT_ENOMEM = 2,    /* device or host allocation failed                               */
    GSORT_EHIP = 3,      /* HIP runtime error                                              */
    GSORT_ERCCL = 4,     /* RCCL error                                                     */
    GSORT_ENOSAMPLE = 5, /* sample sort: a block is too small for 2P-1 regular samples;
                            the reference aborts with "no enough sample"
                            (mpi_sample_sort.c:94-99)                                      */
    GSORT_ECOMM = 6      /* rank group (in-process or IPC) misuse / peer failure           */
} gsort_status;

/* Wraps an ncclUniqueId (rccl.h:43).  Rank 0 creates it, the host broadcasts it (MPI_Bcast in
 * the CLIs, torch.distributed in bench.py).  Replaces the reference's MPI_COMM_WORLD. */
typedef struct { char internal[128]; } gsort_uid;

/* Per-call device-time breakdown (hipEvents on the context's stream), filled when non-NULL. */
typedef struct {
    double ms_total;          /* whole call, device time                                    */
    double ms_hist;           /* K1 digit histograms (+ K2 scans, K12 plans in the MSD sort)  */
    double ms_pass[4];        /* K3 onesweep passes of the final local sort, by digit        */
    double ms_local_sort;     /* all local-sort kernels (K1+K3), every local sort in the call */
    double ms_exchange;       /* RCCL key exchange(s), all passes                           */
    double ms_place;          /* K8 receive-side placement (radix, P > 1)                   */
    double ms_sample;         /* K4-K6 sampling, splitters, bucket bounds (sample)          */
    double ms_merge;          /* K7 final merge (sample, P > 1)                             */
    uint64_t keys_local_in;   /* keys this rank held before the call                        */
    uint64_t keys_local_out;  /* keys this rank holds after the call                        */
    uint64_t bytes_sent;      /* key bytes this rank sent to OTHER ranks, all passes        */
    uint64_t max_pair_bytes;  /* largest single (this rank -> peer) message, bytes          */
    int passes_run;           /* LSD passes (or MSD levels) run by the final local sort     */
    int exchanges;            /* RCCL all-to-all rounds                                      */
    double ms_level[4];       /* MSD: K3u partition of level 3..0 (its counts: ms_hist)      */
    double ms_bucket_sort;    /* MSD: K11 in-LDS bucket sorts                                */
    uint64_t keys_level[4];   /* MSD: keys partitioned at level 3..0                         */
    uint64_t keys_bucket_sort;/* MSD: keys sorted by K11                                     */
    uint64_t buckets_local;   /* MSD: buckets finished by K11                                */
    int local_algo;           /* local sort used: GSORT_LOCAL_MSD or GSORT_LOCAL_LSD         */
} gsort_stats;

/* Local (one-GPU) sort algorithm.  MSD: unstable LDS-atomic partitions of the top digits and
 * in-LDS bucket sorts (default).  LSD: four stable K1/K2/K3 passes (kept for comparison and
 * as the path the distributed radix pass structure is built on). */
enum { GSORT_LOCAL_MSD = 0, GSORT_LOCAL_LSD = 1 };

/* ---- context -------------------------------------------------------------------------- */
/* gsort_get_uid: an RCCL unique id (one process per GPU, xGMI between GPUs).
 * gsort_get_uid_ipc: the id of a same-node process group of nranks processes that exchange
 * through HIP IPC handles -- any number of ranks per GPU (RCCL refuses two ranks on one device),
 * e.g. `mpirun -np 8` on a one-GPU node.  Rank 0 makes either id; every rank passes it to
 * gsort_create.  gsort_visible_devices: HIP devices this process sees (0 on error). */
gsort_status gsort_get_uid(gsort_uid *out);
gsort_status gsort_get_uid_ipc(int nranks, gsort_uid *out);
int gsort_visible_devices(void);

/* The HIP runtime and RCCL this process's libgsort is bound to (hipRuntimeGetVersion,
 * ncclGetVersion) and the files they were loaded from (dladdr).  Both are resolved by soname,
 * so a process that loaded them first decides: under PyTorch (tests, bench.py: torch is
 * imported first) libgsort runs on torch's bundled HIP runtime and RCCL; the drop-in CLIs (and
 * Python without torch) on /opt/rocm's.  Not in the reference (diagnostics). */
typedef struct {
    int hip_runtime; /* hipRuntimeGetVersion */
    int rccl;        /* ncclGetVersion, e.g. 22707 = 2.27.7 */
    char hip_path[256];
    char rccl_path[256];
} gsort_runtime_info_t;
gsort_status gsort_runtime_info(gsort_runtime_info_t *out);
/* Context of one rank (one process); the uid's kind picks the transport (RCCL or IPC group).
 * nranks == 1 needs no uid (uid may be NULL).
 * hip_device >= 0 selects that GPU; hip_device = -1 - local_rank selects
 * local_rank % (visible GPUs), the usual one-rank-per-GPU placement.
 * Replaces MPI_Init/MPI_Comm_size/MPI_Comm_rank + the MPI communicator
 * (mpi_radix_sort.c:212-214, mpi_sample_sort.c:225-227). */
gsort_status gsort_create(gsort_ctx **ctx, int rank, int nranks, int hip_device,
                          const gsort_uid *uid);
/* In-process rank group: nranks contexts driven by nranks threads of ONE process, exchanging
 * through device-to-device copies, all on ONE GPU (gsort_create_in_group refuses a rank on a
 * device other than the first rank's with GSORT_EINVAL: the group's collectives are ordered by
 * device-scope events).  Used to run the distributed algorithm with P ranks on a single GPU;
 * ranks on several GPUs use gsort_create (RCCL, one process per GPU). */
gsort_status gsort_group_create(gsort_group **grp, int nranks);
gsort_status gsort_group_destroy(gsort_group *grp);
gsort_status gsort_create_in_group(gsort_ctx **ctx, gsort_group *grp, int rank, int hip_device);
gsort_status gsort_destroy(gsort_ctx *ctx);
/* Pre-size device scratch for n_local keys (keeps hipMalloc out of timed regions). */
gsort_status gsort_reserve(gsort_ctx *ctx, size_t n_local);
/* Select the local sort algorithm (GSORT_LOCAL_MSD / GSORT_LOCAL_LSD) for later calls. */
gsort_status gsort_set_local_algo(gsort_ctx *ctx, int algo);
/* Sample sort bucket rule: 0 (default) = the reference's, bucket j = first j with key <= s[j]
 * (mpi_sample_sort.c:148-155; every copy of a splitter value goes to the lower bucket, so a
 * duplicate-heavy input such as Zipf overloads one rank); 1 = duplicate-aware
 * balanced buckets (gsort_plan_split_balanced).  The concatenated output is the same sorted
 * array either way; only the per-rank bucket sizes (gsort_sample_info) differ. */
gsort_status gsort_set_sample_balanced(gsort_ctx *ctx, int on);
/* Reference-compat radix: outside the parity domain (negative keys, P = 1,
 * P = 3's digit under-count) the reference's radix sort is not a numeric sort but a stable sort
 * of the values by the base-P digits of |v| it extracts (number_digit_at, mpi_radix_sort.c:54-58),
 * number_digits(max element) of them (:48-52, :100), one stable pass each (:133-195).
 * radix_p > 0: later gsort_radix calls reproduce that order for a reference run with radix_p
 * processes (any rank count of this context; the order does not depend on the block layout);
 * radix_p = -1: with P = this context's rank count; 0: off (numeric order, the default).
 * Inputs on which the reference indexes outside its buckets (an INT_MIN key, Q5) or allocates a
 * negative last block (N < (P-1) * ceil(N/P) + 1, Q8) return GSORT_EINVAL.  Inside the parity
 * domain both orders are the same sorted array. */
gsort_status gsort_set_ref_compat(gsort_ctx *ctx, int radix_p);
const char *gsort_strerror(gsort_status st);
const char *gsort_last_error(const gsort_ctx *ctx);
int gsort_rank(const gsort_ctx *ctx);
int gsort_nranks(const gsort_ctx *ctx);

/* ---- device-resident hot path ----------------------------------------------------------
 * d_keys: this rank's n_local keys, already on this GPU (block layout, like the reference's
 * initial_sort after MPI_Scatter).  On return *d_out holds this rank's slice of the globally
 * sorted sequence (ctx-owned, valid until the next sort call on ctx); d_keys is unchanged.
 *
 * gsort_radix replaces the radix pass loop mpi_radix_sort.c:133-195 (digit extraction
 * :144-147, count + data all-to-all :150-174, gather/scatter through rank 0 :139,:180-192).
 * Output: balanced blocks -- rank q holds global positions [q*B, min((q+1)*B, N)),
 * B = ceil(N / P), N = sum of n_local over ranks (the reference's size_batch, radix:114).
 *
 * gsort_sample replaces mpi_sample_sort.c:76-197 (local qsort :85, regular sampling
 * :89-105, splitter selection :109-128, splitter broadcast :126-133, bucket partition
 * :148-155, all-to-all :160-170, final qsort :174).  Output: rank q holds bucket q (keys in
 * (s[q-1], s[q]]), so *n_out varies by rank exactly as the reference's size_current_bucket. */
gsort_status gsort_radix(gsort_ctx *ctx, const int32_t *d_keys, size_t n_local,
                         int32_t **d_out, size_t *n_out, gsort_stats *stats);
gsort_status gsort_sample(gsort_ctx *ctx, const int32_t *d_keys, size_t n_local,
                          int32_t **d_out, size_t *n_out, gsort_stats *stats);
/* After gsort_sample: the P-1 splitters (mpi_sample_sort.c:123, "[MASTER] Splitter" lines)
 * and this rank's P bucket lengths ("[COMMON] r: Bucket j=len", :156-158). */
gsort_status gsort_sample_info(const gsort_ctx *ctx, int32_t *splitters,
                               uint64_t *bucket_counts);
/* Which plan the last one-rank local sort of ctx took (diagnostics; no reference
 * counterpart): 0 the exact two-level plan (or a small / distributed case), 1 the sampled
 * plan, 2 the sampled plan found the block ineligible or a region overflowed, and the block
 * was sorted again on the exact plan, 3 the sampled plan on digits below a key prefix every key
 * shares (e.g. 16- or 24-bit keys in int32) after a first sampled attempt found the block
 * ineligible, 4 one 16-bit child held at least half of the keys (Zipf, 8- or 16-bit keys, one
 * frequent value): its keys were sorted by counting their low 16 bits, the others apart
 * (GSORT_EST=0 turns the sampled plan off, GSORT_GIANT=0 the counted child). */
int gsort_last_plan(const gsort_ctx *ctx);

/* ---- drop-in staging (replaces MPI_Scatter / MPI_Gather(v) through rank 0) ---------------
 * gsort_scatter_from_root: rank 0's host array (n_total keys; h_root ignored elsewhere) ->
 * each rank's block [r*B, min((r+1)*B, N)) on its GPU.  Replaces MPI_Scatter
 * (mpi_radix_sort.c:139, mpi_sample_sort.c:82).  *d_keys is ctx-owned.
 * gsort_gather_to_root: every rank's (d_out, n_out) -> rank 0's host array in rank order.
 * Replaces MPI_Gather + MPI_Gatherv (mpi_radix_sort.c:181-192, mpi_sample_sort.c:183-195). */
gsort_status gsort_scatter_from_root(gsort_ctx *ctx, const int32_t *h_root, size_t n_total,
                                     int32_t **d_keys, size_t *n_local);
gsort_status gsort_gather_to_root(gsort_ctx *ctx, const int32_t *d_out, size_t n_out,
                                  int32_t *h_root);

/* ---- device utilities (bench + parity; not in the reference) ------------------------------
 * gsort_generate: K10, the canonical splitmix64 stream; dist 0 = uniform
 * [0, 2^31-1], 1 = zipf s=1.5.  Key i of the stream is written to d_out[i - start].
 * gsort_fingerprint: K9, order-independent multiset fingerprint (sum and xor of mix64(key))
 * plus is-sorted; first/last keys let the host check order across ranks. */
gsort_status gsort_generate(gsort_ctx *ctx, int dist, uint64_t seed, uint64_t start, size_t n,
                            int32_t *d_out);
gsort_status gsort_fingerprint(gsort_ctx *ctx, const int32_t *d_keys, size_t n, uint64_t *sum,
                               uint64_t *xr, int *sorted, int32_t *first, int32_t *last);
/* Copy helpers for hosts that have no HIP headers (the C CLIs, ctypes).  Buffers from
 * gsort_device_alloc belong to ctx: gsort_destroy releases every one still allocated (do not use
 * them afterwards), and gsort_device_free accepts only pointers gsort_device_alloc returned on
 * the same ctx (anything else returns GSORT_EINVAL and frees nothing). */
gsort_status gsort_device_alloc(gsort_ctx *ctx, size_t bytes, void **d_ptr);
gsort_status gsort_device_free(gsort_ctx *ctx, void *d_ptr);
gsort_status gsort_copy_to_host(gsort_ctx *ctx, void *h_dst, const void *d_src, size_t bytes);
gsort_status gsort_copy_to_device(gsort_ctx *ctx, void *d_dst, const void *h_src, size_t bytes);
/* The bench's HBM ceiling for a read + write pass: a streaming copy kernel (16 B per lane,
 * one block per 16 KiB chunk, nontemporal stores) of `bytes` between two scratch buffers,
 * timed with hipEvents, median of reps.  *ms = one copy, *gbps = 2 * bytes / time. */
gsort_status gsort_copy_ceiling(gsort_ctx *ctx, size_t bytes, int reps, double *ms, double *gbps);
/* Which kernel configuration the local sort uses (tile = keys per workgroup). */
size_t gsort_onesweep_tile(void);

/* ---- rank-0 text input (host only) ---------------------------------------------------------
 * gsort_parse_text: parse whitespace-separated decimal keys with the reference reader's
 * fscanf("%d") semantics (mpi_radix_sort.c:85-97, mpi_sample_sort.c:50-60): optional sign,
 * values wrap mod 2^32 after saturating at the 64-bit long range.  Writes up to cap keys to out
 * (out may be NULL to count) and returns the key count, or -1 on a non-numeric token (the
 * reference spins on such a token until realloc fails and then reports the file invalid).  A
 * trailing delimiter adds no phantom element.  threads > 1 parses in chunks. */
long long gsort_parse_text(const char *buf, size_t len, int32_t *out, size_t cap, int threads);
/* gsort_format_dump: the reference's sorted dump, printf("%u|%u\n", i, int_buf[i]) per key on
 * rank 0 (mpi_radix_sort.c:198-200, mpi_sample_sort.c:202-204), rendered as "%llu|%u\n"
 * (index first_index + i, key as unsigned) for keys[0 .. n) into out on `threads` threads.
 * Returns the byte count (out == NULL: only count), or -1 if cap is too small. */
long long gsort_format_dump(const int32_t *keys, size_t n, uint64_t first_index, char *out,
                            size_t cap, int threads);

/* gsort_write_report: the drop-in programs' stdout contract lines for one rank, written to fd
 * (write(2); flush any stdio buffer on fd first), in the reference's order:
 *   sample, rank 0:       "Each bucket will be put %llu items.\n", B = ceil(N/P)
 *                         (mpi_sample_sort.c:72-74)
 *   sample, debug >= 1:   rank 0 "[MASTER] Splitter: %u.\n" x (P-1) (:124); then every rank
 *                         "[COMMON] r: Bucket j=len\n" for j < P (:156-158)
 *   rank 0, the dump:     "%u|%u\n" index|key of sorted[0 .. N) at radix debug > 2
 *                         (mpi_radix_sort.c:198-200) or sample debug >= 1 (sample:202-204)
 *   rank 0:               "The n/2-th sorted element: %d\n" = sorted[N/2 - 1], sorted[0] for
 *                         N = 1 (radix:201, sample:205; quirk Q14)
 * The reference's other debug lines are free-form progress output, not reproduced.  splitters
 * (rank 0, P-1) and bucket_counts (P) come from gsort_sample_info; sorted is rank 0's gathered
 * array (gsort_gather_to_root).  Replaces the printf calls listed above. */
enum { GSORT_REPORT_RADIX = 0, GSORT_REPORT_SAMPLE = 1 };
typedef struct {
    int algo;                      /* GSORT_REPORT_RADIX / GSORT_REPORT_SAMPLE               */
    int rank, nranks, debug;       /* debug: the programs' argv[2] (0 when absent)            */
    uint64_t n_total;              /* N                                                       */
    const int32_t *splitters;      /* sample, debug >= 1, rank 0: P-1 splitters               */
    const uint64_t *bucket_counts; /* sample, debug >= 1: this rank's P bucket lengths        */
    const int32_t *sorted;         /* rank 0: the N sorted keys                               */
    int stage;                     /* 0: every line; 1: only what the reference prints before
                                      its sort ("Each bucket", sample:74); 2: only the rest     */
} gsort_report;
gsort_status gsort_write_report(const gsort_report *r, int fd);

/* ---- host-only planning (no GPU; exported so CPU tests can check it) ----------------------
 * gsort_plan_radix_route: the K8 routing of one distributed LSD pass.  hist = P x 256 per-rank
 * digit counts, B = block size.  Fills send[P] / recv[P] key counts for rank `me` and the
 * receive-side placement rows seg[4*k] = {src rank, offset in src's chunk, dest offset,
 * length}; *nseg = k (<= P*256).  Semantics of mpi_radix_sort.c:150-192 (stable: digit, then
 * source rank, then source order).
 * gsort_plan_splitters: sort the P*(2P-1) rank-ordered samples and pick
 * splitters[i] = S[(i+1)(2P-1)] (mpi_sample_sort.c:116-123). */
gsort_status gsort_plan_radix_route(int P, const uint64_t *hist, uint64_t B, int me,
                                    uint64_t *send, uint64_t *recv, uint64_t *seg,
                                    size_t *nseg);
gsort_status gsort_plan_splitters(int P, const int32_t *samples, int32_t *splitters);
/* gsort_plan_split: the one exchange of the distributed radix sort (replaces the per-digit
 * routing of mpi_radix_sort.c:139,150-192).  n_all[P] = keys per rank (each block sorted);
 * lt / le = P x (P-1): keys of rank p < / <= v_q, the g_q = min(qB, N)-th smallest key of all
 * (B = ceil(N/P)).  Copies of v_q are taken left of a boundary in rank order.  Outputs the
 * keys rank `me` sends to / receives from every rank (contiguous, in rank order). */
gsort_status gsort_plan_split(int P, const uint64_t *n_all, const uint64_t *lt,
                              const uint64_t *le, int me, uint64_t *send, uint64_t *recv);
/* gsort_plan_split_balanced: the same cut for the balanced sample sort, where v_q is the q-th
 * splitter (mpi_sample_sort.c:109-128) rather than the g_q-th key: the boundary moves to
 * clamp(min(qB, N), sum_p lt + 1, sum_p le), i.e. the copies of a splitter value are shared
 * out in rank order instead of all going to the lower bucket (mpi_sample_sort.c:148-155); a
 * value held once goes to the lower bucket, as there. */
gsort_status gsort_plan_split_balanced(int P, const uint64_t *n_all, const uint64_t *lt,
                                       const uint64_t *le, int me, uint64_t *send,
                                       uint64_t *recv);

/* gsort_plan_ref_digits: the reference radix sort's digit plan with its own double math --
 * loop = number_digits(max_element, P) (mpi_radix_sort.c:48-52, :100; <= 0 means no pass, as at
 * P = 1), mod[d] = (int)pow(P, d+1) as x86 converts it (out of range -> INT_MIN) and
 * scale[d] = pow(P, d) for d < loop (mpi_radix_sort.c:57).  mod / scale may be NULL; they must
 * hold cap entries, and loop > cap with either given returns GSORT_EINVAL. */
gsort_status gsort_plan_ref_digits(int P, int32_t max_element, int *loop, int32_t *mod,
                                   double *scale, int cap);

#ifdef __cplusplus
}
#endif
#endif /* GSORT_H */
