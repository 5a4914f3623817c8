/*
 * oracle.c -- CPU restatement of the acgrid/mpi-test sort paths.
 *
 * TEST INFRASTRUCTURE ONLY.  This file is the parity checker, never the thing measured or
 * shipped.  Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load it
 * (as oracle/liborcl.so through ctypes).  The product (libgsort.so and the radix_sort /
 * sample_sort binaries) never links, loads or calls it.
 *
 * Parity is PINNED: tests/test_oracle_golden.py checks every function below against golden
 * vectors produced by the reference programs themselves (built unchanged from
 * /root/reference by oracle/Makefile into oracle/_ref/ and run under mpirun by
 * tests/golden/make_golden.py).
 *
 * What is restated (cites are /root/reference/<file>:<line>):
 *   orc_ref_radix   mpi_radix_sort/mpi_radix_sort.c:60-205  base-P LSD passes, simulated ranks
 *   orc_ref_sample  mpi_sample_sort/mpi_sample_sort.c:28-218 regular-sampling sample sort
 *   orc_read_ints   mpi_radix_sort/mpi_radix_sort.c:85-97 / mpi_sample_sort.c:50-60 (%d reader)
 * and the build's own algorithm, restated scalar so the GPU path can be checked against it:
 *   orc_gen            SURVEY.md 8(d) splitmix64 generator (uniform / zipf)
 *   orc_lsd8           8-bit LSD radix sort of int32 (sign-flipped) -- what libgsort computes
 *   orc_radix_route    distributed placement of one LSD pass (global positions -> blocks)
 *   orc_sample_plan    splitter selection + bucket bounds on a sorted block
 *   orc_fingerprint    order-independent multiset fingerprint + is-sorted
 *
 * Everything is plain C99 (gcc -O2 -ffp-contract=off); no MPI, no HIP.
 */
#include <limits.h>
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#define ORC_OK 0
#define ORC_E_OUTSIDE_PD 1   /* the reference would crash / read garbage here (Q-list)   */
#define ORC_E_NO_SAMPLE 2    /* mpi_sample_sort.c:96-99 "no enough sample" abort (Q9)    */
#define ORC_E_OVERFLOW 3     /* mpi_sample_sort.c:144,161,167 bucket overflow (Q11/Q12)  */
#define ORC_E_NOMEM 4

/* ------------------------------------------------------------------------------------------
 * Canonical generator.  Counter based: key i of a stream uses
 * state = seed + (i+1) * golden, so rank r can start at key index r*B.
 * ---------------------------------------------------------------------------------------- */
static uint64_t orc_mix64(uint64_t z)
{
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
    return z ^ (z >> 31);
}

int32_t orc_gen_one(int dist, uint64_t seed, uint64_t index)
{
    uint64_t z = orc_mix64(seed + (index + 1) * 0x9E3779B97F4A7C15ULL);
    if (dist == 0) return (int32_t)(z >> 33); /* uniform in [0, 2^31-1] */
    /* zipf-like discrete Pareto tail, s = 1.5: u in (0,1], k = floor(1/u^2) clipped */
    double u = (double)((z >> 11) + 1) * 0x1p-53;
    double k = floor(1.0 / (u * u));
    if (k > 2147483647.0) k = 2147483647.0;
    return (int32_t)k;
}

void orc_gen(int dist, uint64_t seed, uint64_t start, size_t n, int32_t *out)
{
    for (size_t i = 0; i < n; i++) out[i] = orc_gen_one(dist, seed, start + i);
}

/* ------------------------------------------------------------------------------------------
 * %d reader.  mpi_radix_sort.c:85-97 / mpi_sample_sort.c:50-60 loop `!feof` over fscanf("%d").
 * with_phantom = 1 reproduces the reference exactly (Q6: a trailing delimiter appends one more
 * element; ref-radix repeats the previous value, mpi_radix_sort.c:89-90).  with_phantom = 0 is
 * the build's contract (no phantom).  Returns the number of elements, or -1.
 * ---------------------------------------------------------------------------------------- */
long orc_read_ints(const char *path, int32_t *out, long cap, int with_phantom)
{
    FILE *fp = fopen(path, "r");
    if (!fp) return -1;
    long n = 0;
    int cur = 0;
    while (!feof(fp)) {
        int got = fscanf(fp, "%d", &cur);
        if (got == 0) break; /* non-numeric token: the reference spins forever here */
        if (got != 1 && !with_phantom) break;
        if (n < cap) out[n] = cur; /* on a failed scan `cur` keeps the previous value */
        n++;
    }
    fclose(fp);
    return n;
}

/* ------------------------------------------------------------------------------------------
 * Reference radix digit math, restated with the same double arithmetic.
 *   number_digits   mpi_radix_sort.c:48-52   (int)(log|v| / log P) + 1
 *   number_digit_at mpi_radix_sort.c:54-58   (|v| % (int)P^pos) / P^(pos-1)
 * x86 cvttsd2si turns every out-of-range double (inf, nan, >= 2^31) into INT_MIN; that is what
 * the reference binary does (Q1, Q2), so the conversion is spelled out.
 * ---------------------------------------------------------------------------------------- */
static int orc_x86_dtoi(double x)
{
    if (!(x > -2147483649.0 && x < 2147483648.0)) return INT_MIN;
    return (int)x;
}

int orc_ref_number_digits(int value, int radix)
{
    int mag = value < 0 ? (value == INT_MIN ? INT_MIN : -value) : value;
    double l = log(mag > 0 ? (double)mag : 1.0) / log((double)radix);
    return orc_x86_dtoi(l) + 1;
}

int orc_ref_digit_at(int value, int radix, int position)
{
    int mag = value < 0 ? (value == INT_MIN ? INT_MIN : -value) : value;
    int modulus = orc_x86_dtoi(pow((double)radix, (double)position));
    int rem = (modulus == 0 || modulus == -1) ? 0 : mag % modulus;
    return orc_x86_dtoi((double)rem / pow((double)radix, (double)position - 1.0));
}

/* ------------------------------------------------------------------------------------------
 * orc_ref_radix -- mpi_radix_sort.c:60-205 with P simulated ranks.
 * Per pass (radix:133-195): rank r takes block [rB, min((r+1)B, N)) (MPI_Scatter :139),
 * pushes each key into bucket[digit] (:144-147), sends bucket j to rank j (:164-166), rank j
 * concatenates what it receives from sources 0..P-1 in order (:168-173), and the blocks are
 * gathered back in rank order (:185-192).  loop = number_digits(max element) (:91, :100).
 * Returns ORC_E_OUTSIDE_PD where the reference crashes (Q5 negative digit of an INT_MIN key,
 * Q8 empty last block).
 * *passes_out receives the pass count the reference runs (<= 0 means none, Q1).
 * ---------------------------------------------------------------------------------------- */
int orc_ref_radix(const int32_t *in, size_t n, int P, int32_t *out, int *passes_out)
{
    if (P < 1 || n < 1) return ORC_E_OUTSIDE_PD;
    size_t B = (n + (size_t)P - 1) / (size_t)P;
    if ((long long)n - (long long)B * (P - 1) <= 0) return ORC_E_OUTSIDE_PD; /* Q8 */
    int max_el = -1;
    for (size_t i = 0; i < n; i++)
        if (in[i] > max_el) max_el = in[i];
    int loop = orc_ref_number_digits(max_el, P);
    if (passes_out) *passes_out = loop;
    memcpy(out, in, n * sizeof(int32_t));
    if (loop < 1) return ORC_OK; /* Q1: P = 1 runs zero passes */

    int32_t *tmp = malloc(n * sizeof(int32_t));
    size_t *cnt = calloc((size_t)P * P, sizeof(size_t)); /* cnt[src*P + dst] */
    unsigned char *dig = malloc(n);
    if (!tmp || !cnt || !dig) { free(tmp); free(cnt); free(dig); return ORC_E_NOMEM; }
    for (int pos = 1; pos <= loop; pos++) {
        memset(cnt, 0, (size_t)P * P * sizeof(size_t));
        for (int r = 0; r < P; r++) {
            size_t lo = (size_t)r * B, hi = lo + B < n ? lo + B : n;
            for (size_t i = lo; i < hi; i++) {
                int d = orc_ref_digit_at(out[i], P, pos);
                if (d < 0 || d >= P) { /* Q5: abs(INT_MIN) < 0 indexes buckets[-k] */
                    free(tmp); free(cnt); free(dig);
                    return ORC_E_OUTSIDE_PD;
                }
                dig[i] = (unsigned char)d;
                cnt[(size_t)r * P + d]++;
            }
        }
        /* receiver j gets src 0..P-1 in order; gather concatenates receivers 0..P-1 */
        size_t w = 0;
        for (int j = 0; j < P; j++)
            for (int r = 0; r < P; r++) {
                size_t lo = (size_t)r * B, hi = lo + B < n ? lo + B : n;
                for (size_t i = lo; i < hi; i++)
                    if (dig[i] == j) tmp[w++] = out[i];
            }
        memcpy(out, tmp, n * sizeof(int32_t));
    }
    free(tmp); free(cnt); free(dig);
    return ORC_OK;
}

/* ------------------------------------------------------------------------------------------
 * orc_ref_sample -- mpi_sample_sort.c:28-218 with P simulated ranks.
 *   B = ceil(N/P), last block N - B(P-1) (:72-73); qsort each block (:85)
 *   k = 2P-1 samples at i*floor(B/k) (:89-105), abort if the index runs past the block (:96-99)
 *   root gathers rank 0's samples then ranks 1..P-1 (:103, :110-115), sorts them (:116),
 *   splitter i = S[(i+1)k] (:122-123)
 *   bucket j = first j with key <= s[j], else P-1 (:148-155)
 *   exchange (:160-170), final sort of own bucket (:174), gather in rank order (:182-197)
 * Outputs: out[N] (gathered result), splitters[P-1], matrix[P*P] (rank r's bucket j length --
 * the "[COMMON] r: Bucket j=len" debug lines, :156-158), recv[P] (final bucket sizes).
 * Returns ORC_E_NO_SAMPLE / ORC_E_OVERFLOW where the reference aborts or overruns.
 * ---------------------------------------------------------------------------------------- */
static int orc_cmp_i32(const void *a, const void *b)
{
    int32_t x = *(const int32_t *)a, y = *(const int32_t *)b;
    return (x > y) - (x < y);
}

int orc_ref_sample(const int32_t *in, size_t n, int P, int32_t *out, int32_t *splitters,
                   long long *matrix, long long *recv)
{
    if (P < 2 || n < 1) return ORC_E_OUTSIDE_PD; /* P = 1 reads splitters[-1] (Q10) */
    long long B = ((long long)n + P - 1) / P;
    long long small = (long long)n - B * (P - 1);
    if (small < 0) return ORC_E_OUTSIDE_PD; /* Q8: calloc of a negative count */
    int k = 2 * P - 1;
    long long interval = B / k;
    long long maxb = (long long)floor((double)B * 1.5); /* :140 max_size_bucket */

    int32_t *blk = malloc(n * sizeof(int32_t));
    int32_t *samp = malloc((size_t)P * k * sizeof(int32_t));
    if (!blk || !samp) { free(blk); free(samp); return ORC_E_NOMEM; }
    memcpy(blk, in, n * sizeof(int32_t));
    int rc = ORC_OK;
    for (int r = 0; r < P && rc == ORC_OK; r++) {
        long long lo = (long long)r * B, len = r == P - 1 ? small : B;
        qsort(blk + lo, (size_t)len, sizeof(int32_t), orc_cmp_i32);
        for (int i = 0; i < k; i++) {
            long long idx = (long long)i * interval;
            if (idx >= len) { rc = ORC_E_NO_SAMPLE; break; }
            samp[r * k + i] = blk[lo + idx];
        }
    }
    if (rc != ORC_OK) { free(blk); free(samp); return rc; }
    qsort(samp, (size_t)P * k, sizeof(int32_t), orc_cmp_i32);
    for (int i = 0; i < P - 1; i++) splitters[i] = samp[(i + 1) * k];

    for (int r = 0; r < P; r++) {
        long long lo = (long long)r * B, len = r == P - 1 ? small : B;
        for (int j = 0; j < P; j++) matrix[r * P + j] = 0;
        for (long long i = 0; i < len; i++) {
            int32_t v = blk[lo + i];
            int j = 0;
            while (j < P - 1 && !(v <= splitters[j])) j++;
            matrix[r * P + j]++;
        }
    }
    /* overflow checks: push capacity 2*maxb (:144), send size maxb with tag=len (:161),
     * receive writes maxb at the running offset into capacity 2*maxb (:165-169) */
    for (int j = 0; j < P; j++) {
        long long have = matrix[j * P + j];
        for (int r = 0; r < P; r++) {
            if (matrix[r * P + j] > maxb) rc = ORC_E_OVERFLOW;
            if (r == j) continue;
            if (have + maxb > 2 * maxb) rc = ORC_E_OVERFLOW;
            have += matrix[r * P + j];
        }
        recv[j] = have;
    }
    /* bucket j of the output = all keys with bucket index j, sorted; gather in rank order.
     * Because every block is sorted and buckets are value ranges, this equals the sorted
     * concatenation of buckets 0..P-1. */
    size_t w = 0;
    for (int j = 0; j < P; j++) {
        size_t start = w;
        for (int r = 0; r < P; r++) {
            long long lo = (long long)r * B, len = r == P - 1 ? small : B;
            for (long long i = 0; i < len; i++) {
                int32_t v = blk[lo + i];
                int b = 0;
                while (b < P - 1 && !(v <= splitters[b])) b++;
                if (b == j) out[w++] = v;
            }
        }
        qsort(out + start, w - start, sizeof(int32_t), orc_cmp_i32);
    }
    free(blk); free(samp);
    return rc;
}

/* ------------------------------------------------------------------------------------------
 * The build's algorithm, restated scalar.
 * ---------------------------------------------------------------------------------------- */

/* orc_lsd8: stable 8-bit LSD radix sort of int32 in ascending signed order.  Each key is
 * mapped u = x ^ 0x80000000 so unsigned digit order is signed numeric order.  This is what
 * gsort_radix computes on one GPU (K1 histogram, K3 onesweep passes). */
int orc_lsd8(const int32_t *in, size_t n, int32_t *out)
{
    uint32_t *a = malloc((n ? n : 1) * sizeof(uint32_t));
    uint32_t *b = malloc((n ? n : 1) * sizeof(uint32_t));
    if (!a || !b) { free(a); free(b); return ORC_E_NOMEM; }
    for (size_t i = 0; i < n; i++) a[i] = (uint32_t)in[i] ^ 0x80000000u;
    for (int pass = 0; pass < 4; pass++) {
        size_t cnt[256] = {0}, off[256];
        int sh = 8 * pass;
        for (size_t i = 0; i < n; i++) cnt[(a[i] >> sh) & 0xFF]++;
        size_t s = 0;
        for (int d = 0; d < 256; d++) { off[d] = s; s += cnt[d]; }
        for (size_t i = 0; i < n; i++) b[off[(a[i] >> sh) & 0xFF]++] = a[i];
        uint32_t *t = a; a = b; b = t;
    }
    for (size_t i = 0; i < n; i++) out[i] = (int32_t)(a[i] ^ 0x80000000u);
    free(a); free(b);
    return ORC_OK;
}

/* orc_digit_hist: 256-bin histogram of digit `pass` (0..3) of the sign-flipped keys. */
void orc_digit_hist(const int32_t *in, size_t n, int pass, uint64_t *hist)
{
    memset(hist, 0, 256 * sizeof(uint64_t));
    for (size_t i = 0; i < n; i++) hist[(((uint32_t)in[i] ^ 0x80000000u) >> (8 * pass)) & 0xFF]++;
}

/* orc_radix_route -- distributed placement of one LSD pass (the K8 routing of SURVEY 2.1).
 * Inputs: hist[P*256] per-rank digit counts of this pass, B = block size (rank q owns global
 * positions [qB, (q+1)B)).  Global position of rank r's i-th key of digit d (stable order:
 * digit, then source rank, then local order -- mpi_radix_sort.c:164-173 + :185-192) is
 *   G[d] + R[r][d] + i,  G[d] = sum_{d'<d} total[d'],  R[r][d] = sum_{r'<r} hist[r'][d].
 * Outputs for rank `me`:
 *   send[P]  keys rank `me` sends to each destination (contiguous ranges of its digit-sorted
 *            block, in destination order)
 *   recv[P]  keys rank `me` receives from each source
 *   seg[*]   receive-side placement: rows of 4 uint64 {src rank, offset in src's chunk,
 *            dest offset in my block, length}, ordered by (src, digit); returns the row count.
 */
long orc_radix_route(int P, const uint64_t *hist, uint64_t B, int me, uint64_t *send,
                     uint64_t *recv, uint64_t *seg)
{
    uint64_t G[256], s = 0;
    for (int d = 0; d < 256; d++) {
        G[d] = s;
        for (int r = 0; r < P; r++) s += hist[(size_t)r * 256 + d];
    }
    for (int q = 0; q < P; q++) { send[q] = 0; recv[q] = 0; }
    uint64_t lo_me = (uint64_t)me * B, hi_me = lo_me + B;
    long rows = 0;
    for (int r = 0; r < P; r++) {
        uint64_t chunk_off = 0; /* offset inside the chunk r sends to me */
        for (int d = 0; d < 256; d++) {
            uint64_t R = 0;
            for (int r2 = 0; r2 < r; r2++) R += hist[(size_t)r2 * 256 + d];
            uint64_t c = hist[(size_t)r * 256 + d];
            uint64_t a = G[d] + R, e = a + c; /* global range of (r, d) */
            if (r == me) {
                for (int q = 0; q < P; q++) {
                    uint64_t qa = (uint64_t)q * B, qe = qa + B;
                    uint64_t x = a > qa ? a : qa, y = e < qe ? e : qe;
                    if (y > x) send[q] += y - x;
                }
            }
            uint64_t x = a > lo_me ? a : lo_me, y = e < hi_me ? e : hi_me;
            if (y > x) {
                seg[rows * 4 + 0] = (uint64_t)r;
                seg[rows * 4 + 1] = chunk_off;
                seg[rows * 4 + 2] = x - lo_me;
                seg[rows * 4 + 3] = y - x;
                rows++;
                chunk_off += y - x;
                recv[r] += y - x;
            }
        }
    }
    return rows;
}

/* orc_sample_plan -- splitter selection and bucket bounds of gsort_sample.
 * samples[P*k]: rank-ordered samples (rank 0's k first) as gathered at the root
 * (mpi_sample_sort.c:103,110-115).  Writes splitters[P-1] = sorted[(i+1)k] (:116,:122-123).
 * For a sorted block blk[n], bounds[j] = number of keys <= splitters[j] (j < P-1), i.e. the
 * end of bucket j under the rule of :148-155; bucket P-1 ends at n. */
void orc_sample_plan(int P, const int32_t *samples, const int32_t *blk, uint64_t n,
                     int32_t *splitters, uint64_t *bounds)
{
    int k = 2 * P - 1;
    int32_t *s = malloc((size_t)P * k * sizeof(int32_t));
    memcpy(s, samples, (size_t)P * k * sizeof(int32_t));
    qsort(s, (size_t)P * k, sizeof(int32_t), orc_cmp_i32);
    for (int i = 0; i < P - 1; i++) splitters[i] = s[(i + 1) * k];
    free(s);
    for (int j = 0; j < P - 1; j++) {
        uint64_t lo = 0, hi = n; /* upper_bound */
        while (lo < hi) {
            uint64_t mid = lo + (hi - lo) / 2;
            if (blk[mid] <= splitters[j]) lo = mid + 1; else hi = mid;
        }
        bounds[j] = lo;
    }
    bounds[P - 1] = n;
}

/* orc_fingerprint -- K9's order-independent multiset fingerprint + is-sorted check.
 * sum = sum of mix64(key as u32), xr = xor of the same; *sorted = non-decreasing (signed). */
void orc_fingerprint(const int32_t *a, size_t n, uint64_t *sum, uint64_t *xr, int *sorted)
{
    uint64_t s = 0, x = 0;
    int ok = 1;
    for (size_t i = 0; i < n; i++) {
        uint64_t m = orc_mix64((uint64_t)(uint32_t)a[i]);
        s += m; x ^= m;
        if (i && a[i - 1] > a[i]) ok = 0;
    }
    *sum = s; *xr = x; *sorted = ok;
}

/* Scalar reference sort timing helper for bench.py's cpu_baseline "port" leg: a plain
 * single-thread qsort (what the reference's local step does, mpi_sample_sort.c:85). */
void orc_qsort_i32(int32_t *a, size_t n) { qsort(a, n, sizeof(int32_t), orc_cmp_i32); }

/* Text writer for generated inputs: '\n'-separated, no trailing newline. */
int orc_write_text(const char *path, const int32_t *a, size_t n)
{
    FILE *fp = fopen(path, "w");
    if (!fp) return -1;
    for (size_t i = 0; i < n; i++) fprintf(fp, i + 1 < n ? "%d\n" : "%d", a[i]);
    return fclose(fp);
}
