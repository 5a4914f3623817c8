/*
 * gsort_cli.c -- host side of the drop-in radix_sort / sample_sort programs (C + MPI
 * bootstrap).  Keeps the reference's program contract:
 *   mpirun -np P ./radix_sort|./sample_sort <file> [debug]
 *   argc not in {2,3}      -> rank 0: "Usage: %s <file: Data file to read>\n", abort(1)
 *                             (mpi_radix_sort.c:217-221, mpi_sample_sort.c:230-234)
 *   unreadable file        -> "sort(): '%s' is not a valid file for read.\n", abort(1)
 *                             (mpi_radix_sort.c:80-83)
 *   sample stdout          -> "Each bucket will be put %u items.\n" (mpi_sample_sort.c:74)
 *   debug dump             -> "%u|%u\n" index|value, radix at debug > 2 (radix:198-200),
 *                             sample at debug >= 1 (sample:202-204); sample debug also prints
 *                             "[MASTER] Splitter: %u.\n" and "[COMMON] r: Bucket j=len"
 *   stdout                 -> "The n/2-th sorted element: %d\n" = sorted[N/2-1] (radix:201)
 *   stderr                 -> "Endtime()-Starttime() = %.5f sec\n" (radix:203)
 * The timer spans what the reference's spans -- from after the rank-0 read to after the final
 * gather (radix:98,197; sample:61,201) -- and, like the reference's, excludes process setup
 * (MPI_Init there; MPI_Init + GPU context + RCCL communicator here).
 * MPI carries only the bootstrap: N and the RCCL unique id.  Keys move H2D on rank 0, over
 * xGMI between GPUs (RCCL), and D2H on rank 0 -- never over MPI.
 */
#include <mpi.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/stat.h>

#include "gsort.h"
#include "gsort_cli.h"

static void die(const char *msg)
{
    fprintf(stderr, "%s\n", msg);
    fflush(stderr);
    MPI_Abort(MPI_COMM_WORLD, EXIT_FAILURE);
    exit(EXIT_FAILURE);
}

static void check(gsort_status st, gsort_ctx *ctx, const char *what)
{
    if (st == GSORT_OK) return;
    char msg[1024];
    snprintf(msg, sizeof msg, "%s(): %s: %s", what, gsort_strerror(st),
             ctx ? gsort_last_error(ctx) : "");
    die(msg);
}

/* rank-0 reader (mpi_radix_sort.c:73-97): whole file, then a %d-compatible parse.
 * phantom (reference-compat mode): the reference's !feof loop stores one more element -- a copy
 * of the last value -- when anything follows the last number (quirk Q6, mpi_radix_sort.c:85-91) */
static int32_t *read_keys(const char *file, size_t *n_out, int phantom)
{
    char msg[4096 + 64];
    snprintf(msg, sizeof msg, "sort(): '%s' is not a valid file for read.", file);
    FILE *fp = fopen(file, "rb");
    if (!fp) die(msg);
    struct stat sb;
    if (fstat(fileno(fp), &sb) != 0) die(msg);
    size_t len = (size_t)sb.st_size;
    char *buf = malloc(len ? len : 1);
    if (!buf || (len && fread(buf, 1, len, fp) != len)) die(msg);
    fclose(fp);
    size_t cap = len / 2 + 1; /* every key but the last takes >= 2 bytes */
    int32_t *keys = malloc(cap * sizeof(int32_t));
    if (!keys) die(msg);
    long long n = gsort_parse_text(buf, len, keys, cap, 16);
    const int trailing = len > 0 && strchr(" \t\n\v\f\r", buf[len - 1]) != NULL;
    free(buf);
    if (n <= 0) die(msg); /* empty or non-numeric: the reference never completes a valid run */
    if (phantom && trailing && (size_t)n < cap) keys[n] = keys[n - 1], n++;
    *n_out = (size_t)n;
    return keys;
}

/* the full sorted dump (radix:198-200, sample:202-204) in blocks of kDumpBlock keys, each
 * rendered on 16 threads by gsort_format_dump and written with one fwrite */
static void print_dump(const int32_t *keys, unsigned long long n)
{
    enum { kDumpBlock = 1 << 21, kMaxLine = 32 };
    char *buf = malloc((size_t)kDumpBlock * kMaxLine);
    if (!buf) die("print_dump: out of host memory");
    fflush(stdout);
    for (unsigned long long a = 0; a < n; a += kDumpBlock) {
        const size_t m = n - a < kDumpBlock ? (size_t)(n - a) : (size_t)kDumpBlock;
        const long long len =
            gsort_format_dump(keys + a, m, a, buf, (size_t)kDumpBlock * kMaxLine, 16);
        if (len < 0 || fwrite(buf, 1, (size_t)len, stdout) != (size_t)len)
            die("print_dump: write failed");
    }
    free(buf);
}

static int local_rank(int rank)
{
    const char *vars[] = {"MPI_LOCALRANKID", "OMPI_COMM_WORLD_LOCAL_RANK", "LOCAL_RANK"};
    for (int i = 0; i < 3; i++) {
        const char *v = getenv(vars[i]);
        if (v && *v) return atoi(v);
    }
    return rank;
}

int gsort_cli_main(int argc, char **argv, int algo)
{
    int rank, size;
    MPI_Init(&argc, &argv);
    MPI_Comm_size(MPI_COMM_WORLD, &size);
    MPI_Comm_rank(MPI_COMM_WORLD, &rank);
    if (argc != 2 && argc != 3) {
        if (rank == 0) fprintf(stderr, "Usage: %s <file: Data file to read>\n", argv[0]);
        MPI_Abort(MPI_COMM_WORLD, EXIT_FAILURE);
        exit(EXIT_FAILURE);
    }
    const char *file = argv[1];
    const int debug = argc == 3 ? atoi(argv[2]) : 0;

    /* GSORT_REF_COMPAT=1 (radix_sort): the reference's own output order outside the parity
     * domain -- negative keys, P = 1, P = 3 (gsort_set_ref_compat) -- and its reader's phantom
     * element after trailing whitespace */
    const char *cmp = getenv("GSORT_REF_COMPAT");
    const int compat = algo == CLI_RADIX && cmp && atoi(cmp);
    int32_t *int_buf = NULL;
    unsigned long long n_total = 0;
    if (rank == 0) {
        size_t n;
        int_buf = read_keys(file, &n, compat);
        n_total = n;
    }

    /* bootstrap: one context per rank == one GPU; RCCL id broadcast over MPI */
    gsort_uid uid;
    memset(&uid, 0, sizeof uid);
    if (size > 1) {
        if (rank == 0) check(gsort_get_uid(&uid), NULL, "gsort_get_uid");
        MPI_Bcast(&uid, (int)sizeof uid, MPI_BYTE, 0, MPI_COMM_WORLD);
    }
    gsort_ctx *ctx = NULL;
    check(gsort_create(&ctx, rank, size, -1 - local_rank(rank), size > 1 ? &uid : NULL), NULL,
          "gsort_create");
    /* GSORT_SAMPLE_BALANCED=1: duplicate-aware sample buckets (not the reference's rule) */
    const char *bal = getenv("GSORT_SAMPLE_BALANCED");
    if (algo == CLI_SAMPLE && bal && atoi(bal))
        check(gsort_set_sample_balanced(ctx, 1), ctx, "gsort_set_sample_balanced");
    if (compat) check(gsort_set_ref_compat(ctx, -1), ctx, "gsort_set_ref_compat");

    MPI_Barrier(MPI_COMM_WORLD);
    const double start = MPI_Wtime();
    MPI_Bcast(&n_total, 1, MPI_UNSIGNED_LONG_LONG, 0, MPI_COMM_WORLD);
    const unsigned long long B = (n_total + (unsigned long long)size - 1) / (unsigned long long)size;
    if (algo == CLI_SAMPLE && rank == 0) printf("Each bucket will be put %llu items.\n", B);

    int32_t *d_keys = NULL, *d_out = NULL;
    size_t n_local = 0, n_out = 0;
    check(gsort_scatter_from_root(ctx, int_buf, n_total, &d_keys, &n_local), ctx,
          "gsort_scatter_from_root");
    if (algo == CLI_RADIX) {
        check(gsort_radix(ctx, d_keys, n_local, &d_out, &n_out, NULL), ctx, "gsort_radix");
        if (debug) printf("[COMMON] %d: sorted block of %zu keys\n", rank, n_out);
    } else {
        gsort_status st = gsort_sample(ctx, d_keys, n_local, &d_out, &n_out, NULL);
        if (st == GSORT_ENOSAMPLE) {
            /* mpi_sample_sort.c:97 prints from the short rank; every rank knows here */
            if (rank == 0)
                fprintf(stderr, "[ERROR] %d: no enough sample, try smaller processes. %s\n",
                        rank, gsort_last_error(ctx));
            fflush(stderr);
            MPI_Abort(MPI_COMM_WORLD, EXIT_FAILURE);
        }
        check(st, ctx, "gsort_sample");
        if (debug) {
            int32_t *spl = calloc((size_t)size, sizeof(int32_t));
            uint64_t *cnt = calloc((size_t)size, sizeof(uint64_t));
            check(gsort_sample_info(ctx, spl, cnt), ctx, "gsort_sample_info");
            if (rank == 0)
                for (int i = 0; i < size - 1; i++)
                    printf("[MASTER] Splitter: %u.\n", (unsigned)spl[i]);
            for (int j = 0; j < size; j++)
                printf("[COMMON] %d: Bucket %d=%llu\n", rank, j, (unsigned long long)cnt[j]);
            free(spl);
            free(cnt);
        }
    }
    check(gsort_gather_to_root(ctx, d_out, n_out, int_buf), ctx, "gsort_gather_to_root");
    if (rank == 0) {
        const double end = MPI_Wtime();
        if ((algo == CLI_RADIX && debug > 2) || (algo == CLI_SAMPLE && debug))
            print_dump(int_buf, n_total);
        /* index N/2-1 (radix:201); N = 1 would read int_buf[-1] in the reference (Q14) */
        const long long med = n_total >= 2 ? (long long)(n_total / 2) - 1 : 0;
        printf("The n/2-th sorted element: %d\n", int_buf[med]);
        fflush(stdout);
        free(int_buf);
        fprintf(stderr, "Endtime()-Starttime() = %.5f sec\n", end - start);
    }
    gsort_destroy(ctx);
    MPI_Finalize();
    return EXIT_SUCCESS;
}
