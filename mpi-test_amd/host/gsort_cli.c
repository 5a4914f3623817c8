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
 *   (every stdout line above comes from gsort_write_report, which the tests call too)
 *   stderr                 -> "Endtime()-Starttime() = %.5f sec\n" (radix:203)
 * The timer spans what the reference's spans -- from after the rank-0 read to after the final
 * gather (radix:98,197; sample:61,201) -- and, like the reference's, excludes process setup
 * (MPI_Init there; MPI_Init + GPU context + RCCL communicator here).
 * MPI carries only the bootstrap: N and the group id (RCCL unique id, or the IPC process
 * group's when there are more ranks than GPUs).  Keys move H2D on rank 0, GPU to GPU between
 * ranks (RCCL over xGMI, or HIP IPC copies), and D2H on rank 0 -- never over MPI.
 */
#include <mpi.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/stat.h>
#include <unistd.h>

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

    /* bootstrap: one context per rank; the group's id broadcast over MPI.  One GPU per rank:
     * RCCL over xGMI.  More ranks than GPUs (RCCL refuses two ranks on one device): the same-node
     * IPC process group.  GSORT_TRANSPORT=rccl|ipc overrides the choice. */
    gsort_uid uid;
    memset(&uid, 0, sizeof uid);
    if (size > 1) {
        /* the IPC group (POSIX shm + HIP IPC handles) only spans one node: decide from the
         * node-local rank counts, not from rank 0's GPUs against the world size -- 2 nodes x 8
         * GPUs at -np 16 is RCCL */
        MPI_Comm node;
        int node_size = 1, max_node = 1;
        MPI_Comm_split_type(MPI_COMM_WORLD, MPI_COMM_TYPE_SHARED, rank, MPI_INFO_NULL, &node);
        MPI_Comm_size(node, &node_size);
        MPI_Comm_free(&node);
        MPI_Allreduce(&node_size, &max_node, 1, MPI_INT, MPI_MAX, MPI_COMM_WORLD);
        const int one_node = max_node == size;
        if (rank == 0) {
            const char *tr = getenv("GSORT_TRANSPORT");
            const int ipc = tr && *tr ? strcmp(tr, "ipc") == 0
                                      : one_node && gsort_visible_devices() < size;
            if (ipc && !one_node)
                die("GSORT_TRANSPORT=ipc: the IPC process group needs every rank on one node");
            if (ipc) check(gsort_get_uid_ipc(size, &uid), NULL, "gsort_get_uid_ipc");
            else check(gsort_get_uid(&uid), NULL, "gsort_get_uid");
        }
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
    /* stdout: the reference's contract lines (gsort_write_report), "Each bucket" before the sort
     * as there (mpi_sample_sort.c:74), the rest after the final gather */
    gsort_report rep;
    memset(&rep, 0, sizeof rep);
    rep.algo = algo == CLI_RADIX ? GSORT_REPORT_RADIX : GSORT_REPORT_SAMPLE;
    rep.rank = rank;
    rep.nranks = size;
    rep.debug = debug;
    rep.n_total = n_total;
    rep.stage = 1;
    fflush(stdout);
    check(gsort_write_report(&rep, STDOUT_FILENO), ctx, "gsort_write_report");

    int32_t *d_keys = NULL, *d_out = NULL;
    size_t n_local = 0, n_out = 0;
    int32_t *spl = calloc((size_t)size, sizeof(int32_t));
    uint64_t *cnt = calloc((size_t)size, sizeof(uint64_t));
    if (!spl || !cnt) die("out of host memory");
    check(gsort_scatter_from_root(ctx, int_buf, n_total, &d_keys, &n_local), ctx,
          "gsort_scatter_from_root");
    if (algo == CLI_RADIX) {
        check(gsort_radix(ctx, d_keys, n_local, &d_out, &n_out, NULL), ctx, "gsort_radix");
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
        check(gsort_sample_info(ctx, spl, cnt), ctx, "gsort_sample_info");
    }
    check(gsort_gather_to_root(ctx, d_out, n_out, int_buf), ctx, "gsort_gather_to_root");
    const double end = MPI_Wtime();
    rep.splitters = spl;
    rep.bucket_counts = cnt;
    rep.sorted = int_buf;
    rep.stage = 2;
    check(gsort_write_report(&rep, STDOUT_FILENO), ctx, "gsort_write_report");
    if (rank == 0) fprintf(stderr, "Endtime()-Starttime() = %.5f sec\n", end - start);
    free(spl);
    free(cnt);
    free(int_buf);
    gsort_destroy(ctx);
    MPI_Finalize();
    return EXIT_SUCCESS;
}
