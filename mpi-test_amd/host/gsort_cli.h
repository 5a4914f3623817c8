/* gsort_cli.h -- shared driver of the drop-in radix_sort / sample_sort programs. */
#ifndef GSORT_CLI_H
#define GSORT_CLI_H

enum { CLI_RADIX = 0, CLI_SAMPLE = 1 };

/* Runs the whole program: mirrors main() + sort() of the reference
 * (mpi_radix_sort.c:60-228, mpi_sample_sort.c:28-241).  Returns the exit status. */
int gsort_cli_main(int argc, char **argv, int algo);

/* %d-compatible parser of a whole text buffer (mpi_radix_sort.c:85-97 reads with
 * fscanf("%d") in a !feof loop).  Returns the number of keys, or -1 on a non-numeric token
 * (the reference spins on such a token until realloc fails, then reports the file as
 * invalid).  No phantom element for a trailing delimiter. */
long gsort_cli_parse(const char *buf, long len, int *out, long cap);

#endif
