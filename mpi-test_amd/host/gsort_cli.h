/* gsort_cli.h -- shared driver of the drop-in radix_sort / sample_sort programs. */
#ifndef GSORT_CLI_H
#define GSORT_CLI_H

enum { CLI_RADIX = 0, CLI_SAMPLE = 1 };

/* Runs the whole program: mirrors main() + sort() of the reference
 * (mpi_radix_sort.c:60-228, mpi_sample_sort.c:28-241).  Returns the exit status. */
int gsort_cli_main(int argc, char **argv, int algo);

#endif
