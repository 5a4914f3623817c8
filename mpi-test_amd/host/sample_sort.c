/* sample_sort -- drop-in for the reference's sample_sort (mpi_sample_sort/Makefile:2,
 * mpi_sample_sort.c:220-241).  Sorting runs on the GPUs through libgsort (gsort_sample). */
#include "gsort_cli.h"

int main(int argc, char *argv[]) { return gsort_cli_main(argc, argv, CLI_SAMPLE); }
