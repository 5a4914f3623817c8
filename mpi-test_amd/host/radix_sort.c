/* radix_sort -- drop-in for the reference's radix_sort (mpi_radix_sort/Makefile:2,
 * mpi_radix_sort.c:207-228).  Sorting runs on the GPUs through libgsort (gsort_radix). */
#include "gsort_cli.h"

int main(int argc, char *argv[]) { return gsort_cli_main(argc, argv, CLI_RADIX); }
