/* ./bin/coo — see driver.c; replaces the reference's coo.c main(). */
#include "driver.h"

int main(int argc, char **argv) { return spmv_driver_main(argc, argv, FMT_COO); }
