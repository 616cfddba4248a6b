/* ./bin/sigma_c — see driver.c; replaces the reference's sigma_c.c main(). */
#include "driver.h"

int main(int argc, char **argv) { return spmv_driver_main(argc, argv, FMT_SELL); }
