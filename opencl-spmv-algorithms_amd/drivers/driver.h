/*
 * driver.h — shared main() of the five per-format programs
 * ./bin/{coo,csr,ell,sigma_c,cmrs}, the drop-in replacements of the
 * reference's coo.c / csr.c / ell.c / sigma_c.c / cmrs.c drivers.
 */
#ifndef SPMV_DRIVER_H
#define SPMV_DRIVER_H

typedef enum { FMT_COO, FMT_CSR, FMT_ELL, FMT_SELL, FMT_CMRS } spmv_format;

int spmv_driver_main(int argc, char **argv, spmv_format fmt);

#endif
